#!/bin/bash
# Evidence from ONE lease: smoke, PMC traffic (two passes) copied to
# profiles/traffic_c3.json, the driver's bench command (C3: --gpus 1 --steps 20
# --warmup 5) that reads it, the
# rocprofv3 kernel statistics of the same command, SQ counters of k_persist,
# and the other configuration lines.  Usage: bash scripts/gpu_evidence.sh TAG
set -o pipefail
TAG=${1:-ev}
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/$TAG; export TMPDIR=/tmp
O=gpurun_out/$TAG
# a line under gpurun_out/ every 50 s: C4's CPU-baseline sample prints nothing for
# minutes, which gpurun's silence watchdog takes for a hang (lease r06f)
( while sleep 50; do date +%s >> $O/heartbeat.txt; done ) &
trap "kill $! 2>/dev/null" EXIT
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -5 $O/smoke.log; exit 3; }
tail -1 $O/smoke.log
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $C -d $O/pmc_$C -o run --output-format csv \
    -- python bench.py --no-cpu --no-profile --no-e2e --steps 1 --warmup 0 > $O/pmc_$C.log 2>&1 || { echo "pmc $C failed"; tail -5 $O/pmc_$C.log; exit 3; }
done
F=$(find $O/pmc_FETCH_SIZE -name "*counter_collection.csv" | head -1)
W=$(find $O/pmc_WRITE_SIZE -name "*counter_collection.csv" | head -1)
python tools/traffic_from_pmc.py $F $W profiles/traffic_c3.json "bench.py (C3), lease $TAG" || exit 3
cp profiles/traffic_c3.json $O/traffic_c3.json
timeout -k 10 500 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_c3.json 2> $O/bench_c3.err || { echo "bench failed"; tail -5 $O/bench_c3.err; exit 3; }
python -c "import json;d=json.load(open('$O/bench_c3.json'));r=d['roofline'];print('C3', round(d['value']), 'ms', round(d['ms_per_step'],1), 'frac', round(r['frac'],3), 'traffic', r['traffic'], 'k_persist ms', round(r['ms_per_launch'],1), 'cpu', round(d['cpu_baseline']['value']))"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --no-e2e > $O/prof.log 2>&1 || { echo "prof failed"; exit 3; }
find $O/prof -name "*kernel_stats.csv" | head -1 | xargs -r cut -d, -f1-4 | grep -E "Name|k_persist"
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
P2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_INSTS_SALU"
i=0
for C in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $C -d $O/sq_p$i -o run --output-format csv \
    -- python bench.py --no-cpu --no-profile --no-e2e --steps 1 --warmup 0 --maxit 20 > $O/sq_p$i.log 2>&1 || { echo "sq pass $i failed"; tail -5 $O/sq_p$i.log; exit 3; }
  S=$(find $O/sq_p$i -name "*counter_collection.csv" | head -1)
  python tools/pmc_summary.py $S | grep -E "k_persist" | tee $O/sq_p$i.txt
done
for cfg in "stamps31" "stamps31_kl" "app375" "sub375" "sub450" "c5" "c2" "c4 --storage f32" "c4"; do
  name=$(echo $cfg | tr ' ' '_' | tr -d '-')
  timeout -k 10 400 python bench.py --config $cfg > $O/bench_$name.json 2> $O/bench_$name.err || { echo "bench $cfg failed"; tail -5 $O/bench_$name.err; exit 3; }
  python -c "import json;d=json.load(open('$O/bench_$name.json'));r=d['roofline'] or {};c=d.get('cpu_baseline') or {};print('$name', round(d['value']), 'frac', round(r.get('frac') or 0,3), 'solve', round((r.get('solve') or {}).get('frac_timed',0),3), 'cpu', round(c.get('value') or 0,1))"
done
