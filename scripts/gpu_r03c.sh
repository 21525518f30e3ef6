#!/bin/bash
# Round 3: stamp + long parity (revised bars), single-image configs with the
# XCD-hierarchical team barrier, the star-stamp bench. Usage: TAG
set -o pipefail
TAG=${1:-r03c}
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
PYT="python -u -m pytest -m gpu -v -s -rf -p no:cacheprovider --timeout 240 --timeout-method thread"
timeout -k 10 400 $PYT tests/test_gpu_long.py tests/test_gpu_stamps.py tests/test_gpu_parity.py -k "long or stop3 or team or stamps or profiled" > gpurun_out/${TAG}_long.log 2>&1
rc=$?; echo "LONG EXIT $rc"; grep -E "PASSED|FAILED|^E  |parted" gpurun_out/${TAG}_long.log | cut -c1-400 | head -40
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for c in c2 c4; do
  for st in f64 f32; do
    [ $c == c2 ] && [ $st == f32 ] && continue
    timeout -k 10 300 python bench.py --config $c --storage $st --no-cpu --no-e2e --steps 5 --warmup 1 > gpurun_out/${TAG}_${c}_${st}.json 2> gpurun_out/${TAG}_${c}_${st}.err || { echo "bench $c failed"; tail -3 gpurun_out/${TAG}_${c}_${st}.err; exit 3; }
    python -c "import json;d=json.load(open('gpurun_out/${TAG}_${c}_${st}.json'));print('$c $st', round(d['value']), round(d['ms_per_step'],1))"
  done
done
timeout -k 10 400 python bench.py --config stamps31 --no-cpu --no-e2e --steps 3 --warmup 1 > gpurun_out/${TAG}_stamps.json 2> gpurun_out/${TAG}_stamps.err || { echo "stamps bench failed"; tail -5 gpurun_out/${TAG}_stamps.err; exit 3; }
python -c "import json;d=json.load(open('gpurun_out/${TAG}_stamps.json'));print('stamps', round(d['value']), round(d['ms_per_step'],1), d['vs_baseline'], d['roofline']['kernel'], round(d['roofline']['frac'],3))"
timeout -k 10 400 python bench.py --no-cpu --steps 5 --warmup 1 > gpurun_out/${TAG}_c3.json 2> gpurun_out/${TAG}_c3.err || { echo "c3 bench failed"; tail -5 gpurun_out/${TAG}_c3.err; exit 3; }
python -c "import json;d=json.load(open('gpurun_out/${TAG}_c3.json'));r=d['roofline'];print('c3', round(d['value']), r['kernel'], round(r['frac'],3), round(r['solve']['frac_timed'],3), d['end_to_end']['value'])"
