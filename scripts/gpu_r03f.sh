#!/bin/bash
# Round 3 evidence at HEAD: the whole GPU suite, smoke(), the default bench
# line, rocprofv3 kernel statistics of the same command, the HBM-traffic PMC
# passes of the bench workload, the star-stamp bench with its CPU baseline.
# Usage: TAG
set -o pipefail
TAG=${1:-r03f}
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
PYT="python -u -m pytest -m gpu -v -s -rf -p no:cacheprovider --timeout 240 --timeout-method thread"
timeout -k 10 900 $PYT tests > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "TESTS EXIT $rc"; grep -E "FAILED|^E  |passed|failed" gpurun_out/${TAG}_tests.log | cut -c1-300 | tail -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { echo "smoke failed"; tail -5 gpurun_out/${TAG}_smoke.log; exit 3; }
tail -1 gpurun_out/${TAG}_smoke.log
timeout -k 10 400 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { echo "bench failed"; tail -5 gpurun_out/${TAG}_bench.err; exit 3; }
python -c "import json;d=json.load(open('gpurun_out/${TAG}_bench.json'));r=d['roofline'];print('c3', round(d['value']), r['kernel'], round(r['frac'],3), round(r['ms_per_launch'],2), d['cpu_baseline']['value'], d['end_to_end']['value'])"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run --output-format csv -- python bench.py --no-cpu > gpurun_out/${TAG}_prof.log 2>&1 || { echo "prof failed"; exit 3; }
find gpurun_out/${TAG}_prof -name "*kernel_stats.csv" | head -1 | xargs -r cut -d, -f1-4 | grep -E "Name|bsgp::k_"
bash scripts/gpu_traffic.sh c3_${TAG} || exit 3
timeout -k 10 600 python bench.py --config stamps31 --steps 3 --warmup 1 > gpurun_out/${TAG}_stamps.json 2> gpurun_out/${TAG}_stamps.err || { echo "stamps bench failed"; tail -5 gpurun_out/${TAG}_stamps.err; exit 3; }
python -c "import json;d=json.load(open('gpurun_out/${TAG}_stamps.json'));print('stamps', round(d['value']), d['vs_baseline'], d['cpu_baseline'])"
