#!/bin/bash
# Round 3 re-entry check at HEAD: GPU suite, default bench, stamps31 bench.
set -o pipefail
TAG=${1:-r03j}
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v -rf -p no:cacheprovider --timeout 240 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "TESTS EXIT $rc"; grep -E "FAILED|ERROR" gpurun_out/${TAG}_tests.log | head -20; tail -2 gpurun_out/${TAG}_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { echo "bench failed"; tail -5 gpurun_out/${TAG}_bench.err; exit 3; }
python -c "import json;d=json.load(open('gpurun_out/${TAG}_bench.json'));print('c3', round(d['value']), d['roofline']['frac'])"
timeout -k 10 600 python bench.py --config stamps31 --steps 3 --warmup 1 --no-cpu > gpurun_out/${TAG}_stamps.json 2> gpurun_out/${TAG}_stamps.err || { echo "stamps bench failed"; tail -5 gpurun_out/${TAG}_stamps.err; exit 3; }
python -c "import json;d=json.load(open('gpurun_out/${TAG}_stamps.json'));print('stamps', round(d['value']), d['vs_baseline'])"
