#!/bin/bash
# Round 3: persistent solver first (isolated), then the long-run parity test with
# its failure text, the rest of the GPU suite, and the persistent A/B on C3. Usage: TAG
set -o pipefail
TAG=${1:-r03b}
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
PYT="python -u -m pytest -m gpu -v -s -rf -p no:cacheprovider --timeout 240 --timeout-method thread"
timeout -k 10 300 $PYT -x tests/test_gpu_persist.py > gpurun_out/${TAG}_persist.log 2>&1
rc=$?; echo "PERSIST EXIT $rc"; grep -E "PASSED|FAILED|Error|error" gpurun_out/${TAG}_persist.log | head -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 $PYT tests/test_gpu_long.py tests/test_gpu_stamps.py > gpurun_out/${TAG}_long.log 2>&1
rc=$?; echo "LONG EXIT $rc"; grep -E "PASSED|FAILED|^E  |parted" gpurun_out/${TAG}_long.log | cut -c1-300 | head -40
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 900 $PYT tests --deselect tests/test_gpu_persist.py --deselect tests/test_gpu_long.py --deselect tests/test_gpu_stamps.py > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "SUITE EXIT $rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/${TAG}_tests.log | head -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for i in 0 1; do
  for p in 0 1; do
    timeout -k 10 300 python bench.py --no-cpu --no-profile --steps 3 --persistent $p > gpurun_out/${TAG}_p${p}_$i.json 2> gpurun_out/${TAG}_p${p}_$i.err || { echo "bench p$p failed"; tail -3 gpurun_out/${TAG}_p${p}_$i.err; exit 3; }
    python -c "import json;d=json.load(open('gpurun_out/${TAG}_p${p}_$i.json'));print('persistent $p', round(d['value']), round(d['ms_per_step'],1))"
  done
done
