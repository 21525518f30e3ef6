#!/bin/bash
# Round 3: revised long/stamp bars + persistent-solver tuning A/B. Usage: TAG
set -o pipefail
TAG=${1:-r03d}
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
PYT="python -u -m pytest -m gpu -v -s -rf -p no:cacheprovider --timeout 240 --timeout-method thread"
timeout -k 10 400 $PYT tests/test_gpu_long.py tests/test_gpu_stamps.py tests/test_gpu_parity.py -k "long or stop3 or stamps or profiled" > gpurun_out/${TAG}_long.log 2>&1
rc=$?; echo "LONG EXIT $rc"; grep -E "PASSED|FAILED|^E  |parted" gpurun_out/${TAG}_long.log | cut -c1-300 | head -30
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash scripts/gpu_ab.sh ${TAG}_ab 2 base bb4 acc2 ls2 all2 comp -- --no-e2e --no-profile
