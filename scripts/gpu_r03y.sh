#!/bin/bash
# Ready ring in the persistent solver: persist/stamp/long tests, stamps and C3 A/B.
set -o pipefail
TAG=${1:-r03y}
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_persist.py tests/test_gpu_stamps.py tests/test_gpu_long.py tests/test_gpu_abi.py -m gpu -v -s -rf -p no:cacheprovider --timeout 240 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "TESTS EXIT $rc"; grep -E "FAILED|^E  |passed|failed" gpurun_out/${TAG}_tests.log | cut -c1-300 | tail -12
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash scripts/gpu_ab.sh ${TAG}_stamps 2 prev base -- --config stamps31 --steps 2 --no-e2e || exit $?
bash scripts/gpu_ab.sh ${TAG}_c3 2 prev base -- --no-e2e
