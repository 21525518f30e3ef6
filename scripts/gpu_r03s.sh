#!/bin/bash
# Parallel float32 pairwise leaves: stamp tests (bitwise bars), stamps A/B;
# sub375 with the column kernel on the plan's groups.
set -o pipefail
TAG=${1:-r03s}
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_stamps.py tests/test_gpu_app.py tests/test_gpu_persist.py -m gpu -v -s -rf -p no:cacheprovider --timeout 240 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "TESTS EXIT $rc"; grep -E "FAILED|^E  |passed|failed|parted" gpurun_out/${TAG}_tests.log | cut -c1-300 | tail -12
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash scripts/gpu_ab.sh ${TAG}_stamps 2 old base -- --config stamps31 --steps 2 --no-e2e || exit $?
bash scripts/gpu_ab.sh ${TAG}_sub375 2 base cg0 -- --config sub375 --maxit 50 --steps 2 --no-e2e
