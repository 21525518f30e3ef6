#!/bin/bash
# Column passes fused into the row kernels for teams (C2): GPU suite with the
# widest variant, then A/B on C2 and C3.
set -o pipefail
TAG=${1:-r03dd}
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
BSGP_LIB=$PWD/beta-sgp_amd/libbsgp_ft6.so timeout -k 10 900 python -u -m pytest tests -m gpu -v -rf -p no:cacheprovider --timeout 240 --timeout-method thread --deselect tests/test_gpu_abi.py::test_integration_stub_runs_verbatim > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "TESTS EXIT $rc"; grep -E "FAILED|ERROR|^E  " gpurun_out/${TAG}_tests.log | cut -c1-250 | head -20; tail -2 gpurun_out/${TAG}_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash scripts/gpu_ab.sh ${TAG}_c2 3 base ft2 ft6 -- --config c2 --steps 10 --no-e2e || exit $?
bash scripts/gpu_ab.sh ${TAG}_c3 2 base ft6 -- --no-e2e
