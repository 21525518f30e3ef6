#!/bin/bash
# One-wave workgroups for tiny images: GPU suite, smoke, stamps A/B.
set -o pipefail
TAG=${1:-r03u}
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v -rf -p no:cacheprovider --timeout 240 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "TESTS EXIT $rc"; grep -E "FAILED|ERROR" gpurun_out/${TAG}_tests.log | head -20; tail -2 gpurun_out/${TAG}_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -2
bash scripts/gpu_ab.sh ${TAG}_stamps 2 nowave1 base -- --config stamps31 --steps 2 --no-e2e
