#!/bin/bash
# Direct-DFT stage on lane pairs: GPU suite, stamps A/B.
set -o pipefail
TAG=${1:-r03ee}
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s -rf -p no:cacheprovider --timeout 240 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "TESTS EXIT $rc"; grep -E "FAILED|ERROR|^E  |parted late|worst" gpurun_out/${TAG}_tests.log | cut -c1-250 | head -20; tail -2 gpurun_out/${TAG}_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash scripts/gpu_ab.sh ${TAG}_stamps 2 prev base -- --config stamps31 --steps 2 --no-e2e
