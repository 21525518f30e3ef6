#!/bin/bash
# DC/Nyquist column pairing in the one-group cooperative column pass: GPU suite, C4 A/B.
set -o pipefail
TAG=${1:-r03jj}
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v -rf -p no:cacheprovider --timeout 240 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "TESTS EXIT $rc"; grep -E "FAILED|ERROR|^E  " gpurun_out/${TAG}_tests.log | cut -c1-250 | head -20; tail -2 gpurun_out/${TAG}_tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash scripts/gpu_ab.sh ${TAG}_c4f32 3 prev base -- --config c4 --storage f32 --steps 10 --no-e2e || exit $?
bash scripts/gpu_ab.sh ${TAG}_c4 2 prev base -- --config c4 --steps 10 --no-e2e
