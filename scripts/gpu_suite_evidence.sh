#!/bin/bash
# Full GPU suite, then the evidence lease (scripts/gpu_evidence.sh). Usage: TAG
set -o pipefail
TAG=${1:-fin}
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v -rf -p no:cacheprovider --timeout 300 \
  --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?
echo "TESTS $rc"; grep -E "FAILED|ERROR" gpurun_out/${TAG}_tests.log | head -20; tail -1 gpurun_out/${TAG}_tests.log
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_evidence.sh $TAG
