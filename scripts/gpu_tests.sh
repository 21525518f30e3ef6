#!/bin/bash
# GPU parity tests only (verbose, per-test time limit). Usage: bash scripts/gpu_tests.sh TAG [pytest -k expr]
set -o pipefail
TAG=${1:-tests}; K=${2:-}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -n "$K" ]; then KARG=(-k "$K"); else KARG=(); fi
timeout -k 10 900 python -u -m pytest tests -m gpu -v -rf -p no:cacheprovider --timeout 240 --timeout-method thread "${KARG[@]}" > gpurun_out/${TAG}.log 2>&1
rc=$?
echo "TESTS EXIT $rc"; grep -E "PASSED|FAILED|ERROR" gpurun_out/${TAG}.log | grep -v PASSED | head -40; tail -3 gpurun_out/${TAG}.log
exit $rc
