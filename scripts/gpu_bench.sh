#!/bin/bash
# Tests (optional -k expr), then bench.py with the given args, then a rocprofv3
# kernel-trace summary of the same bench command (no CPU baseline, no PMC).
# Usage: bash scripts/gpu_bench.sh TAG "pytest -k expr or empty" [bench args...]
set -o pipefail
TAG=${1:-run}; K=${2:-}; shift; shift
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -v -rf -p no:cacheprovider --timeout 240 --timeout-method thread -k "$K" > gpurun_out/${TAG}_tests.log 2>&1
  rc=$?
  echo "TESTS EXIT $rc"; grep -E "FAILED|ERROR" gpurun_out/${TAG}_tests.log | head -20; tail -2 gpurun_out/${TAG}_tests.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping: tests ended abnormally"; exit $rc; fi
fi
timeout -k 10 600 python -u bench.py "$@" > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
rc=$?
echo "BENCH EXIT $rc"; cat gpurun_out/${TAG}_bench.json; tail -3 gpurun_out/${TAG}_bench.err
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run --output-format csv -- python bench.py "$@" --no-cpu > gpurun_out/${TAG}_prof.log 2>&1
echo "PROF EXIT $?"
find gpurun_out/${TAG}_prof -name "*kernel_stats.csv" | head -1 | xargs -r cut -d, -f1-8 | head -14
