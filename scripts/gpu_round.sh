#!/bin/bash
# One GPU round: parity tests -> bench -> rocprofv3 kernel trace (stats).
# Usage: bash scripts/gpu_round.sh TAG [bench args...]
# Stops before the next GPU step after a fault, abort, segfault or time limit.
set -o pipefail
TAG=${1:-run}; shift
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -q -rf -p no:cacheprovider > gpurun_out/${TAG}_tests.log 2>&1
rc=$?
echo "TESTS EXIT $rc"; tail -5 gpurun_out/${TAG}_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping: tests ended abnormally"; exit $rc; fi
timeout -k 10 600 python bench.py "$@" > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run --output-format csv -- python bench.py "$@" --no-cpu > gpurun_out/${TAG}_prof.log 2>&1
echo "BENCH/PROF EXIT $?"
cat gpurun_out/${TAG}_bench.json; tail -3 gpurun_out/${TAG}_bench.err
cut -d, -f1-5 gpurun_out/${TAG}_prof/run_kernel_stats.csv 2>/dev/null | head -12
