#!/bin/bash
# Kernel-trace profile of one bench configuration.
# Usage: bash scripts/gpu_prof.sh TAG [bench args...]
set -o pipefail
TAG=${1:-prof}; shift
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run --output-format csv -- python bench.py "$@" --no-cpu > gpurun_out/${TAG}_prof.log 2>&1
rc=$?
echo "PROF EXIT $rc"
grep '^{' gpurun_out/${TAG}_prof.log | head -1 | cut -c1-400
cut -d, -f1-5 gpurun_out/${TAG}_prof/run_kernel_stats.csv 2>/dev/null | head -8
exit $rc
