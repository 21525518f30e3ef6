#!/bin/bash
# PMC counter passes (kernel-trace only, no sys/runtime trace) for the bench
# workload.  Usage: bash scripts/gpu_pmc.sh TAG "COUNTERS..." [bench args]
set -o pipefail
TAG=$1; shift; CTRS=$1; shift
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --pmc $CTRS -d gpurun_out/${TAG} -o run --output-format csv \
  -- python bench.py --no-cpu "$@" > gpurun_out/${TAG}.log 2>&1
rc=$?; echo "PMC EXIT $rc"; tail -3 gpurun_out/${TAG}.log
ls gpurun_out/${TAG}
