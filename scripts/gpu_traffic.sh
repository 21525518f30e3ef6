#!/bin/bash
# Two separate PMC passes (FETCH_SIZE, WRITE_SIZE), kernel-trace only, on one
# one-stream solve of the bench workload (a launch = the whole batch, as in
# bench.py's profiled solve); writes gpurun_out/traffic_<TAG>.json with HBM
# bytes per launch per kernel.  Usage: TAG [bench args]
set -o pipefail
TAG=$1; shift
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $C -d gpurun_out/pmc_${TAG}_$C -o run --output-format csv \
    -- python bench.py --no-cpu --no-profile --streams 1 --steps 1 --warmup 0 "$@" > gpurun_out/pmc_${TAG}_$C.log 2>&1 || { echo "pmc $C failed"; tail -5 gpurun_out/pmc_${TAG}_$C.log; exit 3; }
done
F=$(find gpurun_out/pmc_${TAG}_FETCH_SIZE -name "*counter_collection.csv" | head -1)
W=$(find gpurun_out/pmc_${TAG}_WRITE_SIZE -name "*counter_collection.csv" | head -1)
python tools/traffic_from_pmc.py $F $W gpurun_out/traffic_${TAG}.json "bench.py --streams 1 $*"
