#!/bin/bash
# Two separate PMC passes (FETCH_SIZE, WRITE_SIZE), kernel-trace only, on the
# bench workload; writes gpurun_out/traffic_<TAG>.json.  Usage: TAG STEPS [bench args]
set -o pipefail
TAG=$1; STEPS=$2; shift 2
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 600 rocprofv3 --kernel-trace --pmc $C -d gpurun_out/pmc_${TAG}_$C -o run --output-format csv \
    -- python bench.py --no-cpu --steps $STEPS --warmup 0 "$@" > gpurun_out/pmc_${TAG}_$C.log 2>&1 || { echo "pmc $C failed"; tail -5 gpurun_out/pmc_${TAG}_$C.log; exit 3; }
done
F=$(find gpurun_out/pmc_${TAG}_FETCH_SIZE -name "*counter_collection.csv" | head -1)
W=$(find gpurun_out/pmc_${TAG}_WRITE_SIZE -name "*counter_collection.csv" | head -1)
python tools/traffic_from_pmc.py $F $W gpurun_out/traffic_${TAG}.json $STEPS
