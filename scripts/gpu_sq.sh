#!/bin/bash
# SQ counter passes (kernel-trace only) on a short streams=1 bench run.
# Usage: bash scripts/gpu_sq.sh TAG [bench args]
set -o pipefail
TAG=${1:-sq}; shift
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
P2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT"
i=0
for C in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $C -d gpurun_out/${TAG}_p$i -o run --output-format csv \
    -- python bench.py --no-cpu --streams 1 --steps 1 --warmup 0 --maxit 20 "$@" > gpurun_out/${TAG}_p$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 gpurun_out/${TAG}_p$i.log; exit 3; }
  F=$(find gpurun_out/${TAG}_p$i -name "*counter_collection.csv" | head -1)
  python tools/pmc_summary.py $F | grep -E "k_dir|k_col|k_ls|k_bb|k_persist"
done
