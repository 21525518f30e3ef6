#!/bin/bash
# Persistent kernel at two waves per SIMD (two workgroups per CU), with and without
# four-column operand batches, against HEAD's three waves: C3 and 375^2 tiles.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
bash scripts/gpu_ab.sh r04t_c3 3 base w2 w2j4 -- --no-e2e --no-profile || exit 3
bash scripts/gpu_ab.sh r04t_sub375 2 base w2 w2j4 -- --config sub375 --no-e2e --no-profile || exit 3
