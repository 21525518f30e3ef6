#!/bin/bash
# C3: column-pass loads inside the persistent kernel: the transfer-function column with the column (tfpre), the wave's next column ahead of the inverse transform (npf).
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
bash scripts/gpu_ab.sh r04ze_c3 3 base tfpre npf -- --no-e2e --no-profile || exit 3
