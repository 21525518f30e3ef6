#!/bin/bash
# C3's persistent kernel with two operand batches in flight (p1) or the first batch ahead of
# the transform (p2), against HEAD.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
bash scripts/gpu_ab.sh r04y_c3 3 base p1 p2 -- --no-e2e --no-profile || exit 3
