#!/bin/bash
# Team phase kernels (C2) with the register budget of one wave per SIMD: whole-row operand
# batches (t1) or two single-column batches in flight (t2), both with the first batch before
# the transform, against HEAD.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
bash scripts/gpu_ab.sh r04w_c2 3 base t1 t2 -- --config c2 --no-e2e || exit 3
