#!/bin/bash
# SQ counters: star stamps on the phase kernels, C3 on the persistent solver.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
bash scripts/gpu_sq.sh r03v_stamps --config stamps31 --batch 4096 --persistent 0 || exit $?
bash scripts/gpu_sq.sh r03v_c3
