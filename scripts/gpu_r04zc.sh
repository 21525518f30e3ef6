#!/bin/bash
# Application build with composite radix stages in the line-search and BB row passes (c1).
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
bash scripts/gpu_ab.sh r04zc_sub375 2 base c1 -- --config sub375 --no-e2e --no-profile || exit 3
bash scripts/gpu_ab.sh r04zc_sub450 2 base c1 -- --config sub450 --no-e2e --no-profile || exit 3
