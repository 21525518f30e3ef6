#!/bin/bash
# C2 team size: 16 / 24 / 32 (auto) members.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
bash scripts/gpu_ab.sh r04zd_c2 2 base,--team,16 base,--team,24 base -- --config c2 --no-e2e || exit 3
