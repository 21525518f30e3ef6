#!/bin/bash
# Coop groups A/B: C4 f32 and the 375^2 subdivision-size batch; old build vs groups (2/4),
# groups with the column kernel at full LDS, one group.
set -o pipefail
TAG=${1:-r03p}
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
bash scripts/gpu_ab.sh ${TAG}_c4f32 3 old base g1 -- --config c4 --storage f32 --steps 10 --no-e2e || exit $?
bash scripts/gpu_ab.sh ${TAG}_sub375 2 old base g1 -- --config sub375 --maxit 50 --steps 2 --no-e2e
