#!/bin/bash
# Team size A/B on C2 (single 256^2 image) and C4.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
bash scripts/gpu_ab.sh r03cc_c2 2 base,--team,16 base,--team,24 base,--team,32 base,--team,48 base,--team,64 -- --config c2 --steps 10 --no-e2e || exit $?
bash scripts/gpu_ab.sh r03cc_c4 2 base,--team,192 base,--team,256 -- --config c4 --storage f32 --steps 10 --no-e2e
