#!/bin/bash
# Regression hunt: HEAD (compact 400 roots) vs the r04g commit's library (old), one box.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
bash scripts/gpu_ab.sh r04j_c3 2 base old -- --no-e2e --no-profile || exit 3
bash scripts/gpu_ab.sh r04j_sub375 2 base old -- --config sub375 --no-e2e --no-profile || exit 3
bash scripts/gpu_ab.sh r04j_c2 2 base old -- --config c2 --no-e2e --no-profile || exit 3
BSGP_TW400C=0 timeout -k 10 300 python bench.py --config sub375 --no-cpu --no-e2e --no-profile --steps 3 > gpurun_out/r04j_sub375_c0.json 2>/dev/null && python -c "import json;print('sub375 base TW400C=0', round(json.load(open('gpurun_out/r04j_sub375_c0.json'))['value']))"
