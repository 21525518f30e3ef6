#!/bin/bash
# C4 with the wide first-pass projection bracket (BSGP_PROJ_WIDE_PX=32 covers its 32 pixels per thread).
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
bash scripts/gpu_ab.sh r04zb_c4f32 2 base wide32 -- --config c4 --storage f32 --no-e2e || exit 3
python -c "import json;[print(f, json.load(open('gpurun_out/r04zb_c4f32_'+f+'_1.json'))['roofline']['counters_per_iter']) for f in ('0','1')]"
