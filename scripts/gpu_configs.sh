#!/bin/bash
# Bench lines of the other BASELINE configs at HEAD (one GPU): C5 on one rank
# (all 8192 subdivisions on one device), C4 2048^2 in float32 and float64
# storage, C2 single 256^2 image.  Usage: bash scripts/gpu_configs.sh TAG
set -o pipefail
TAG=${1:-cfg}
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
run() { local name=$1; shift
  timeout -k 10 300 python -u bench.py "$@" > gpurun_out/${TAG}_$name.json 2> gpurun_out/${TAG}_$name.err || { echo "$name failed"; tail -5 gpurun_out/${TAG}_$name.err; exit 3; }
  python -c "import json;d=json.load(open('gpurun_out/${TAG}_$name.json'));print('$name', round(d['value']), d['unit'], 'ms/step', round(d['ms_per_step'],1), 'solve frac', round(d['roofline']['solve']['frac_timed'],3) if d.get('roofline') else None)"
}
run c5 --config c5 --steps 2 --warmup 1 --no-cpu
run c4f32 --config c4 --storage f32 --steps 3 --warmup 1
run c4f64 --config c4 --storage f64 --steps 3 --warmup 1 --no-cpu
run c2 --config c2 --steps 5 --warmup 1
