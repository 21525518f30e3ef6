#!/bin/bash
# Stream-count sweep + a streams=1 kernel trace (per-kernel times without overlap).
# Usage: bash scripts/gpu_streams.sh TAG
set -o pipefail
TAG=${1:-st}
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
for S in 1 2 3 4; do
  timeout -k 10 300 python bench.py --no-cpu --streams $S --steps 2 > gpurun_out/${TAG}_s$S.json 2> gpurun_out/${TAG}_s$S.err || { echo "bench s$S failed"; tail -3 gpurun_out/${TAG}_s$S.err; exit 3; }
  python -c "import json;d=json.load(open('gpurun_out/${TAG}_s$S.json'));print('streams $S', round(d['value']), 'ms', round(d['ms_per_step'],1))"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof1 -o run --output-format csv -- python bench.py --no-cpu --streams 1 --steps 2 > gpurun_out/${TAG}_prof1.log 2>&1 || { echo "prof failed"; exit 3; }
cut -d, -f1-4 gpurun_out/${TAG}_prof1/run_kernel_stats.csv | head -7
