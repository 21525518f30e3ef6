#!/bin/bash
# Evidence for the bench line at HEAD (one call): bench (default config),
# rocprofv3 kernel stats of the default command and of --streams 1 (whose
# per-kernel averages are the launch unit of bench.py's profiled roofline),
# the PMC traffic passes and the SQ counter passes.  Usage: TAG [bench args]
set -o pipefail
TAG=${1:-meas}; shift
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py --steps 5 --warmup 1 "$@" > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { echo "bench failed"; tail -5 gpurun_out/${TAG}_bench.err; exit 3; }
cat gpurun_out/${TAG}_bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof3 -o run --output-format csv -- python bench.py --no-cpu --steps 5 --warmup 1 "$@" > gpurun_out/${TAG}_prof3.log 2>&1 || { echo "prof3 failed"; exit 3; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof1 -o run --output-format csv -- python bench.py --no-cpu --streams 1 --steps 2 --warmup 1 "$@" > gpurun_out/${TAG}_prof1.log 2>&1 || { echo "prof1 failed"; exit 3; }
for d in prof3 prof1; do echo "== $d"; find gpurun_out/${TAG}_$d -name "*kernel_stats.csv" | head -1 | xargs -r cut -d, -f1-4 | grep -E "Name|bsgp::k_" ; done
bash scripts/gpu_traffic.sh ${TAG} "$@" || exit 3
bash scripts/gpu_sq.sh ${TAG}_sq "$@" || exit 3
