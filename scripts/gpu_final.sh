#!/bin/bash
# Round-end evidence at HEAD: smoke(), the default bench line, and the
# rocprofv3 kernel statistics of the same command.  Usage: bash scripts/gpu_final.sh TAG
set -o pipefail
TAG=${1:-final}
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { echo "smoke failed"; tail -5 gpurun_out/${TAG}_smoke.log; exit 3; }
tail -1 gpurun_out/${TAG}_smoke.log
timeout -k 10 400 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { echo "bench failed"; tail -5 gpurun_out/${TAG}_bench.err; exit 3; }
cat gpurun_out/${TAG}_bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run --output-format csv -- python bench.py --no-cpu > gpurun_out/${TAG}_prof.log 2>&1 || { echo "prof failed"; exit 3; }
find gpurun_out/${TAG}_prof -name "*kernel_stats.csv" | head -1 | xargs -r cut -d, -f1-4 | grep -E "Name|bsgp::k_"
