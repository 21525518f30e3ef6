#!/bin/bash
# Parity tests + bench at streams 1/2 + streams=1 kernel trace.  Usage: TAG [bench args]
set -o pipefail
TAG=${1:-q}; shift
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "TESTS EXIT $rc"; tail -3 gpurun_out/${TAG}_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for S in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu --streams $S --steps 2 "$@" > gpurun_out/${TAG}_s$S.json 2> gpurun_out/${TAG}_s$S.err || { echo "bench s$S failed"; tail -3 gpurun_out/${TAG}_s$S.err; exit 3; }
  python -c "import json;d=json.load(open('gpurun_out/${TAG}_s$S.json'));print('streams $S', round(d['value']), 'ms', round(d['ms_per_step'],1), 'frac', round(d['roofline']['frac'],3))"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof1 -o run --output-format csv -- python bench.py --no-cpu --streams 1 --steps 2 "$@" > gpurun_out/${TAG}_prof1.log 2>&1 || { echo "prof failed"; exit 3; }
python - <<PY
import csv
for r in csv.DictReader(open('gpurun_out/${TAG}_prof1/run_kernel_stats.csv')):
    if 'bsgp::k_' in r['Name']: print(r['Name'][:40], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us', r['Percentage'])
PY
