#!/bin/bash
# parity tests, then one bench line per argument string.
# Usage: bash scripts/gpu_multi.sh TAG "bench args A" "bench args B" ...
set -o pipefail
TAG=${1:-multi}; shift
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -q -rf -p no:cacheprovider > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "TESTS EXIT $rc"; tail -15 gpurun_out/${TAG}_tests.log
[ $rc -eq 0 ] || exit $rc
i=0
for A in "$@"; do
  i=$((i+1))
  timeout -k 10 300 python bench.py --no-cpu $A > gpurun_out/${TAG}_$i.json 2>gpurun_out/${TAG}_$i.err || { echo "bench $A failed"; tail -5 gpurun_out/${TAG}_$i.err; exit 3; }
  python -c "
import json;d=json.load(open('gpurun_out/${TAG}_$i.json'));r=d['roofline']
print('$A', '|', round(d['value']), 'img-it/s frac', round(r['frac'],3), 'E_ls', round(r['E_ls_per_iter'],2), 'passes', round(r.get('ls_passes_per_iter',0),2), 'series', round(r.get('ls_series_per_iter',0),2), 'E_p', round(r['E_p_per_iter'],2))"
done
