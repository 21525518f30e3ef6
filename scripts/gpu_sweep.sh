#!/bin/bash
# parity tests, then a bench sweep over line-search speculation width
set -o pipefail
TAG=${1:-sweep}; shift
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -q -rf -p no:cacheprovider > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; echo "TESTS EXIT $rc"; tail -15 gpurun_out/${TAG}_tests.log
[ $rc -eq 0 ] || exit $rc
for K in "$@"; do
  timeout -k 10 300 python bench.py --steps 2 --warmup 1 --maxit 50 --no-cpu --ls-spec $K > gpurun_out/${TAG}_ls$K.json 2>/dev/null || exit 3
  python -c "import json;d=json.load(open('gpurun_out/${TAG}_ls$K.json'));print('ls',$K,round(d['value']),round(d['roofline']['frac'],3),d['roofline']['E_ls_per_iter'])"
done
