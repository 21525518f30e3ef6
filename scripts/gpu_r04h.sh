#!/bin/bash
# 375^2 tiles: 3 WG/CU with the compact 400-point root table in LDS (BSGP_TW400C=1) vs
# 2 WG/CU with the full table (0); tests of the tile paths first.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 \
  --timeout-method thread -k "persist or crowded or app or sub or parity" > gpurun_out/r04h_tests.log 2>&1
rc=$?
echo "TESTS $rc"; grep -E "FAILED|ERROR" gpurun_out/r04h_tests.log | head; tail -1 gpurun_out/r04h_tests.log
case $rc in 124|134|137|139) exit $rc;; esac
for i in 1 2; do
  for v in c1 c0; do
    case $v in c1) ENVV="BSGP_TW400C=1";; c0) ENVV="BSGP_TW400C=0";; esac
    env $ENVV timeout -k 10 300 python bench.py --config sub375 --no-cpu --no-e2e --no-profile \
      --steps 3 --warmup 1 > gpurun_out/r04h_sub375_${v}_$i.json 2> gpurun_out/r04h_sub375_${v}_$i.err \
      || { echo "bench $v failed"; tail -5 gpurun_out/r04h_sub375_${v}_$i.err; exit 3; }
    python -c "import json;d=json.load(open('gpurun_out/r04h_sub375_${v}_$i.json'));print('sub375 $v', round(d['value']))"
  done
done
