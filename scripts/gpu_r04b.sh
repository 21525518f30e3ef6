#!/bin/bash
# Round 4: full GPU suite, C3 A/B of the series tail bound, sub375 at 1024 tiles.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 1200 python -u -m pytest tests -m gpu -v -rf -p no:cacheprovider --timeout 300 \
  --timeout-method thread > gpurun_out/r04b_tests.log 2>&1
rc=$?
echo "TESTS $rc"; grep -E "FAILED|ERROR" gpurun_out/r04b_tests.log | head -20; tail -2 gpurun_out/r04b_tests.log
case $rc in 124|134|137|139) exit $rc;; esac
bash scripts/gpu_ab.sh r04b_c3 3 base sb0 -- --no-e2e --no-profile || exit 3
for v in p1 w3; do
  case $v in
    p1) ENVV="";;
    w3) ENVV="BSGP_PERWAVE_MIN_WG=3";;
  esac
  env $ENVV timeout -k 10 300 python bench.py --config sub375 --batch 1024 --no-cpu --no-e2e \
    --no-profile --steps 3 --warmup 1 > gpurun_out/r04b_sub375_$v.json 2> gpurun_out/r04b_sub375_$v.err \
    || { echo "bench $v failed"; tail -5 gpurun_out/r04b_sub375_$v.err; exit 3; }
  python -c "import json;d=json.load(open('gpurun_out/r04b_sub375_$v.json'));print('sub375 B=1024 $v', round(d['value']))"
done
