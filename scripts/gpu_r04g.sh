#!/bin/bash
# 375^2 / 450^2 tiles: LDS twiddles at 2 WG/CU (BSGP_PERWAVE_TW=1) vs global twiddles at 3 WG/CU.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 \
  --timeout-method thread -k "persist or crowded or app or sub" > gpurun_out/r04g_tests.log 2>&1
rc=$?
echo "TESTS $rc"; grep -E "FAILED|ERROR" gpurun_out/r04g_tests.log | head; tail -1 gpurun_out/r04g_tests.log
case $rc in 124|134|137|139) exit $rc;; esac
for i in 1 2; do
  for v in tw1 tw0; do
    case $v in tw1) ENVV="BSGP_PERWAVE_TW=1";; tw0) ENVV="BSGP_PERWAVE_TW=0";; esac
    for cfg in sub375 sub450; do
      env $ENVV timeout -k 10 300 python bench.py --config $cfg --no-cpu --no-e2e --no-profile \
        --steps 3 --warmup 1 > gpurun_out/r04g_${cfg}_${v}_$i.json 2> gpurun_out/r04g_${cfg}_${v}_$i.err \
        || { echo "bench $cfg $v failed"; tail -5 gpurun_out/r04g_${cfg}_${v}_$i.err; exit 3; }
      python -c "import json;d=json.load(open('gpurun_out/r04g_${cfg}_${v}_$i.json'));print('$cfg $v', round(d['value']))"
    done
  done
done
