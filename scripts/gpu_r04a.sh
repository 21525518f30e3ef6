#!/bin/bash
# Round 4: cooperative persistent solver + CROWDED tests, then sub375 A/B:
# phase kernels (coop) vs persistent coop vs per-wave transforms at 3 WG/CU.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -rf -p no:cacheprovider --timeout 240 \
  --timeout-method thread -k "persist or crowded" > gpurun_out/r04a_tests.log 2>&1
rc=$?
echo "TESTS $rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r04a_tests.log | tail -8
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for v in p0 p1 w3; do
    case $v in
      p0) ENVV=""; A="--persistent 0";;
      p1) ENVV=""; A="--persistent 1";;
      w3) ENVV="BSGP_PERWAVE_MIN_WG=3"; A="--persistent 1";;
    esac
    env $ENVV timeout -k 10 300 python bench.py --config sub375 --no-cpu --no-e2e --no-profile \
      --steps 3 --warmup 1 $A > gpurun_out/r04a_sub375_${v}_$i.json 2> gpurun_out/r04a_sub375_${v}_$i.err \
      || { echo "bench $v failed"; tail -5 gpurun_out/r04a_sub375_${v}_$i.err; exit 3; }
    python -c "import json;d=json.load(open('gpurun_out/r04a_sub375_${v}_$i.json'));print('$v', round(d['value']), d['config'].get('team'), d['config'].get('persistent'))"
  done
done
