#!/bin/bash
# Full GPU suite; C2 gathered team lists A/B (g0 = off); 375^2 compact-root A/B (BSGP_TW400C).
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v -rf -p no:cacheprovider --timeout 300 \
  --timeout-method thread > gpurun_out/r04i_tests.log 2>&1
rc=$?
echo "TESTS $rc"; grep -E "FAILED|ERROR" gpurun_out/r04i_tests.log | head -20; tail -1 gpurun_out/r04i_tests.log
case $rc in 124|134|137|139) exit $rc;; esac
bash scripts/gpu_ab.sh r04i_c2 3 base g0 -- --config c2 --no-e2e --no-profile || exit 3
for i in 1 2; do
  for v in c1 c0; do
    case $v in c1) ENVV="BSGP_TW400C=1";; c0) ENVV="BSGP_TW400C=0";; esac
    env $ENVV timeout -k 10 300 python bench.py --config sub375 --no-cpu --no-e2e --no-profile \
      --steps 3 --warmup 1 > gpurun_out/r04i_sub375_${v}_$i.json 2> gpurun_out/r04i_sub375_${v}_$i.err \
      || { echo "bench $v failed"; tail -5 gpurun_out/r04i_sub375_${v}_$i.err; exit 3; }
    python -c "import json;d=json.load(open('gpurun_out/r04i_sub375_${v}_$i.json'));print('sub375 $v', round(d['value']))"
  done
done
