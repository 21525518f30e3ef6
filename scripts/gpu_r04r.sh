#!/bin/bash
# Wide first-pass projection bracket for teams with few pixels per thread (BSGP_PROJ_WIDE_PX):
# GPU suite, then C2 A/B against the variant without it (libbsgp_pw0.so).
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r04r; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 \
  --timeout-method thread > gpurun_out/r04r/tests.log 2>&1
rc=$?; echo "TESTS $rc"; tail -1 gpurun_out/r04r/tests.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_ab.sh r04r_c2 3 base pw0 -- --config c2 --no-e2e || exit 3
python -c "import json;d=json.load(open('gpurun_out/r04r_c2_0_2.json'));print(d['roofline']['counters_per_iter'])"
