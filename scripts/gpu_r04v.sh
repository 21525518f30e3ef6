#!/bin/bash
# Application build with two operand batches in flight: suite subset, then A/B of combos
# (b1: + two-column batches, b2: + first batch before the transform) on 375^2 and 450^2.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r04v; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_app.py tests/test_gpu_persist.py -x -q -p no:cacheprovider --timeout 300 \
  --timeout-method thread > gpurun_out/r04v/tests.log 2>&1
rc=$?; echo "TESTS $rc"; tail -1 gpurun_out/r04v/tests.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_ab.sh r04v_sub375 2 base b1 b2 -- --config sub375 --no-e2e --no-profile || exit 3
bash scripts/gpu_ab.sh r04v_sub450 2 base b1 b2 -- --config sub450 --no-e2e --no-profile || exit 3
