#!/bin/bash
# Round 4: out-of-line 400/480 transforms (base) vs inline (inl) vs none (nostat).
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 \
  --timeout-method thread -k "persist or crowded or app or sub or satellite or stamps" > gpurun_out/r04d_tests.log 2>&1
rc=$?
echo "TESTS $rc"; grep -E "FAILED|ERROR" gpurun_out/r04d_tests.log | head; tail -1 gpurun_out/r04d_tests.log
case $rc in 124|134|137|139) exit $rc;; esac
bash scripts/gpu_ab.sh r04d_c3 3 base inl nostat -- --no-e2e --no-profile || exit 3
bash scripts/gpu_ab.sh r04d_sub375 2 base inl -- --config sub375 --no-e2e --no-profile || exit 3
bash scripts/gpu_ab.sh r04d_sub450 1 base inl -- --config sub450 --no-e2e --no-profile || exit 3
