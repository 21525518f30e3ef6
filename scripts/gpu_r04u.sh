#!/bin/bash
# Application build at two waves per SIMD: GPU suite, then operand-batch knobs A/B
# (a1: first batch before the transform, a2: two batches in flight, a3: two-column batches)
# on the 375^2 tiles and 450^2 frames.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r04u; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 \
  --timeout-method thread > gpurun_out/r04u/tests.log 2>&1
rc=$?; echo "TESTS $rc"; tail -1 gpurun_out/r04u/tests.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_ab.sh r04u_sub375 2 base a1 a2 a3 -- --config sub375 --no-e2e --no-profile || exit 3
bash scripts/gpu_ab.sh r04u_sub450 2 base a1 a2 a3 -- --config sub450 --no-e2e --no-profile || exit 3
