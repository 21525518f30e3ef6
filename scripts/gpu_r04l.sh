#!/bin/bash
# C4 cooperative-pass prefetch (BSGP_COOP1_PF): GPU suite on the new library, then
# interleaved A/B against the PF=0 build (libbsgp_pf0.so), C4 f32 and f64.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 \
  --timeout-method thread > gpurun_out/r04l_tests.log 2>&1
rc=$?; echo "TESTS $rc"; tail -1 gpurun_out/r04l_tests.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_ab.sh r04l_c4f32 3 base pf0 -- --config c4 --storage f32 --no-e2e --no-profile || exit 3
bash scripts/gpu_ab.sh r04l_c4 2 base pf0 -- --config c4 --no-e2e --no-profile || exit 3
