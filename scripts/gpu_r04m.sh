#!/bin/bash
# C4 cooperative-pass prefetch per call site: GPU suite on the new library (k_dir CPF 1,
# k_bb CPF 3), then interleaved A/B against no prefetch (pf0), k_dir off (cpfd0), k_bb gather only (cpfb1).
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 \
  --timeout-method thread > gpurun_out/r04m_tests.log 2>&1
rc=$?; echo "TESTS $rc"; tail -1 gpurun_out/r04m_tests.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_ab.sh r04m_c4f32 3 base pf0 cpfd0 cpfb1 -- --config c4 --storage f32 --no-e2e --no-profile || exit 3
bash scripts/gpu_ab.sh r04m_c4 2 base pf0 -- --config c4 --no-e2e --no-profile || exit 3
# where C4's timed step spends the time the profiled kernels do not account for
mkdir -p gpurun_out/r04m_c4prof
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/r04m_c4prof -o run --output-format csv \
  -- python bench.py --config c4 --storage f32 --no-cpu --no-e2e --no-profile --steps 3 --warmup 1 > gpurun_out/r04m_c4prof.log 2>&1 || exit 3
find gpurun_out/r04m_c4prof -name "*stats.csv" | xargs -r -n1 cut -d, -f1-4 | head -40
