#!/bin/bash
# Host launch throughput of the team configurations (tools/step_timing.py) and a C2 kernel trace.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r04n; export TMPDIR=/tmp
for c in "c2" "c4 --storage f32"; do
  timeout -k 10 300 python tools/step_timing.py --config $c --steps 5 || exit 3
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04n/c2prof -o run --output-format csv \
  -- python bench.py --config c2 --no-cpu --no-e2e --no-profile --steps 3 --warmup 1 > gpurun_out/r04n/c2prof.log 2>&1 || exit 3
echo done
