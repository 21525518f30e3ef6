#!/bin/bash
# Round 3: star-stamp parity diagnostics. Usage: TAG
set -o pipefail
TAG=${1:-r03e}
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
PYT="python -u -m pytest -m gpu -v -s -rf -p no:cacheprovider --timeout 240 --timeout-method thread"
timeout -k 10 300 $PYT tests/test_gpu_stamps.py -k alone > gpurun_out/${TAG}_stamps.log 2>&1
rc=$?; echo "STAMPS EXIT $rc"; grep -E "PASSED|FAILED|^E  |parted" gpurun_out/${TAG}_stamps.log | cut -c1-600 | head -30
