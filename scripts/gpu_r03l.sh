#!/bin/bash
# Phase profiles at HEAD: C2, C4, C3 (persistent), stamps31.
set -o pipefail
TAG=${1:-r03l}
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
export BSGP_LIB=$PWD/beta-sgp_amd/libbsgp_prof.so
for c in c2 c4 c3 stamps31; do
  B=""; M=20; [ $c == c3 ] && M=100; [ $c == stamps31 ] && { B="--batch 4096"; M=500; }
  timeout -k 10 300 python tools/phase_prof.py --config $c --maxit $M $B > gpurun_out/${TAG}_phase_$c.txt 2>&1 || { echo "phase prof $c failed"; tail -5 gpurun_out/${TAG}_phase_$c.txt; exit 3; }
  echo "== $c"; cat gpurun_out/${TAG}_phase_$c.txt
done
