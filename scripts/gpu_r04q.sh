#!/bin/bash
# Phase profiles (libbsgp_prof.so) of the team configurations C2 and C4.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r04q; export TMPDIR=/tmp
for c in c2 c4; do
  BSGP_LIB=$PWD/beta-sgp_amd/libbsgp_prof.so timeout -k 10 300 python tools/phase_prof.py --config $c --maxit 20 > gpurun_out/r04q/phase_$c.txt 2>&1 || { tail -5 gpurun_out/r04q/phase_$c.txt; exit 3; }
  cat gpurun_out/r04q/phase_$c.txt
done
