#!/bin/bash
# Phase profile of the stamps on the persistent solver at HEAD.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
BSGP_LIB=$PWD/beta-sgp_amd/libbsgp_prof.so timeout -k 10 300 python tools/phase_prof.py --config stamps31 --maxit 500 --batch 16384 --persistent 1 > gpurun_out/r03ff_stamps.txt 2>&1 || { tail -5 gpurun_out/r03ff_stamps.txt; exit 3; }
grep -v amdgpu.ids gpurun_out/r03ff_stamps.txt
