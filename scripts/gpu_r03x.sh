#!/bin/bash
# Phase profiles of the persistent solver: stamps31 (persistent 1 and 0) and C3.
set -o pipefail
TAG=${1:-r03x}
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
export BSGP_LIB=$PWD/beta-sgp_amd/libbsgp_prof.so
run() { timeout -k 10 300 python tools/phase_prof.py "$@" > gpurun_out/${TAG}_$N.txt 2>&1 || { echo "phase prof $N failed"; tail -5 gpurun_out/${TAG}_$N.txt; exit 3; }; echo "== $N"; grep -v amdgpu.ids gpurun_out/${TAG}_$N.txt | awk '$NF != "" {print}' | grep -v " 0 cycles"; }
N=stamps_p1; run --config stamps31 --maxit 500 --batch 16384 --persistent 1
N=stamps_p0; run --config stamps31 --maxit 500 --batch 16384 --persistent 0
N=c3_p1; run --config c3 --maxit 100
