#!/bin/bash
# Phase profiles (shader cycles per image-iteration) of the persistent solver: C3 and sub375.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
L=$PWD/beta-sgp_amd/libbsgp_prof.so
BSGP_LIB=$L timeout -k 10 300 python tools/phase_prof.py --config c3 --persistent 1 --maxit 20 > gpurun_out/r04f_c3.txt 2>&1 || { echo c3 failed; tail -5 gpurun_out/r04f_c3.txt; exit 3; }
BSGP_LIB=$L timeout -k 10 300 python tools/phase_prof.py --config sub375 --persistent 1 --maxit 20 > gpurun_out/r04f_sub375.txt 2>&1 || { echo sub375 failed; tail -5 gpurun_out/r04f_sub375.txt; exit 3; }
paste gpurun_out/r04f_c3.txt gpurun_out/r04f_sub375.txt | awk -F'\t' '{printf "%-70s | %s\n", $1, $2}' | sed 's/cycles per image-iteration//g'
