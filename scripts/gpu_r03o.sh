#!/bin/bash
# C4 phase profiles with one / two coop thread groups; A/B old vs groups (kCCH 4/8).
set -o pipefail
TAG=${1:-r03o}
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
for v in g1 g2; do
  BSGP_LIB=$PWD/beta-sgp_amd/libbsgp_prof_$v.so timeout -k 10 300 python tools/phase_prof.py --config c4 --maxit 20 > gpurun_out/${TAG}_phase_c4_$v.txt 2>&1 || { echo "phase prof $v failed"; tail -5 gpurun_out/${TAG}_phase_c4_$v.txt; exit 3; }
  echo "== $v"; grep -v amdgpu.ids gpurun_out/${TAG}_phase_c4_$v.txt
done
bash scripts/gpu_ab.sh ${TAG}_c4f32 3 old base -- --config c4 --storage f32 --steps 10 --no-e2e
