#!/bin/bash
# GPU suite + A/B of the line search's fused first-pass reduction (libbsgp.so)
# against the previous build (libbsgp_old.so): C3, then C4/C2, interleaved.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
bash scripts/gpu_tests.sh ls_tests || exit 3
bash scripts/gpu_ab.sh lsr 3 base old || exit 3
for i in 0 1 2; do
  for L in base old; do
    LIB=$PWD/beta-sgp_amd/libbsgp_$L.so; [ $L == base ] && LIB=$PWD/beta-sgp_amd/libbsgp.so
    for C in "c4 --storage f32" "c2"; do
      N=$(echo $C | cut -d' ' -f1)
      BSGP_LIB=$LIB timeout -k 10 200 python bench.py --config $C --no-cpu --no-profile --steps 3 > gpurun_out/lsr_${N}_${L}_$i.json 2> gpurun_out/lsr_${N}_${L}_$i.err || { echo "$L $N failed"; exit 3; }
      python -c "import json;d=json.load(open('gpurun_out/lsr_${N}_${L}_$i.json'));print('$L $N', round(d['value']))"
    done
  done
done
