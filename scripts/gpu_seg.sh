#!/bin/bash
# GPU suite + A/B of the projection's linear-segment shortcut (libbsgp.so) against
# the build without it (libbsgp_noseg.so): C3 interleaved, then C4 f32 and C2.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
bash scripts/gpu_tests.sh seg_tests || exit 3
bash scripts/gpu_ab.sh seg 3 base noseg || exit 3
for L in base noseg; do
  LIB=$PWD/beta-sgp_amd/libbsgp_$L.so; [ $L == base ] && LIB=$PWD/beta-sgp_amd/libbsgp.so
  for C in "c4 --storage f32" "c2"; do
    N=$(echo $C | cut -d' ' -f1)
    BSGP_LIB=$LIB timeout -k 10 200 python bench.py --config $C --no-cpu --steps 3 > gpurun_out/seg_${N}_$L.json 2> gpurun_out/seg_${N}_$L.err || { echo "$L $N failed"; tail -3 gpurun_out/seg_${N}_$L.err; exit 3; }
    python -c "import json;d=json.load(open('gpurun_out/seg_${N}_$L.json'));print('$L $N', round(d['value']), d['roofline']['counters_per_iter'])"
  done
done
