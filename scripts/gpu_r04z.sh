#!/bin/bash
# C4 with two thread groups per 512-thread workgroup (BSGP_COOP_ELEMS=8: a 2048-point
# transform per 256-thread group, two row pairs or columns at once) against one group.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r04z; export TMPDIR=/tmp
for i in 0 1; do  # (k_col keeps one group: nfc)
  for e in 4 8; do
    for st in f32 f64; do
      BSGP_COOP_ELEMS=$e timeout -k 10 300 python bench.py --config c4 --storage $st --no-cpu --no-e2e --steps 3 > gpurun_out/r04z/c4_${st}_e${e}_$i.json 2> gpurun_out/r04z/c4_${st}_e${e}_$i.err || { echo "bench e$e $st failed"; tail -3 gpurun_out/r04z/c4_${st}_e${e}_$i.err; exit 3; }
      python -c "import json;d=json.load(open('gpurun_out/r04z/c4_${st}_e${e}_$i.json'));k=d['roofline']['kernels'];print('e$e $st', round(d['value']), {n:round(v.get('ms_per_launch',0)*1e3,1) for n,v in k.items() if v.get('launches')})"
    done
  done
done
BSGP_COOP_ELEMS=8 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "c4 or 2048" -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r04z/tests.log 2>&1; echo "TESTS e8 $?"; tail -1 gpurun_out/r04z/tests.log
