#!/bin/bash
# Round 4: full GPU suite; static 400/480 FFT plans A/B (C3, sub375); sub450 coop vs per-wave.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 1200 python -u -m pytest tests -m gpu -v -rf -p no:cacheprovider --timeout 300 \
  --timeout-method thread > gpurun_out/r04c_tests.log 2>&1
rc=$?
echo "TESTS $rc"; grep -E "FAILED|ERROR" gpurun_out/r04c_tests.log | head -20; tail -2 gpurun_out/r04c_tests.log
case $rc in 124|134|137|139) exit $rc;; esac
bash scripts/gpu_ab.sh r04c_c3 2 base nostat -- --no-e2e --no-profile || exit 3
bash scripts/gpu_ab.sh r04c_sub375 2 base nostat -- --config sub375 --no-e2e --no-profile || exit 3
for v in coop w2; do
  case $v in
    coop) ENVV="";;
    w2) ENVV="BSGP_PERWAVE_MIN_WG=2";;
  esac
  env $ENVV timeout -k 10 300 python bench.py --config sub450 --no-cpu --no-e2e \
    --no-profile --steps 3 --warmup 1 > gpurun_out/r04c_sub450_$v.json 2> gpurun_out/r04c_sub450_$v.err \
    || { echo "bench $v failed"; tail -5 gpurun_out/r04c_sub450_$v.err; exit 3; }
  python -c "import json;d=json.load(open('gpurun_out/r04c_sub450_$v.json'));print('sub450 $v', round(d['value']))"
done
timeout -k 10 300 python bench.py --config sub375 --no-cpu --no-e2e --steps 2 --warmup 1 \
  > gpurun_out/r04c_sub375_prof.json 2> gpurun_out/r04c_sub375_prof.err || { echo "prof failed"; exit 3; }
python - <<'PY'
import json
d = json.load(open("gpurun_out/r04c_sub375_prof.json"))
r = d["roofline"]
print("sub375", round(d["value"]), "frac", round(r["frac"], 3), "solve frac", round(r["solve"]["frac_timed"], 3))
for k, v in r["phase_kernels"]["kernels"].items():
    print(" ", k, {a: round(b, 3) for a, b in v.items() if isinstance(b, float)})
PY
