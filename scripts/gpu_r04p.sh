#!/bin/bash
# PSF check on plan build only (batch API): GPU suite, host timing of C4, C4 bench lines.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r04p; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 \
  --timeout-method thread > gpurun_out/r04p/tests.log 2>&1
rc=$?; echo "TESTS $rc"; tail -1 gpurun_out/r04p/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/step_timing.py --config c4 --storage f32 --steps 5 || exit 3
for cfg in "c4 --storage f32" "c4" "c2"; do
  name=$(echo $cfg | tr ' ' '_' | tr -d '-')
  timeout -k 10 400 python bench.py --config $cfg --no-cpu > gpurun_out/r04p/bench_$name.json 2> gpurun_out/r04p/bench_$name.err || { echo "bench $cfg failed"; tail -5 gpurun_out/r04p/bench_$name.err; exit 3; }
  python -c "import json;d=json.load(open('gpurun_out/r04p/bench_$name.json'));print('$name', round(d['value']), round(d['ms_per_step'],2))"
done
