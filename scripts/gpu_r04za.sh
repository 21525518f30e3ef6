#!/bin/bash
# Two thread groups for one-group cooperative plans (C4) by default: GPU suite and C4 lines.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/r04za; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 \
  --timeout-method thread > gpurun_out/r04za/tests.log 2>&1
rc=$?; echo "TESTS $rc"; tail -1 gpurun_out/r04za/tests.log; [ $rc -eq 0 ] || exit $rc
for cfg in "c4 --storage f32" "c4"; do
  name=$(echo $cfg | tr ' ' '_' | tr -d '-')
  timeout -k 10 400 python bench.py --config $cfg --no-cpu > gpurun_out/r04za/bench_$name.json 2> gpurun_out/r04za/bench_$name.err || { echo "bench $cfg failed"; tail -5 gpurun_out/r04za/bench_$name.err; exit 3; }
  python -c "import json;d=json.load(open('gpurun_out/r04za/bench_$name.json'));print('$name', round(d['value']), round(d['ms_per_step'],2))"
done
