#!/bin/bash
# Round 3: full GPU suite (long-run parity, float32 batch path, persistent solver)
# + interleaved A/B of the persistent solver on C3 + batch sweep. Usage: TAG
set -o pipefail
TAG=${1:-r03a}
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s -rf -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?
echo "TESTS EXIT $rc"; grep -E "FAILED|ERROR|x rel|passed|failed" gpurun_out/${TAG}_tests.log | head -40
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for i in 0 1; do
  for p in 0 1; do
    timeout -k 10 300 python bench.py --no-cpu --no-profile --steps 3 --persistent $p > gpurun_out/${TAG}_p${p}_$i.json 2> gpurun_out/${TAG}_p${p}_$i.err || { echo "bench p$p failed"; tail -3 gpurun_out/${TAG}_p${p}_$i.err; exit 3; }
    python -c "import json;d=json.load(open('gpurun_out/${TAG}_p${p}_$i.json'));print('persistent $p', round(d['value']), round(d['ms_per_step'],1))"
  done
done
for b in 768 1536; do
  for p in 0 1; do
    timeout -k 10 300 python bench.py --no-cpu --no-profile --steps 3 --batch $b --persistent $p > gpurun_out/${TAG}_b${b}_p$p.json 2> gpurun_out/${TAG}_b${b}_p$p.err || { echo "bench $b failed"; tail -3 gpurun_out/${TAG}_b${b}_p$p.err; exit 3; }
    python -c "import json;d=json.load(open('gpurun_out/${TAG}_b${b}_p$p.json'));print('batch $b persistent $p', round(d['value']), round(d['ms_per_step'],1))"
  done
done
