#!/bin/bash
# Final evidence at HEAD: smoke, default bench line + rocprofv3 kernel stats, stamps and C4 lines.
set -o pipefail
TAG=${1:-r03kk}
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
bash scripts/gpu_final.sh ${TAG} || exit $?
for c in "stamps31 --steps 3" "c4 --storage f32 --steps 10" "c4 --steps 10"; do
  set -- $c; n=$1; shift; s=""; [ "$1" == "--storage" ] && s="_$2"
  timeout -k 10 400 python bench.py --config $n --no-cpu "$@" > gpurun_out/${TAG}_bench_$n$s.json 2> gpurun_out/${TAG}_bench_$n$s.err || { echo "bench $n failed"; tail -3 gpurun_out/${TAG}_bench_$n$s.err; exit 3; }
  python -c "import json;d=json.load(open('gpurun_out/${TAG}_bench_$n$s.json'));print('$n$s', round(d['value']), d['roofline']['kernel'], round(d['roofline']['frac'],3))"
done
