#!/bin/bash
# Round-3 evidence at HEAD: smoke, default bench (C3) + rocprofv3 kernel stats,
# the other configs' bench lines, C3 PMC traffic.
set -o pipefail
TAG=${1:-r03w}
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
bash scripts/gpu_final.sh ${TAG} || exit $?
for c in "c4 --storage f32 --steps 10" "c4 --steps 10" "c2 --steps 10" "stamps31 --steps 3" "sub375 --steps 3" "c5"; do
  set -- $c; n=$1; shift; s=""; [ "$1" == "--storage" ] && s="_$2"
  timeout -k 10 400 python bench.py --config $n --no-cpu "$@" > gpurun_out/${TAG}_bench_$n$s.json 2> gpurun_out/${TAG}_bench_$n$s.err || { echo "bench $n failed"; tail -3 gpurun_out/${TAG}_bench_$n$s.err; exit 3; }
  python -c "import json;d=json.load(open('gpurun_out/${TAG}_bench_$n$s.json'));print('$n$s', round(d['value']), d['roofline']['kernel'], round(d['roofline']['frac'],3))"
done
bash scripts/gpu_traffic.sh c3_${TAG}
