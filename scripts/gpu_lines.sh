#!/bin/bash
# Bench lines of several configurations on one lease (no CPU baseline).
# Usage: bash scripts/gpu_lines.sh TAG [config ...]   (default: c3 c2 "c4 --storage f32" c4 sub375)
set -o pipefail
TAG=${1:-lines}; shift
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/$TAG; export TMPDIR=/tmp
O=gpurun_out/$TAG
CFGS=("$@"); [ ${#CFGS[@]} -eq 0 ] && CFGS=("c3" "c2" "c4 --storage f32" "c4" "sub375")
for cfg in "${CFGS[@]}"; do
  name=$(echo $cfg | tr ' ' '_' | tr -d '-')
  timeout -k 10 300 python bench.py --no-cpu --config $cfg > $O/bench_$name.json 2> $O/bench_$name.err || { echo "bench $cfg failed"; tail -5 $O/bench_$name.err; exit 3; }
  python - $O/bench_$name.json $name <<'PY'
import json, sys
d = json.load(open(sys.argv[1])); r = d.get("roofline") or {}
k = r.get("kernels") or {}
print(sys.argv[2], round(d["value"]), "frac", round(r.get("frac") or 0, 3),
      {n: round(v.get("ms_per_launch", 0) * 1e3, 1) for n, v in k.items() if isinstance(v, dict)})
PY
done
