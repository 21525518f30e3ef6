#!/bin/bash
# Interleaved A/B/... benchmark of library variants, REPS rounds, median per variant.
# Usage: bash scripts/gpu_ab.sh TAG REPS name... [-- bench args]   (name "base" = libbsgp.so)
set -o pipefail
TAG=$1; REPS=$2; shift 2
NAMES=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do NAMES+=("$1"); shift; done
[ "$1" == "--" ] && shift
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
for ((i=0; i<REPS; i++)); do
  for V in "${NAMES[@]}"; do
    L=$PWD/beta-sgp_amd/libbsgp_$V.so; [ "$V" == "base" ] && L=$PWD/beta-sgp_amd/libbsgp.so
    BSGP_LIB=$L timeout -k 10 300 python bench.py --no-cpu --steps 3 "$@" > gpurun_out/${TAG}_${V}_$i.json 2> gpurun_out/${TAG}_${V}_$i.err || { echo "bench $V failed"; tail -3 gpurun_out/${TAG}_${V}_$i.err; exit 3; }
  done
done
python - "$TAG" "$REPS" "${NAMES[@]}" <<'PY'
import json, sys, statistics
tag, reps, names = sys.argv[1], int(sys.argv[2]), sys.argv[3:]
for v in names:
    vals = [json.load(open(f"gpurun_out/{tag}_{v}_{i}.json"))["value"] for i in range(reps)]
    print(f"{v:10s} median {statistics.median(vals):9.0f}  all {[round(x) for x in vals]}")
PY
