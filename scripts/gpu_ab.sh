#!/bin/bash
# Interleaved A/B/... benchmark, REPS rounds, median per variant.
# Usage: bash scripts/gpu_ab.sh TAG REPS spec... [-- common bench args]
#   spec = LIB[,extra,bench,args][,NAME=VALUE env]   LIB "base" = libbsgp.so, else libbsgp_LIB.so
set -o pipefail
TAG=$1; REPS=$2; shift 2
SPECS=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do SPECS+=("$1"); shift; done
[ "$1" == "--" ] && shift
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
for ((i=0; i<REPS; i++)); do
  for k in "${!SPECS[@]}"; do
    IFS=',' read -ra PARTS <<< "${SPECS[$k]}"
    V=${PARTS[0]}; EXTRA=(); ENVS=()
    for x in "${PARTS[@]:1}"; do
      if [[ "$x" == --* || "$x" != *=* ]]; then EXTRA+=("$x"); else ENVS+=("$x"); fi
    done
    L=$PWD/beta-sgp_amd/libbsgp_$V.so; [ "$V" == "base" ] && L=$PWD/beta-sgp_amd/libbsgp.so
    env "${ENVS[@]}" BSGP_LIB=$L timeout -k 10 300 python bench.py --no-cpu --steps 3 "${EXTRA[@]}" "$@" > gpurun_out/${TAG}_${k}_$i.json 2> gpurun_out/${TAG}_${k}_$i.err || { echo "bench ${SPECS[$k]} failed"; tail -3 gpurun_out/${TAG}_${k}_$i.err; exit 3; }
  done
done
python - "$TAG" "$REPS" "${SPECS[@]}" <<'PY'
import json, sys, statistics
tag, reps, specs = sys.argv[1], int(sys.argv[2]), sys.argv[3:]
for k, v in enumerate(specs):
    js = [json.load(open(f"gpurun_out/{tag}_{k}_{i}.json")) for i in range(reps)]
    vals = [j["value"] for j in js]
    kern = ""
    rl = js[-1].get("roofline")
    if rl and "kernels" in rl:
        kern = " ".join(f"{n}={d.get('ms_per_launch', d['ms_total']):.3f}"
                        for n, d in rl["kernels"].items())
    print(f"{v:28s} median {statistics.median(vals):9.0f}  all {[round(x) for x in vals]}  {kern}")
PY
