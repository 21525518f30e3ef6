#!/bin/bash
# Interleaved A/B of whole source trees (each with its own bench.py, drop-in
# and built libbsgp.so; e.g. a `git worktree` of an older round under
# scratch/), REPS rounds, median per tree.  The driver's own command line
# (python3 bench.py --gpus 1 --steps 20 --warmup 5) plus the common args.
# Usage: bash scripts/gpu_ab_trees.sh TAG REPS DIR... [-- common bench args]
#   DIR "." = this tree
set -o pipefail
TAG=$1; REPS=$2; shift 2
DIRS=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do DIRS+=("$1"); shift; done
[ "$1" == "--" ] && shift
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
OUT=$PWD/gpurun_out
for ((i=0; i<REPS; i++)); do
  for k in "${!DIRS[@]}"; do
    D=${DIRS[$k]}
    ( cd $D && timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu "$@" \
        > $OUT/${TAG}_${k}_$i.json 2> $OUT/${TAG}_${k}_$i.err ) ||
      { echo "bench in $D failed"; tail -3 $OUT/${TAG}_${k}_$i.err; exit 3; }
    echo "$TAG $D rep $i: $(python3 -c "import json;print(round(json.load(open('$OUT/${TAG}_${k}_$i.json'))['value']))")"
  done
done
python3 - "$TAG" "$REPS" "${DIRS[@]}" <<'PY'
import json, sys, statistics
tag, reps, dirs = sys.argv[1], int(sys.argv[2]), sys.argv[3:]
for k, d in enumerate(dirs):
    js = [json.load(open(f"gpurun_out/{tag}_{k}_{i}.json")) for i in range(reps)]
    vals = [j["value"] for j in js]
    kern = ""
    rl = js[-1].get("roofline")
    if rl and "kernels" in rl:
        kern = " ".join(f"{n}={v.get('ms_per_launch', v['ms_total']):.3f}"
                        for n, v in rl["kernels"].items() if v["launches"])
    print(f"{tag} {d:14s} median {statistics.median(vals):9.1f}  all {[round(x) for x in vals]}  {kern}")
PY
