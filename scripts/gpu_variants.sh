#!/bin/bash
# Bench each library variant (beta-sgp_amd/libbsgp_<name>.so): TAG name... [-- bench args]
set -o pipefail
TAG=$1; shift
NAMES=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do NAMES+=("$1"); shift; done
[ "$1" == "--" ] && shift
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
for V in "${NAMES[@]}"; do
  L=$PWD/beta-sgp_amd/libbsgp_$V.so; [ "$V" == "base" ] && L=$PWD/beta-sgp_amd/libbsgp.so
  for S in 1 2; do
    BSGP_LIB=$L timeout -k 10 300 python bench.py --no-cpu --streams $S --steps 2 "$@" > gpurun_out/${TAG}_${V}_s$S.json 2> gpurun_out/${TAG}_${V}_s$S.err || { echo "bench $V failed"; tail -3 gpurun_out/${TAG}_${V}_s$S.err; exit 3; }
    python -c "import json;d=json.load(open('gpurun_out/${TAG}_${V}_s$S.json'));print('$V streams $S', round(d['value']), 'ms', round(d['ms_per_step'],1))"
  done
done
