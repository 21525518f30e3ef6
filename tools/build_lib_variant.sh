#!/bin/bash
# Whole-library variant for A/B runs (scripts/gpu_ab.sh):
#   tools/build_lib_variant.sh NAME "-DFLAG=V ..." [SOURCE_ROOT]
# compiles every translation unit of SOURCE_ROOT (default: this tree; e.g. a
# `git worktree` of an older commit) in parallel -> beta-sgp_amd/libbsgp_NAME.so
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; FLAGS=$2; SRC=${3:-$R}
B=/tmp/bsgp_build_$NAME; mkdir -p $B
CF="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -mcode-object-version=5"
OBJS=(); PIDS=()
rm -f $B/*.o
for f in bsgp_solver bsgp_solver_f32 bsgp_solver_c512 bsgp_persist bsgp_persist_f32 bsgp_persist_c512 bsgp_persist_c512_f32 bsgp_persist_app bsgp_api bsgp_tiles bsgp_psf; do
  /opt/rocm/bin/hipcc $CF $FLAGS -I $SRC/include -c $SRC/beta-sgp_amd/csrc/$f.hip -o $B/$f.o &
  PIDS+=($!); OBJS+=($B/$f.o)
done
for p in "${PIDS[@]}"; do wait $p || { echo "variant $NAME: a translation unit failed"; exit 1; }; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $R/beta-sgp_amd/libbsgp_$NAME.so "${OBJS[@]}"
