#!/bin/bash
# Variants of the persistent solver's float64 build only (bsgp_persist.hip),
# linked with the prebuilt objects of every other translation unit (build/*.o
# from __graft_entry__.build()):
#   tools/build_persist_variants.sh NAME "-DFLAG=V ..." [NAME "FLAGS" ...]
# -> beta-sgp_amd/libbsgp_NAME.so (for scripts/gpu_ab.sh)
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
B=$R/build
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -mcode-object-version=5"
OTHERS="$B/bsgp_solver.o $B/bsgp_solver_f32.o $B/bsgp_solver_c512.o $B/bsgp_persist_f32.o $B/bsgp_persist_c512.o $B/bsgp_persist_c512_f32.o $B/bsgp_persist_app.o $B/bsgp_api.o $B/bsgp_tiles.o $B/bsgp_psf.o"
while [ $# -ge 2 ]; do
  ( /opt/rocm/bin/hipcc $FLAGS $2 -I $R/include -c $R/beta-sgp_amd/csrc/bsgp_persist.hip -o $B/persist_$1.o &&
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $R/beta-sgp_amd/libbsgp_$1.so $B/persist_$1.o $OTHERS ) &
  shift 2
done
wait
