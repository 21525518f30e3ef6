#!/bin/bash
# Build tuning variants of the library: tools/build_variants.sh NAME "-DFLAG=V ..." [NAME "FLAGS" ...]
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
while [ $# -ge 2 ]; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off \
    -mcode-object-version=5 $2 -I $R/include -o $R/beta-sgp_amd/libbsgp_$1.so \
    $R/beta-sgp_amd/csrc/bsgp_solver.hip $R/beta-sgp_amd/csrc/bsgp_solver_f32.hip $R/beta-sgp_amd/csrc/bsgp_solver_c512.hip $R/beta-sgp_amd/csrc/bsgp_api.hip $R/beta-sgp_amd/csrc/bsgp_tiles.hip $R/beta-sgp_amd/csrc/bsgp_psf.hip &
  shift 2
done
wait
