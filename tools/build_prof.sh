#!/bin/bash
# Build the phase-profiling variant of the library (libbsgp_prof.so, diagnostics only).
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off \
  -mcode-object-version=5 -DBSGP_PHASE_PROF "$@" -I $R/include -o $R/beta-sgp_amd/libbsgp_prof.so \
  $R/beta-sgp_amd/csrc/bsgp_solver.hip $R/beta-sgp_amd/csrc/bsgp_solver_f32.hip $R/beta-sgp_amd/csrc/bsgp_solver_c512.hip $R/beta-sgp_amd/csrc/bsgp_persist.hip $R/beta-sgp_amd/csrc/bsgp_persist_f32.hip $R/beta-sgp_amd/csrc/bsgp_api.hip $R/beta-sgp_amd/csrc/bsgp_tiles.hip $R/beta-sgp_amd/csrc/bsgp_psf.hip
