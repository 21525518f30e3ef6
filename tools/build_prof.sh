#!/bin/bash
# Build the phase-profiling variant of the library (libbsgp_prof.so, diagnostics
# only): every translation unit with -DBSGP_PHASE_PROF (tools/build_lib_variant.sh).
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
bash $R/tools/build_lib_variant.sh prof "-DBSGP_PHASE_PROF $*"
