#!/bin/bash
# Print VGPR / spill / scratch of every kernel in a solver translation unit
# (gfx950).  Usage: tools/regcheck.sh [file.hip (default bsgp_solver.hip)] [extra hipcc flags]
set -e
R=${REGROOT:-$(cd "$(dirname "$0")/.." && pwd)}
SRC=${1:-bsgp_solver.hip}; shift || true
D=$(mktemp -d)
cd $D
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -mcode-object-version=5 \
  -I $R/include -c $R/beta-sgp_amd/csrc/$SRC -o s.o -save-temps "$@" 2>/dev/null
python3 - "${SRC%.hip}" <<'PY'
import re, sys
s=open(f'{sys.argv[1]}-hip-amdgcn-amd-amdhsa-gfx950.s').read()
blocks=s.split('.name:')
for b in blocks[1:]:
    name=b.split()[0]
    def g(k):
        m=re.search(r'\.'+k+r':\s+(\d+)', b); return m.group(1) if m else '?'
    print(f"{name[:60]:60s} vgpr={g('vgpr_count')} spill={g('vgpr_spill_count')} scratch={g('private_segment_fixed_size')} sgpr={g('sgpr_count')}")
PY
rm -rf $D
