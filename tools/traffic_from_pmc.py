"""HBM traffic of the solver kernels from rocprofv3 --pmc CSVs.

Usage: python tools/traffic_from_pmc.py FETCH_CSV WRITE_CSV OUT_JSON launches

FETCH_SIZE / WRITE_SIZE are in KiB per dispatch.  On gfx950 FETCH_SIZE counts
64 B per 128-B request of a wide coalesced stream, i.e. exactly half of the
bytes (MI355X_MICROARCH.md §HBM), so it is doubled; WRITE_SIZE is exact for
16-B/lane stores.  Sums every bsgp solver kernel (k_setup, k_dir, k_col,
k_ls, k_bb) over the profiled run and divides by the number of solves
(`launches`), giving HBM bytes per solve to compare with the algorithmic
bytes of bench.py's roofline.
"""
import csv
import json
import sys
from collections import defaultdict

SOLVER = ("k_setup", "k_dir", "k_col", "k_ls", "k_bb")


def load(f, ctr):
    per = defaultdict(float)
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] != ctr:
            continue
        name = r["Kernel_Name"]
        if any(f"bsgp::{k}" in name for k in SOLVER):
            key = next(k for k in SOLVER if f"bsgp::{k}" in name)
            per[key] += float(r["Counter_Value"]) * 1024.0
    return per


fetch = load(sys.argv[1], "FETCH_SIZE")
write = load(sys.argv[2], "WRITE_SIZE")
n = float(sys.argv[4])
out = {"fetch_bytes_per_solve": {k: 2.0 * v / n for k, v in fetch.items()},
       "write_bytes_per_solve": {k: v / n for k, v in write.items()}}
out["bytes_per_launch"] = sum(out["fetch_bytes_per_solve"].values()) + \
    sum(out["write_bytes_per_solve"].values())
out["note"] = ("HBM bytes per solve (all phase kernels), FETCH_SIZE x2 (gfx950 "
               "coalesced-stream correction) + WRITE_SIZE, from rocprofv3 --pmc")
json.dump(out, open(sys.argv[3], "w"), indent=1)
print(json.dumps(out, indent=1))
