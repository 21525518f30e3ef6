"""HBM traffic of the solver kernels from rocprofv3 --pmc CSVs.

Usage: python tools/traffic_from_pmc.py FETCH_CSV WRITE_CSV OUT_JSON [note]

FETCH_SIZE / WRITE_SIZE are in KiB per dispatch.  On gfx950 FETCH_SIZE counts
64 B per 128-B request of a wide coalesced stream, i.e. exactly half of the
bytes (MI355X_MICROARCH.md §HBM), so it is doubled; WRITE_SIZE is exact for
16-B/lane stores.  Both count the L2's fabric requests (Infinity-Cache hits
included).  For every solver kernel class (k_setup, k_dir, k_col, k_ls, k_bb, k_persist)
the bytes are averaged over its dispatches, giving HBM bytes per launch to
compare with bench.py's per-kernel algorithmic bytes (run the PMC passes with
--streams 1 so a launch is the whole batch, as in bench.py's profiled solve).
"""
import csv
import re
import json
import sys
from collections import defaultdict

SOLVER = ("k_setup", "k_dir", "k_col", "k_ls", "k_bb", "k_persist")


def load(f, ctr):
    tot = defaultdict(float)
    disp = defaultdict(set)
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] != ctr:
            continue
        name = r["Kernel_Name"]
        # any build namespace: bsgp, bsgp_c512 (cooperative), bsgp_app (400/480 grids)
        key = next((k for k in SOLVER if re.search(r"bsgp\w*::" + k + r"<", name)), None)
        if key is None:
            continue
        tot[key] += float(r["Counter_Value"]) * 1024.0
        disp[key].add(r.get("Dispatch_Id") or r.get("Correlation_Id") or len(disp[key]))
    return tot, {k: len(v) for k, v in disp.items()}


def main():
    fetch, nf = load(sys.argv[1], "FETCH_SIZE")
    write, nw = load(sys.argv[2], "WRITE_SIZE")
    kernels = {}
    for k in SOLVER:
        if k not in fetch or k not in write:
            continue
        f = 2.0 * fetch[k] / nf[k]
        w = write[k] / nw[k]
        kernels[k] = {"fetch_bytes_per_launch": f, "write_bytes_per_launch": w,
                      "bytes_per_launch": f + w, "launches": nf[k]}
    out = {"kernels": kernels,
           "note": ("HBM bytes per launch per solver kernel: FETCH_SIZE x2 (gfx950 coalesced-"
                    "stream correction) + WRITE_SIZE, averaged over the kernel's dispatches "
                    "(rocprofv3 --pmc, one counter per pass)"
                    + (f"; {sys.argv[4]}" if len(sys.argv) > 4 else ""))}
    json.dump(out, open(sys.argv[3], "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
