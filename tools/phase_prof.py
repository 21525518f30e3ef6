"""Per-phase cycle breakdown of the solver kernels (diagnostics).

Build a profiling variant of the library and run the bench workload with it:

    hipcc ... -DBSGP_PHASE_PROF -o beta-sgp_amd/libbsgp_prof.so ...   (tools/build_prof.sh)
    BSGP_LIB=$PWD/beta-sgp_amd/libbsgp_prof.so python tools/phase_prof.py [--streams S]

Thread 0 of every workgroup adds the shader cycles (s_memtime) it spent in
each phase; the table is the mean per workgroup-iteration (image-iteration
for team size 1), i.e. the latency one image spends in the phase.
"""
import argparse
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "beta-sgp_amd")):
    sys.path.insert(0, p)

SLOTS = {0: "k_dir projection", 1: "k_dir row pass", 2: "k_dir total", 3: "k_col total",
         4: "k_ls pass 1 (rows of A(d))", 5: "k_ls search loop", 6: "k_ls accept rows",
         7: "k_ls total", 8: "k_bb rows + BB sums", 10: "  proj first pass",
         11: "  proj list evals", 12: "  proj miss passes",
         13: "  ls1 rows: operand batches", 14: "  ls1 rows: FFT", 15: "  ls1 rows: stage/unpack",
         16: "  accept rows: operand batches", 17: "  accept rows: FFT", 18: "  accept rows: stores",
         19: "  bb rows: operand batches", 20: "  bb rows: FFT", 21: "  bb rows: stage/unpack",
         22: "  dir rows: operand batches", 23: "  dir rows: FFT", 24: "  dir rows: stores",
         25: "  coop rows: spectrum gathers | ls1 red.: own waves", 26: "  coop rows: FFTs | ls1 red.: other members", 27: "  coop rows: operands",
         28: "  coop rows: spectrum stores", 29: "  coop cols: loads", 30: "  coop cols: FFT+TF+store",
         31: "persistent: dequeue + wait for the previous iteration"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--streams", type=int, default=1)
    ap.add_argument("--maxit", type=int, default=20)
    ap.add_argument("--batch", type=int, default=None)
    ap.add_argument("--config", default="c3")
    ap.add_argument("--persistent", type=int, default=None,
                    help="1: the persistent solver (default for c3; stamps default 0)")
    args = ap.parse_args()
    import torch  # noqa: F401  (one HIP runtime, loaded before the library)
    import bench
    import _bsgp
    import sgp
    bench.torch = torch
    L = _bsgp.lib()
    L.bsgp_phase_prof.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32]
    buf = (ctypes.c_uint64 * 32)()
    if args.config == "app375":  # one application subdivision (bench.py app375), automatic team
        img, psf, bk, akw, betas = bench.app375_inputs()
        gn = torch.from_numpy(np.asarray(img, dtype=np.float32).copy()).cuda()[None]
        bkg = torch.from_numpy(np.asarray(bk, dtype=np.float64)).cuda()[None]
        kw = {k: v for k, v in akw.items() if k not in ("save", "verbose", "flux")}
        kw.update(betaParams=[betas[0]], flux=np.array([akw["flux"]]), streams=args.streams)
        cfg, B = {}, 1
    else:
        cfg = bench.CONFIGS[args.config]
        B = args.batch or cfg["batch"]
    if args.config == "app375":
        pass
    elif cfg.get("stamps"):  # the star-stamp workload (bench.py stamps31), phase kernels
        cuts, psf, bk, fl, betas = bench.stamp_inputs(B)
        gn = cuts
        bkg = bk
        kw = dict(bench.stamp_kwargs(args.maxit), betaParams=betas, flux=fl, streams=args.streams,
                  persistent=args.persistent or 0, team=1)
    else:
        gn, psf = bench.synth_batch(B, cfg["n"], cfg["k"], cfg["nstars"], 0,
                                    circular=cfg["circular"])
        bkg = torch.full((B,), 100.0, dtype=torch.float64, device="cuda")
        kw = bench.solve_kwargs(args.maxit, None, args.streams, None, circular=cfg["circular"],
                                persistent=args.persistent)
    sgp.sgp_betaDiv_batch(gn, psf, bkg, device_out=True, **kw)
    _bsgp.check(L.bsgp_phase_prof(buf, 32, 1))  # reset after warm-up
    out = sgp.sgp_betaDiv_batch(gn, psf, bkg, device_out=True, **kw)
    _bsgp.check(L.bsgp_phase_prof(buf, 32, 1))
    n = float(out["iters"].sum().item()) * float(out["counters"][0, 5].item())  # x team size
    for k, name in SLOTS.items():
        print(f"{name:32s} {buf[k] / n:12.0f} cycles per image-iteration"
              + (" (2 launches)" if k == 3 else ""))


if __name__ == "__main__":
    main()
