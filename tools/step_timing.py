"""Diagnostics: where a team-image solve's wall time goes between its kernels.

For one bench configuration, times STEPS back-to-back solves three ways:
the host time each sgp_betaDiv_batch call takes to return (launch throughput),
the GPU span of each solve (torch events around the call), and the whole loop.
A host call that returns only when its GPU work is nearly done means the host
could not queue ahead, and the host work of the next call shows up as GPU idle
time between solves.

    python tools/step_timing.py --config c4 [--storage f32] [--steps 5]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "beta-sgp_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402

bench.torch = torch  # (bench imports torch lazily)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c4")
    ap.add_argument("--storage", default="f64")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--maxit", type=int, default=100)
    args = ap.parse_args()
    import sgp
    cfg = bench.CONFIGS[args.config]
    gn, psf = bench.synth_batch(cfg["batch"], cfg["n"], cfg["k"], cfg["nstars"], seed0=0,
                                circular=cfg["circular"])
    bkg = torch.full((cfg["batch"],), 100.0, dtype=torch.float64, device="cuda")
    kw = bench.solve_kwargs(args.maxit, None, circular=cfg["circular"], storage=args.storage)

    def step():
        return sgp.sgp_betaDiv_batch(gn, psf, bkg, device_out=True, **kw)

    step()
    torch.cuda.synchronize()
    host, ev = [], []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        h0 = time.perf_counter()
        e0.record()
        step()
        e1.record()
        host.append((time.perf_counter() - h0) * 1e3)
        ev.append((e0, e1))
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) * 1e3
    gpu = [a.elapsed_time(b) for a, b in ev]
    gaps = [ev[i][1].elapsed_time(ev[i + 1][0]) for i in range(len(ev) - 1)]
    print(f"{args.config} storage={args.storage}: wall {wall / args.steps:.2f} ms/step; "
          f"host call ms {np.round(host, 2).tolist()}; GPU span ms {np.round(gpu, 2).tolist()}; "
          f"gap between solves ms {np.round(gaps, 3).tolist()}")


if __name__ == "__main__":
    main()
