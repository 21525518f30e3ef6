"""bench.py's timed path, checked (GPU test helper; also runs as a script so a
test can start it in a fresh process with another GPU_MAX_HW_QUEUES).

BASELINE config C3 exactly as bench.py times it: 1024 x 256x256 images from
the bench generator, beta 1.05, 25x25 PSF, linear A, projection, MAXIT 100,
stop rule 1, team 1 (auto for 1024 images), the default sub-batch streams
(one per hardware queue: 4 by default, 8 under bench.py) and gn_compact on.
Image 0 is replaced by the reference's own input of ref_c3long_s0 (the
bench generator's statistics, seed 0) and must match that run; every image:
finite, x >= 0, sum(x) == flux; 8 sampled images bitwise equal to
single-image solves with gn_compact on and off.

    python tests/bench_path.py [--maxit 100]      (exit 0 = all checks passed)
"""
import argparse
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (HERE, ROOT, os.path.join(ROOT, "beta-sgp_amd"), os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402


def check(maxit=100, samples=(1, 137, 341, 511, 512, 700, 1000, 1023)):
    """Runs the checks (raises AssertionError on a failure); returns a summary."""
    import torch

    import bench
    import sgp
    from conftest import compare_trials, golden, ref_kwargs
    bench.torch = torch
    B = 1024
    gn, psf = bench.synth_batch(B, 256, 25, 200, seed0=0)
    fx = golden("ref_c3long_s0.npz")
    np.testing.assert_allclose(psf, fx["psf"], rtol=1e-15)
    gn[0] = torch.from_numpy(fx["gn"].astype(np.float64)).cuda()
    bkg = torch.full((B,), 100.0, dtype=torch.float64, device="cuda")
    kw = bench.solve_kwargs(maxit, None)
    ref = ref_kwargs(fx)
    for k in ("init_recon", "proj_type", "stop_criterion", "alpha", "ccd_sat_level", "betaParam",
              "schedule_lr", "adapt_beta", "use_original_SGP_Afunction"):
        assert kw[k] == ref[k], (k, kw[k], ref[k])
    assert kw["streams"] is None and kw["team"] is None
    assert sgp.GN_COMPACT_DEFAULT == 1
    out = sgp.sgp_betaDiv_batch(gn, psf, bkg, **kw)
    x = out["x"]
    assert np.all(out["counters"][:, 5] == 1) and np.all(out["counters"][:, 3] == 0)
    assert np.all(out["iters"] == maxit)
    assert np.all(np.isfinite(x)) and np.all(x >= 0)
    g = gn.cpu().numpy()
    flux = np.sum(g - 100.0, axis=(1, 2))
    np.testing.assert_allclose(x.sum(axis=(1, 2)), flux, rtol=1e-9)
    summary = {"streams": sgp.STREAMS_DEFAULT, "hw_queues": os.environ.get("GPU_MAX_HW_QUEUES"),
               "maxit": maxit}
    if maxit == int(fx["iters"]):
        r = np.linalg.norm(x[0] - fx["x"]) / np.linalg.norm(fx["x"])
        assert r < 1e-5, r
        np.testing.assert_allclose(out["discr"][0, :maxit + 1], fx["discr"], rtol=1e-7)
        diff = compare_trials(np.asarray(out["flags"][0, 1:maxit + 1]) >> 8, fx["trials"],
                              "bench image 0")
        summary.update(rel_x0=float(r), stagnating_trial_diffs=len(diff))
    for i in samples:
        for compact in (1, 0):
            one = sgp.sgp_betaDiv_batch(gn[i:i + 1], psf, bkg[i:i + 1],
                                        **dict(kw, team=1, streams=1, gn_compact=compact))
            assert one["iters"][0] == out["iters"][i]
            np.testing.assert_array_equal(one["x"][0], x[i])
            np.testing.assert_array_equal(one["discr"][0], out["discr"][i])
    return summary


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--maxit", type=int, default=100)
    a = ap.parse_args()
    print(json.dumps(check(a.maxit)), flush=True)
