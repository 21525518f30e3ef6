"""The boundary as other hosts use it, and the multi-device host path at
BASELINE config C5's size (MI355X tests).

* INTEGRATION.md §2's stand-alone ctypes stub, run as it stands through
  bsgp_solve_host (host buffers in, host buffers out), against
  bsgp_solve_device on the same inputs and parameters (bit for bit) and
  against the reference's 100-iteration run of image 0.
* C5: 8192 x 256x256 subdivisions through
  sgp_betaDiv_batch(devices=[0] * 8): eight shards, eight host threads on the
  one GPU of a test box (the round-end 8-GPU run spreads them over eight
  devices).  Every image: finite, x >= 0, sum(x) == flux; sampled images
  bitwise equal to single-image solves.
"""
import os
import re

import numpy as np
import pytest

from conftest import ROOT, golden

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def sgpmod():
    import _bsgp
    _bsgp.require_gpu()
    import sgp
    return sgp


def integration_stub():
    txt = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    sec = txt[txt.index("## 2. The C ABI"):]
    return re.search(r"```python\n(.*?)```", sec, re.S).group(1)


def test_integration_stub_runs_verbatim(sgpmod, monkeypatch):
    fx = golden("ref_c3long_s0.npz")
    g0 = fx["gn"].astype(np.float64)
    images = np.stack([g0, np.roll(g0, 17, 0), g0.T.copy(), np.roll(g0, -40, 1)])
    monkeypatch.chdir(ROOT)
    ns = {"images": images, "psf": fx["psf"]}
    exec(compile(integration_stub(), "INTEGRATION.md#2", "exec"), ns)
    x, iters, discr = ns["x"], ns["iters"], ns["discr"]
    assert np.all(iters == 100)
    r = np.linalg.norm(x[0] - fx["x"]) / np.linalg.norm(fx["x"])
    assert r < 1e-5, r
    np.testing.assert_allclose(discr[0], fx["discr"], rtol=1e-7)
    # the device entry point with the stub's parameters (projection without the
    # pixel lists, f64 gn, one stream, automatic team size): the same bits
    out = sgpmod.sgp_betaDiv_batch(images, fx["psf"], 100.0, betaParam=1.05, init_recon=2,
                                   proj_type=1, stop_criterion=1, MAXIT=100, alpha=10.0,
                                   ccd_sat_level=65000.0, use_original_SGP_Afunction=False,
                                   schedule_lr=True, adapt_beta=False, proj_cache=0, gn_compact=0,
                                   streams=1, team=0)
    np.testing.assert_array_equal(out["iters"], iters)
    np.testing.assert_array_equal(out["x"], x)
    np.testing.assert_array_equal(out["discr"], discr)


def test_c5_8192_images_sharded(sgpmod):
    import torch

    import bench
    bench.torch = torch
    B = 8192
    gn, psf = bench.synth_batch(B, 256, 25, 200, seed0=0)
    bkg = torch.full((B,), 100.0, dtype=torch.float64, device="cuda")
    kw = bench.solve_kwargs(5, None)
    out = sgpmod.sgp_betaDiv_batch(gn, psf, bkg, devices=[0] * 8, **kw)
    x = out["x"]
    assert x.shape == (B, 256, 256)
    assert np.all(out["iters"] == 5) and np.all(out["counters"][:, 3] == 0)
    assert np.all(out["counters"][:, 5] == 1)  # shards sharing a GPU run one workgroup per image
    assert np.all(np.isfinite(x)) and np.all(x >= 0)
    flux = (gn - 100.0).sum(dim=(1, 2)).cpu().numpy()
    np.testing.assert_allclose(x.sum(axis=(1, 2)), flux, rtol=1e-9)
    for i in (0, 1, 1023, 1024, 4095, 4096, 6000, 8191):
        one = sgpmod.sgp_betaDiv_batch(gn[i:i + 1], psf, bkg[i:i + 1],
                                       **dict(kw, team=1, streams=1))
        np.testing.assert_array_equal(one["x"][0], x[i])
        np.testing.assert_array_equal(one["discr"][0], out["discr"][i])


def test_per_image_psf_tensor_sharded(sgpmod):
    """devices=[...] with a [B, kh, kw] PSF tensor: each shard's stamps reach
    the plan on the worker's device; results equal the plain
    per-image-PSF batch."""
    import torch
    fx = golden("ref_lin64_beta.npz")
    gn = fx["gn"].astype(np.float64)
    gns = np.stack([np.roll(gn, 3 * i, 1) for i in range(4)])
    k = fx["psf"]
    psfs = torch.from_numpy(np.stack([k, k.T.copy(), k[::-1].copy(), k[:, ::-1].copy()])).cuda()
    kw = dict(init_recon=2, proj_type=1, stop_criterion=1, MAXIT=8, alpha=10.0,
              ccd_sat_level=65000.0, use_original_SGP_Afunction=False, schedule_lr=True,
              adapt_beta=False, betaParams=1.05, team=1)
    plain = sgpmod.sgp_betaDiv_batch(gns, psfs, 100.0, **kw)
    sh = sgpmod.sgp_betaDiv_batch(gns, psfs, 100.0, devices=[0, 0], **kw)
    np.testing.assert_array_equal(sh["x"], plain["x"])


def test_plan_pool_reuses_plans_across_threads(sgpmod):
    """Solve plans are leased from a pool keyed without the host thread:
    repeated devices=[0, 0] calls (new threads every time) never hold more
    plans than shards run at once (2), however the threads interleave (the
    first call's two threads may or may not overlap, so it leaves 1 or 2)."""
    import _bsgp
    fx = golden("ref_lin64_beta.npz")
    gns = np.stack([fx["gn"].astype(np.float64)] * 4)
    kw = dict(init_recon=2, proj_type=1, stop_criterion=1, MAXIT=3, alpha=10.0,
              ccd_sat_level=65000.0, use_original_SGP_Afunction=False, betaParams=1.05)
    _, key = _bsgp._plan_key(64, 64, np.asarray(fx["psf"]), _bsgp.BSGP_CONV_LINEAR_FILL, "f64")
    a = sgpmod.sgp_betaDiv_batch(gns, fx["psf"], 100.0, devices=[0, 0], **kw)
    for _ in range(3):
        b = sgpmod.sgp_betaDiv_batch(gns, fx["psf"], 100.0, devices=[0, 0], **kw)
        assert 1 <= len(_bsgp._pool[key]) <= 2, len(_bsgp._pool[key])
        np.testing.assert_array_equal(a["x"], b["x"])


def test_plan_cache_matches_psf_content(sgpmod):
    """Plans are keyed by a fingerprint of a strided sample of the PSF and
    matched by its full bytes: two PSFs that differ only off the sample share
    a key but never a plan, in the per-thread cache and in the solve pool, and
    a solve with the second PSF equals a solve on a fresh plan of it."""
    import _bsgp
    rng = np.random.default_rng(3)
    psf = rng.random((128, 128))
    psf /= psf.sum()
    psf2 = psf.copy()
    d = 0.5 * psf[0, 2]  # mass moved between elements 1 and 2, off the sample (every 4th)
    psf2[0, 1] += d
    psf2[0, 2] -= d
    mode = _bsgp.BSGP_CONV_CIRCULAR
    k1 = _bsgp._plan_key(128, 128, psf, mode, "f64")[1]
    k2 = _bsgp._plan_key(128, 128, psf2, mode, "f64")[1]
    assert k1 == k2
    p1 = _bsgp.get_plan(128, 128, psf, mode)
    p2 = _bsgp.get_plan(128, 128, psf2, mode)
    assert p1 is not p2 and np.array_equal(p2._psf_host, psf2)
    assert _bsgp.get_plan(128, 128, psf2, mode) is p2
    gn = (rng.poisson(200.0, (1, 128, 128)) + 1.0).astype(np.float64)
    kw = dict(init_recon=2, proj_type=1, stop_criterion=1, MAXIT=3, betaParams=1.05)
    a = sgpmod.sgp_betaDiv_batch(gn, psf, 10.0, **kw)
    b = sgpmod.sgp_betaDiv_batch(gn, psf2, 10.0, **kw)
    _bsgp._pool.clear()
    c = sgpmod.sgp_betaDiv_batch(gn, psf2, 10.0, **kw)
    np.testing.assert_array_equal(b["x"], c["x"])
    assert not np.array_equal(a["x"], b["x"])
    # the batch API checks a PSF's normalisation when it builds its plan, so an
    # unnormalised PSF (never pooled) is refused on every call
    for _ in range(2):
        with pytest.raises(ValueError, match="PSF is not normalized"):
            sgpmod.sgp_betaDiv_batch(gn, 2 * psf, 10.0, **kw)


def test_device_scope_restores_current_device(sgpmod):
    """Every plan entry point restores the caller's current device: after a
    plan is created and destroyed from another thread, this thread's current
    device is unchanged (one GPU: the index stays 0 and HIP stays usable)."""
    import threading

    import _bsgp
    import torch
    dev = torch.cuda.current_device()
    p = _bsgp.Plan(32, 32, np.full((3, 3), 1 / 9.0), _bsgp.BSGP_CONV_LINEAR_FILL)
    t = threading.Thread(target=lambda: p.__del__())
    t.start()
    t.join()
    assert torch.cuda.current_device() == dev
    assert float(torch.ones(3, device="cuda").sum()) == 3.0
