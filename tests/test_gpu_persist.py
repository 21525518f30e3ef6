"""The persistent task-queue solver (k_persist, include/bsgp.h `persistent`):
one launch runs every iteration of every one-workgroup image by dequeuing
(iteration, image) tasks, with an agent-scope hand-off between the workgroups
that run consecutive iterations of an image.  It executes the same phase code
as the per-iteration kernels, so results must be bit-identical to theirs --
for every objective mode, both storages, data-dependent stop rules (tasks of
stopped images are skipped) and batches larger than the resident workgroups
(tasks wait for their predecessor iteration).  MI355X tests.
"""
import numpy as np
import pytest

from conftest import golden, ref_kwargs

pytestmark = pytest.mark.gpu

KEYS = ("x", "iters", "discr", "crit", "flags", "beta_final")


@pytest.fixture(scope="module")
def sgpmod():
    import _bsgp
    _bsgp.require_gpu()
    import sgp
    return sgp


def both(fn, *a, **kw):
    p0 = fn(*a, persistent=0, **kw)
    p1 = fn(*a, persistent=1, **kw)
    for k in KEYS:
        if p0.get(k) is not None:
            np.testing.assert_array_equal(p1[k], p0[k], err_msg=k)
    np.testing.assert_array_equal(p1["counters"][:, :3], p0["counters"][:, :3])
    np.testing.assert_array_equal(p1["counters"][:, 4:], p0["counters"][:, 4:])
    assert np.all(p1["counters"][:, 3] == 0)
    return p1


@pytest.mark.parametrize("case", ["beta", "kl", "adapt", "beta1", "f32storage"])
def test_persistent_bitwise_equal_to_phase_kernels(sgpmod, case):
    fx = golden("ref_lin64_beta.npz")
    gn = fx["gn"].astype(np.float64)
    gns = np.stack([np.roll(gn, 5 * i, 1) for i in range(6)])
    kw = dict(init_recon=2, proj_type=1, stop_criterion=1, MAXIT=12, alpha=10.0,
              ccd_sat_level=65000.0, use_original_SGP_Afunction=False, schedule_lr=True, team=1)
    if case == "kl":
        both(sgpmod.sgp_batch, gns, fx["psf"], 100.0, **kw)
        return
    betas = [1.05, 0.97, 1.02, 0.99, 1.08, 1.01]
    if case == "beta1":
        betas = [1.0] * 6
    extra = dict(adapt_beta=case == "adapt", storage="f32" if case == "f32storage" else "f64")
    both(sgpmod.sgp_betaDiv_batch, gns, fx["psf"], 100.0, betaParams=betas, **kw, **extra)


def test_persistent_stop3_matches_reference(sgpmod):
    """Stop rule 3 inside the persistent launch (no host polling): the
    reference's stop-3 run of the timed workload, and bitwise the phase
    kernels, in a batch whose images stop at different iterations."""
    fx = golden("ref_c3stop3_s0.npz")
    kw = ref_kwargs(fx)
    g = fx["gn"].astype(np.float64)
    gns = np.stack([g, np.roll(g, 40, 0), g.T.copy()])
    out = both(sgpmod.sgp_betaDiv_batch, gns, fx["psf"], 100.0, team=1, **kw)
    assert int(out["iters"][0]) == int(fx["iters"])
    r = np.linalg.norm(out["x"][0] - fx["x"]) / np.linalg.norm(fx["x"])
    assert r < 1e-5, r
    np.testing.assert_allclose(out["discr"][0, :int(fx["iters"]) + 1], fx["discr"], rtol=1e-7)


def test_persistent_more_images_than_slots(sgpmod):
    """1600 images (more than the workgroups the device holds at once): tasks
    of iteration k + 1 wait for iteration k of the same image, handed over
    between workgroups on other CUs and XCDs; bitwise the phase kernels."""
    fx = golden("ref_lin64_beta.npz")
    gn = fx["gn"].astype(np.float64)
    rng = np.random.default_rng(11)
    gns = np.stack([np.roll(np.roll(gn, int(rng.integers(64)), 0), int(rng.integers(64)), 1)
                    for _ in range(1600)])
    kw = dict(init_recon=2, proj_type=1, stop_criterion=1, MAXIT=6, alpha=10.0,
              ccd_sat_level=65000.0, use_original_SGP_Afunction=False, schedule_lr=True,
              adapt_beta=False, betaParams=1.05, team=1)
    both(sgpmod.sgp_betaDiv_batch, gns, fx["psf"], 100.0, **kw)


@pytest.mark.parametrize("stop", [1, 3])
def test_persistent_handoff_timeout_reports_status(sgpmod, monkeypatch, stop):
    """A hand-off wait that gives up (BSGP_SPIN_LIMIT=0: the first poll that
    finds the predecessor iteration unfinished) ends the persistent solve
    with status bit 4 on the images it abandoned (k_persist_finalize), so the
    drop-in raises instead of returning unwritten outputs; the next solve
    (default limit) is bitwise the phase kernels again."""
    import _bsgp
    fx = golden("ref_lin64_beta.npz")
    gn = fx["gn"].astype(np.float64)
    gns = np.stack([np.roll(gn, 3 * i, 0) for i in range(8)])
    kw = dict(init_recon=2, proj_type=1, stop_criterion=stop, MAXIT=60, tol_convergence=1e-9,
              alpha=10.0, ccd_sat_level=65000.0, use_original_SGP_Afunction=False,
              schedule_lr=True, betaParams=1.05, team=1)
    monkeypatch.setenv("BSGP_SPIN_LIMIT", "0")
    with pytest.raises(_bsgp.BsgpError, match="timed out"):
        sgpmod.sgp_betaDiv_batch(gns, fx["psf"], 100.0, persistent=1, **kw)
    out = sgpmod.sgp_betaDiv_batch(gns, fx["psf"], 100.0, persistent=1, device_out=True, **kw)
    st = out["counters"].cpu().numpy()[:, 3]
    it = out["iters"].cpu().numpy()
    assert np.any(st & 4)
    assert np.all(it[(st & 4) != 0] < 60) and np.all(it >= 0)
    monkeypatch.delenv("BSGP_SPIN_LIMIT")
    both(sgpmod.sgp_betaDiv_batch, gns, fx["psf"], 100.0, **kw)


@pytest.mark.parametrize("case", ["app_f32", "f64", "adapt", "f32storage", "kl"])
def test_persistent_cooperative_plans_bitwise(sgpmod, case):
    """Cooperative plans (Geo::coop: transforms too long for per-wave buffers
    at two workgroups per CU, thread-group transforms in 512-thread
    workgroups) run the persistent solver of bsgp_persist_c512.hip: bitwise
    the cooperative phase kernels.  The application's CROWDED float32 frame
    (with its background map and flux, stop rule 3) reflected out to 640x640
    sits on a 675-point grid, which only the cooperative build holds; float64
    images, both storages, adaptive beta and KL."""
    from conftest import crowded_case
    import _bsgp
    gn, psf, bkg, kw, fn, fx = crowded_case("crowded_beta")
    kw = dict(kw)
    b0 = kw.pop("betaParam")
    flux = kw.pop("flux")
    kw.pop("adapt_beta", None)
    g = np.pad(np.asarray(gn, dtype=np.float32), ((0, 190), (0, 190)), mode="reflect")
    bk = np.pad(np.asarray(bkg), ((0, 190), (0, 190)), mode="reflect")
    flux = flux * (640 * 640) / (450 * 450)
    gns = np.stack([g, np.roll(g, 37, 0), np.roll(g, 11, 1)])
    if case != "app_f32":
        gns = gns.astype(np.float64)
    # 675-point grid: per-wave buffers 4 waves x 2 x 677 x 16 B + 1.25 KB = 87.9 KB exceed
    # the 81.7 KB of two workgroups per CU, so the plan is cooperative (bsgp_api.hip)
    plan = _bsgp.get_plan(640, 640, psf, _bsgp.BSGP_CONV_LINEAR_FILL)
    assert plan.P == plan.Q == 675
    kw.update(MAXIT=8, team=1)
    if case == "kl":
        both(sgpmod.sgp_batch, gns, psf, bk, flux=flux, **kw)
        return
    extra = dict(adapt_beta=case == "adapt", storage="f32" if case == "f32storage" else "f64")
    both(sgpmod.sgp_betaDiv_batch, gns, psf, bk, flux=flux, betaParams=[b0, 1.02, 0.97], **kw,
         **extra)


@pytest.mark.parametrize("case", ["beta", "kl"])
def test_persistent_app_build_375_within_rounding(sgpmod, case):
    """The application's 375^2 tiles (400-point grid, per-wave plan) run the
    application build's persistent solver (bsgp_persist_app.hip), whose
    400-point transforms use the compile-time 8*10*5 plan; the phase kernels
    keep the runtime 4*4*5*5 plan, which rounds differently.  So the two paths
    agree to rounding, not bitwise: equal iteration counts, x and the
    discrepancies at rtol 1e-9."""
    from conftest import app_case
    gn, psf, bkg, kw, fn, fx = app_case("app_beta2" if case == "beta" else "app_kl")
    assert gn.shape == (375, 375)
    kw = dict(kw)
    flux = kw.pop("flux")
    kw.update(MAXIT=12, stop_criterion=1, team=1)
    gns = np.stack([gn, np.roll(gn, 17, 0), np.roll(gn, 9, 1)])
    if case == "beta":
        b0 = kw.pop("betaParam")
        fn2, extra = sgpmod.sgp_betaDiv_batch, dict(betaParams=[b0, 1.02, 0.97])
    else:
        fn2, extra = sgpmod.sgp_batch, {}
    p0 = fn2(gns, psf, bkg, flux=flux, persistent=0, **kw, **extra)
    p1 = fn2(gns, psf, bkg, flux=flux, persistent=1, **kw, **extra)
    np.testing.assert_array_equal(p1["iters"], p0["iters"])
    assert np.all(p1["counters"][:, 3] == 0)
    for i in range(3):
        r = np.linalg.norm(p1["x"][i] - p0["x"][i]) / np.linalg.norm(p0["x"][i])
        assert r < 1e-9, (i, r)
        n = int(p0["iters"][i]) + 1
        np.testing.assert_allclose(p1["discr"][i, :n], p0["discr"][i, :n], rtol=1e-9)
