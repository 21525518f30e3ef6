"""The drop-in's headline consumer and the remaining signature paths, on the
MI355X through the C ABI, against outputs of the reference itself
(tests/golden/make_golden.py app / errsave, py3.9 + astropy 4.3.1 + numpy 1.26).

* application_sgp_subdivisions.py:43-107: float32 big-endian FITS data
  (contiguous, and the application's non-contiguous crop of a wider frame),
  the 31x31 DIAPL PSF (>f8), a per-pixel background map, the provided flux
  (float64 and float32), stop rule 3 at tol 1e-5, every beta seed, the KL
  branch; the five seeds as one batched multi-start launch.
* errflag=True (sgp.py:240-257, 394-396) and save=True (sgp.py:223-231,
  416-422).

Tolerances: iteration counts equal, rel. L2 of x <= 1e-5 (north star),
discrepancy rtol 1e-7, against the reference's "_libm" runs (conftest.LIBM:
numpy's float32 power is the C library's powf, which the device evaluates bit
for bit).  The default-numpy (SVML) runs differ from those only through the
reference's float32 sum s*gn**beta, by at most a float32 ulp of it
(conftest.konst_shift, computed exactly); test_application_path_svml_set
checks them with that offset removed.
"""
import os

import numpy as np
import pytest

from conftest import APP_CASES, LIBM, SVML, app_case, golden, konst_shift, ref_kwargs

pytestmark = pytest.mark.gpu

SOLVE_RTOL = 1e-5


@pytest.fixture(scope="module")
def sgpmod():
    import _bsgp
    _bsgp.require_gpu()
    import sgp
    return sgp


def rel(a, b):
    return np.linalg.norm(np.asarray(a) - np.asarray(b)) / max(np.linalg.norm(np.asarray(b)), 1e-300)


@pytest.mark.parametrize("name", APP_CASES)
def test_application_path_matches_reference(name, sgpmod):
    gn, psf, bkg, kw, fn, fx = app_case(name)
    assert gn.dtype == np.dtype(">f4") and psf.dtype == np.dtype(">f8")
    x, it, discr, times, none = getattr(sgpmod, fn)(gn, psf, bkg, **kw)
    assert none is None
    assert it == int(fx["iters"]), (it, int(fx["iters"]))
    assert len(discr) == len(times) == it + 1
    assert rel(x, fx["x"]) < SOLVE_RTOL, rel(x, fx["x"])
    assert konst_shift(gn, kw, fx) == 0.0  # the same float32 sum as the reference's
    np.testing.assert_allclose(discr, fx["discr"], rtol=1e-7)
    # flux conservation of the projection (proj_type=1): sum(x) == flux, up to
    # the float32 rounding of flux/scaling for a float32 flux (sgp.py:666)
    f = float(kw["flux"])
    tol = 1e-7 if isinstance(kw["flux"], np.float32) else 1e-9
    assert abs(x.sum() - f) <= tol * f


def test_crowded_full_frame_matches_reference(sgpmod, monkeypatch):
    """The application's CROWDED mode (application_sgp_subdivisions.py:22,
    44-50, 84-115): the whole 450x450 float32 frame on its 480-point grid, a
    background map, the published flux, beta-SGP from the published best
    initial beta and the KL branch (stop rule 3, tol 1e-5): the single-image
    drop-in (automatic team) and a one-workgroup batch of both frames against
    the reference's runs.  The 480-point grid is a per-wave plan at two
    workgroups per CU (BSGP_PERWAVE_MIN_WG 2), so the batch runs the
    application build's persistent solver (bsgp_persist_app.hip); the
    cooperative persistent build is covered by test_gpu_persist's 640^2 frame."""
    from conftest import crowded_case
    for name in ("crowded_beta", "crowded_kl"):
        gn, psf, bkg, kw, fn, fx = crowded_case(name)
        assert gn.shape == (450, 450) and gn.dtype == np.dtype(">f4")
        x, it, discr, _, _ = getattr(sgpmod, fn)(gn, psf, bkg, **kw)
        assert it == int(fx["iters"]), (name, it, int(fx["iters"]))
        assert rel(x, fx["x"]) < SOLVE_RTOL, (name, rel(x, fx["x"]))
        np.testing.assert_allclose(discr, fx["discr"], rtol=1e-7)
        kb = dict(kw)
        f = kb.pop("flux")
        if fn == "sgp_betaDiv":
            b = kb.pop("betaParam")
            out = sgpmod.sgp_betaDiv_batch(np.stack([gn, gn]), psf, bkg, betaParams=[b, b],
                                           flux=f, team=1, **kb)
        else:
            out = sgpmod.sgp_batch(np.stack([gn, gn]), psf, bkg, flux=f, team=1, **kb)
        for i in range(2):
            assert int(out["iters"][i]) == int(fx["iters"])
            assert rel(out["x"][i], fx["x"]) < SOLVE_RTOL
            np.testing.assert_allclose(out["discr"][i, :it + 1], fx["discr"], rtol=1e-7)


@pytest.mark.parametrize("name", APP_CASES)
def test_application_path_svml_set(name, sgpmod):
    """The same runs against the reference under numpy's default float32
    power (SVML): equal iteration counts, x within 1e-5, and the discrepancy
    at rtol 1e-7 once the exact offset of the reference's float32 sum is
    removed (at most a float32 ulp of K; conftest.konst_shift)."""
    gn, psf, bkg, kw, fn, fx = app_case(name, SVML)
    x, it, discr, _, _ = getattr(sgpmod, fn)(gn, psf, bkg, **kw)
    assert it == int(fx["iters"]), (it, int(fx["iters"]))
    assert rel(x, fx["x"]) < SOLVE_RTOL, rel(x, fx["x"])
    shift = konst_shift(gn, kw, fx)
    assert abs(shift) <= 2e-4 * discr[0]
    np.testing.assert_allclose(discr - shift, fx["discr"], rtol=1e-7)


def test_float32_arithmetic_is_what_the_reference_does(sgpmod):
    """The same image promoted to float64 gives a discrepancy that differs from
    the reference's float32 run by ~6e-4 (its s*gn**beta sum is float32):
    the device's float32 emulation, not a float64 solve, is what matches."""
    gn, psf, bkg, kw, fn, fx = app_case("app_beta2")
    _, it64, d64, _, _ = sgpmod.sgp_betaDiv(gn.astype(np.float64), psf, bkg, **kw)
    assert np.max(np.abs(d64[:3] - fx["discr"][:3]) / fx["discr"][:3]) > 1e-5
    _, it32, d32, _, _ = sgpmod.sgp_betaDiv(gn, psf, bkg, **kw)
    np.testing.assert_allclose(d32, fx["discr"], rtol=1e-7)


def test_multistart_candidates_match_reference(sgpmod, tmp_path, monkeypatch):
    """The five seeds of application_sgp_subdivisions.py:70-76 in one batched
    launch: every candidate against its own reference run; then the argmin of
    the caller's score and the final solve with the best initial beta."""
    gn, psf, bkg, kw, fn, _ = app_case("app_beta0")
    kw = {k: v for k, v in kw.items() if k != "betaParam"}
    inp = golden("app_subdiv_inputs.npz")
    betas = sgpmod.app_beta_candidates()
    np.testing.assert_array_equal(betas, inp["betas"])
    target = [golden(f"ref_app_beta{i}{LIBM}.npz") for i in range(5)]

    def score(x):  # stands in for the photometric score; any function of the image
        return -float(np.max(x))

    monkeypatch.chdir(tmp_path)
    final, info = sgpmod.sgp_betaDiv_multistart(gn, psf, bkg, betas=None, score=score, **kw)
    # sgp.log: every candidate's lines (one sgp_betaDiv call each in the
    # application) and the final call's, which repeats the best candidate's
    import logging
    for h in logging.getLogger().handlers:
        h.flush()
    lines = [l for l in open("sgp.log").read().splitlines() if l.startswith("INFO:root:it ")]
    its = [c[1] for c in info["candidates"]]
    assert len(lines) == sum(i + 1 for i in its) + its[info["best"]] + 1
    assert info["betas"] == betas
    for i, (x, it, discr, times, none) in enumerate(info["candidates"]):
        fx = target[i]
        assert it == int(fx["iters"]), (i, it, int(fx["iters"]))
        assert rel(x, fx["x"]) < SOLVE_RTOL, (i, rel(x, fx["x"]))
        np.testing.assert_allclose(discr, fx["discr"], rtol=1e-7)
    best = int(np.argmin([-np.max(c[0]) for c in info["candidates"]]))
    assert info["best_beta"] == betas[best] and info["best"] == best
    # the application's final solve with the best beta repeats that
    # candidate's run (the reference is deterministic): the candidate is returned
    assert final is info["candidates"][best]
    x, it, discr, _, _ = final
    fx = target[best]
    assert it == int(fx["iters"]) and rel(x, fx["x"]) < SOLVE_RTOL


def test_argmin_strict_is_the_applications_choice(sgpmod):
    """application_sgp_subdivisions.py:78-99: running minimum from +inf with a
    strict '<': first of equal scores, NaN never chosen, None if all NaN."""
    a = sgpmod.argmin_strict
    assert a([0.3, 0.1, 0.1, 0.2]) == 1
    assert a([np.nan, 0.5, np.nan, 0.4]) == 3
    assert a([np.nan, np.nan]) is None
    assert a([np.inf, np.inf]) is None


# ------------------------------------------ float32 images in the batched path
def _app_batch_inputs(names):
    cases = [app_case(n) for n in names]
    gn = cases[0][0]
    assert all(np.array_equal(c[0], gn) for c in cases)
    return cases


@pytest.mark.parametrize("names", [["app_beta0", "app_beta1", "app_beta2", "app_beta3",
                                    "app_beta4"], ["app_beta2_flux32"], ["app_crop_beta"]])
def test_batch_float32_images_match_reference_and_dropin(sgpmod, monkeypatch, names):
    """The application's float32 FITS subdivision (and its non-contiguous crop,
    and the float32 flux) through sgp_betaDiv_batch: the float32 prelude runs
    on the device per image (include/bsgp.h gn_f32, ABI 3).  Every image
    matches its reference run at the application tolerances, and is bitwise
    equal to the single-image drop-in at the same team size."""
    cases = _app_batch_inputs(names)
    gn, psf, bkg, kw, fn, _ = cases[0]
    kw = dict(kw)
    kw.pop("betaParam", None)
    flux = kw.pop("flux")
    betas = [c[3]["betaParam"] for c in cases]
    gns = np.stack([gn] * len(cases))  # float32 (big-endian) batch
    assert gns.dtype.itemsize == 4
    out = sgpmod.sgp_betaDiv_batch(gns, psf, bkg, betaParams=betas, flux=flux, team=1, **kw)
    monkeypatch.setattr(sgpmod, "TEAM_DEFAULT", 1)
    for i, (g, p, b, k, f, fx) in enumerate(cases):
        it = int(out["iters"][i])
        assert it == int(fx["iters"]), (names[i], it, int(fx["iters"]))
        assert rel(out["x"][i], fx["x"]) < SOLVE_RTOL, (names[i], rel(out["x"][i], fx["x"]))
        np.testing.assert_allclose(out["discr"][i, :it + 1], fx["discr"], rtol=1e-7)
        x1, it1, d1, _, _ = sgpmod.sgp_betaDiv(g, p, b, **k)
        assert it1 == it
        np.testing.assert_array_equal(x1, out["x"][i])
        np.testing.assert_array_equal(d1, out["discr"][i, :it + 1])


def test_subdivisions_float32_field_matches_reference(sgpmod):
    """sgp_subdivisions on the application's float32 field, cut as one
    375x375 subdivision: the tile chain keeps the float32 arithmetic and
    reproduces the reference's run (ref_app_beta0)."""
    import subdivisions
    gn, psf, bkg, kw, fn, fx = app_case("app_beta0")
    kw = dict(kw)
    b0 = kw.pop("betaParam")
    mosaic, foot, out = subdivisions.sgp_subdivisions(gn, psf, bkg, subdiv_shape=(375, 375),
                                                      overlap=0, betaParams=[b0], team=1, **kw)
    assert np.all(foot == 1)
    assert int(out["iters"][0]) == int(fx["iters"])
    assert rel(mosaic, fx["x"]) < SOLVE_RTOL, rel(mosaic, fx["x"])
    it = int(fx["iters"])
    np.testing.assert_allclose(out["discr"][0, :it + 1], fx["discr"], rtol=1e-7)


def test_subdivisions_multistart_tile_x_beta(sgpmod):
    """(tile x beta) product in one launch with a per-tile strict argmin: each
    tile's chosen candidate equals that tile solved alone with that beta, and
    the mosaic is co-added from the chosen candidates."""
    import subdivisions
    gn, psf, bkg, kw, fn, _ = app_case("app_beta0")
    kw = dict(kw)
    kw.pop("betaParam")
    kw.pop("flux")
    kw["MAXIT"] = 12
    betas = sgpmod.app_beta_candidates()

    def score(x, tile):  # any function of the candidate and its tile
        return float(np.abs(x - tile).sum())

    field = np.ascontiguousarray(gn[:300, :300])
    bmap = bkg[:300, :300]
    mosaic, foot, info = subdivisions.sgp_subdivisions_multistart(
        field, psf, bmap, betas=betas, score=score, subdiv_shape=(160, 160), overlap=20, team=1,
        **kw)
    boxes = info["boxes"]
    assert info["scores"].shape == (len(boxes), 5)
    np.testing.assert_array_equal(info["best"], np.argmin(info["scores"], axis=1))
    for t, (x0, y0, x1, y1) in enumerate(boxes):
        k = int(info["best"][t])
        one = sgpmod.sgp_betaDiv_batch(field[None, y0:y1, x0:x1], psf, bmap[y0:y1, x0:x1],
                                       betaParams=[betas[k]], team=1, **kw)
        np.testing.assert_array_equal(one["x"][0], info["x"][t])
    ref_m, ref_f, _ = subdivisions.sgp_subdivisions(field, psf, bmap, subdiv_shape=(160, 160),
                                                    overlap=20, betaParams=info["best_beta"],
                                                    team=1, **kw)
    np.testing.assert_array_equal(foot, ref_f)
    np.testing.assert_array_equal(mosaic, ref_m)


def test_errflag_and_save_match_reference(sgpmod, tmp_path, monkeypatch):
    """sgp(errflag=True, obj, save=True): the err array with the reference's
    layout (err[1] == 0, the last iteration's error dropped) and every FITS
    file of SGP_reconstructed_images/ (orig, rec_k, res_k); sgp_betaDiv with
    save=True (it ignores errflag)."""
    import fits_io
    fx = golden("ref_errsave.npz")
    monkeypatch.chdir(tmp_path)
    for tag in ("kl", "beta"):
        kw = ref_kwargs({"kwargs": fx[f"{tag}_kwargs"]})
        if tag == "kl":
            kw["obj"] = fx["obj"]
        x, it, discr, _, err = getattr(sgpmod, str(fx[f"{tag}_fn"]))(
            fx["gn"], fx["psf"], np.float64(100.0), **kw)
        assert it == int(fx[f"{tag}_iters"])
        assert rel(x, fx[f"{tag}_x"]) < SOLVE_RTOL
        np.testing.assert_allclose(discr, fx[f"{tag}_discr"], rtol=1e-7)
        if tag == "kl":
            e = fx["kl_err"]
            assert len(err) == len(e) == it + 1 and err[1] == 0.0
            np.testing.assert_allclose(err, e, rtol=1e-7)
        else:
            assert err is None
        files = sorted(os.path.join("SGP_reconstructed_images", f)
                       for f in os.listdir("SGP_reconstructed_images"))
        assert [os.path.normpath(f) for f in files] == [os.path.normpath(str(f))
                                                        for f in fx[f"{tag}_files"]]
        for f in files:
            key = os.path.basename(f).replace(".fits", "")
            _, data = fits_io.read_fits(f)
            ref = fx[f"{tag}_{key}"]
            fin = np.isfinite(ref)
            assert np.array_equal(fin, np.isfinite(data)), key
            if key.startswith("res_"):
                # (x - gn)/sqrt(x): pixels the projection left at ~1e-13 carry
                # no relative accuracy there; compare where x is significant
                xr = fx[f"{tag}_rec_{key[4:]}"]
                fin &= xr > 1e-9 * xr.max()
            scale = np.abs(ref[fin]).max()
            assert np.max(np.abs(data[fin] - ref[fin])) <= 1e-7 * scale, key
        for f in files:
            os.remove(f)
        os.rmdir("SGP_reconstructed_images")


def test_batch_background_shapes(sgpmod):
    """A batch takes one [H, W] (or [1, H, W]) background map for every image,
    like [B, H, W] copies of it; other shapes raise."""
    fx = golden("ref_lin64_beta_bmap.npz")
    gns = np.stack([fx["gn"].astype(np.float64)] * 3)
    kw = dict(init_recon=2, proj_type=1, stop_criterion=1, MAXIT=5, alpha=10.0,
              ccd_sat_level=65000.0, use_original_SGP_Afunction=False, betaParams=0.97)
    full = sgpmod.sgp_betaDiv_batch(gns, fx["psf"], np.stack([fx["bkg"]] * 3), team=1, **kw)
    for b in (fx["bkg"], fx["bkg"][None]):
        out = sgpmod.sgp_betaDiv_batch(gns, fx["psf"], b, team=1, **kw)
        np.testing.assert_array_equal(out["x"], full["x"])
    with pytest.raises(ValueError):
        sgpmod.sgp_betaDiv_batch(gns, fx["psf"], np.ones(5), **kw)


def test_line_search_beyond_64_trials_matches_oracle(sgpmod):
    """A backtracking factor of 0.7 needs up to 79 trials before lam < 1e-12
    forces acceptance (sgp.py:336); the device follows the oracle."""
    import sgp_oracle
    fx = golden("ref_lin64_beta.npz")
    kw = ref_kwargs(fx)
    kw.update(beta=0.7, MAXIT=25)
    gn = fx["gn"].astype(np.float64)
    st = {}
    xo, ito, do, _, _ = sgp_oracle.sgp_betaDiv(gn, fx["psf"], np.float64(100.0), stats=st, **kw)
    x, it, d, _, _ = sgpmod.sgp_betaDiv(gn, fx["psf"], np.float64(100.0), **kw)
    assert it == ito
    assert rel(x, xo) < SOLVE_RTOL, rel(x, xo)
    np.testing.assert_allclose(d, do, rtol=1e-7)


@pytest.mark.parametrize("persistent", [0, 1])
def test_no_positive_scaling_bound_raises_like_reference(sgpmod, persistent):
    """flux = -bkg/2 makes flux/(flux+bkg) = -1, so y = -AT(gn) has no positive
    entry and the reference's np.min(y[y > 0]) raises ValueError (sgp.py:269-270
    / 711-712) before the first iteration: the oracle raises the same and the
    drop-in raises ValueError; in a batch that image stops at the setup
    (iters 0, status bit 8) while the others solve as they do alone (phase
    kernels and the persistent solver)."""
    import sgp_oracle
    fx = golden("ref_lin64_beta.npz")
    kw = ref_kwargs(fx)
    kw.update(MAXIT=10)
    gn = fx["gn"].astype(np.float64)
    with pytest.raises(ValueError):
        sgp_oracle.sgp_betaDiv(gn, fx["psf"], np.float64(100.0), flux=-50.0, **kw)
    with pytest.raises(ValueError, match="zero-size array"):
        sgpmod.sgp_betaDiv(gn, fx["psf"], np.float64(100.0), flux=-50.0, **kw)
    b = kw.pop("betaParam")
    f0 = float(np.sum(gn - 100.0))
    gns = np.stack([gn] * 3)
    flux = np.array([f0, -50.0, f0])
    with pytest.raises(ValueError, match=r"image\(s\) \[1\]"):
        sgpmod.sgp_betaDiv_batch(gns, fx["psf"], 100.0, flux=flux, team=1,
                                 persistent=persistent, betaParams=[b] * 3, **kw)
    out = sgpmod.sgp_betaDiv_batch(gns, fx["psf"], 100.0, flux=flux, team=1, persistent=persistent,
                                   betaParams=[b] * 3, device_out=True, **kw)
    cnt = out["counters"].cpu().numpy()
    iters = out["iters"].cpu().numpy()
    assert iters[1] == 0 and cnt[1, 3] == 8 and cnt[1, 0] == 0
    one = sgpmod.sgp_betaDiv_batch(gn[None], fx["psf"], 100.0, flux=np.array([f0]), team=1,
                                   persistent=persistent, betaParams=[b], **kw)
    for i in (0, 2):
        assert iters[i] == one["iters"][0] and cnt[i, 3] == 0
        np.testing.assert_array_equal(out["x"][i].cpu().numpy(), one["x"][0])


def test_float32_psf_accepted_by_batch_like_dropin(sgpmod, monkeypatch):
    """A float32 PSF normalised in float32 (float32 sum exactly 1, float64 sum
    off by more than 1e4*eps) passes the reference's check (sgp.py:97-102 sums
    in the PSF's dtype): the single-image drop-in and the batch API accept it
    alike and give the same bits (the batch had summed a float64
    copy and refused it)."""
    from test_abi import _f32_psf_sum_exact
    fx = golden("ref_lin64_beta.npz")
    kw = ref_kwargs(fx)
    kw.update(MAXIT=8)
    gn = fx["gn"].astype(np.float64)
    p = _f32_psf_sum_exact(1)
    monkeypatch.setattr(sgpmod, "TEAM_DEFAULT", 1)  # the batch's team size: the same bits
    x, it, _, _, _ = sgpmod.sgp_betaDiv(gn, p, np.float64(100.0), **kw)
    b = kw.pop("betaParam")
    out = sgpmod.sgp_betaDiv_batch(gn[None], p, 100.0, betaParams=[b], team=1, **kw)
    assert int(out["iters"][0]) == it
    np.testing.assert_array_equal(out["x"][0], x)
    with pytest.raises(ValueError, match="not normalized"):
        sgpmod.sgp_betaDiv_batch(gn[None], p.astype(np.float64), 100.0, betaParams=[b], **kw)
