"""Shared pytest setup: the `gpu` marker, paths to the drop-in package, the
oracle and the golden fixtures."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "beta-sgp_amd")
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (ROOT, PKG, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")


def golden(name):
    with np.load(os.path.join(GOLDEN, name), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def ref_kwargs(fx):
    """The kwargs dict stored (as a repr of plain literals) in a fixture."""
    import ast
    return ast.literal_eval(str(fx["kwargs"]))


@pytest.fixture(scope="session")
def ngc():
    d = golden("ngc7027_inputs.npz")
    return d["gn"], d["psf"], d["bg"][0][0], d["obj"]


STAGNATION_TRIALS = 20  # accepted step 0.4**19 ~ 3e-8: below the objective's rounding floor
STAGNATION_FLOOR = 16  # where the reference stagnates the other side accepts lam <= 0.4**15 ~ 1e-6


def compare_trials(dev, ref, what=""):
    """Line-search trials per iteration, engine (or oracle) vs the reference.

    An iteration whose accepted step lies above the objective's rounding
    floor (the reference needed fewer than STAGNATION_TRIALS trials) must
    take exactly the reference's trials.  In a stagnating iteration the
    Armijo test (sgp.py:784) compares f(lam) - fr ~ lam*gd ~ 1e-9*|gd| with
    differences at the rounding level of f, so which of the trials 20..32 is
    accepted depends on the last bits of the sums: the numpy restatement of
    the reference (oracle/sgp_oracle.py, same formulas, another FFT and
    numpy version) already differs from the reference there in 46 of 59 such
    iterations of c3long_s0 while its iterates agree to 6e-11.  There the
    other side must stagnate too (>= STAGNATION_FLOOR trials: an accepted
    step below 1e-6 of d).  Returns the 1-based stagnating iterations whose
    counts differ, so callers can report them."""
    dev = np.asarray(dev, dtype=np.int64)
    ref = np.asarray(ref, dtype=np.int64)
    assert dev.shape == ref.shape, (what, dev.shape, ref.shape)
    live = ref < STAGNATION_TRIALS
    bad = np.nonzero(live & (dev != ref))[0]
    assert bad.size == 0, (f"{what}: trials differ in non-stagnating iterations {list(bad + 1)}: "
                           f"got {list(dev[bad])}, reference {list(ref[bad])}")
    stag = ~live
    lost = np.nonzero(stag & (dev < STAGNATION_FLOOR))[0]
    assert lost.size == 0, (f"{what}: iterations {list(lost + 1)} stagnate in the reference "
                            f"({list(ref[lost])} trials) but not here ({list(dev[lost])})")
    return list(np.nonzero(stag & (dev != ref))[0] + 1)


# The float32 application fixtures exist in two sets, both made by running the
# unchanged reference (tests/golden/make_golden.py): "_libm" with numpy's SIMD
# float32 kernels disabled, so numpy's float32 ``**`` / ``np.log`` are the C
# library's powf / logf -- the device evaluates exactly those
# (bsgp_math.hpp libm_powf / libm_logf) -- and "" (numpy's default on this
# AVX-512 CPU: SVML, not correctly rounded; 20 % of float32 powers differ from
# libm's by an ulp).  The "_libm" set is the bar; the SVML set is checked up to
# that rounding (konst_shift, konst_ulp_discr).
LIBM = "_libm"
SVML = ""


def app_case(name, variant=LIBM):
    """Inputs + reference outputs of one application-path fixture
    (tests/golden/make_golden.py app): the raw big-endian float32 image as
    fits.getdata returns it (or the application's non-contiguous crop of a
    wider frame), the >f8 DIAPL PSF, the background map, the flux in the
    dtype the fixture was made with, and the application's kwargs."""
    fx = golden(f"ref_{name}{variant}.npz")
    kw = ref_kwargs(fx)
    sub = golden("app_subdiv_inputs.npz")
    if name.startswith("app_crop"):
        crop = golden("app_crop_inputs.npz")
        gn, bkg, flux = crop["wide"][:375, 75:], crop["bkg"], crop["flux"][()]
    else:
        gn, bkg, flux = sub["img"], sub["bkg"], sub["flux"][()]
    kw["flux"] = np.float32(flux) if str(fx["flux_dtype"]) == "float32" else np.float64(flux)
    return gn, sub["psf"], bkg, kw, str(fx["fn"]), fx


def crowded_case(name, variant=LIBM):
    """The application's CROWDED mode (make_golden.py crowded): the whole
    450x450 float32 frame results/CROWDED_SUBDIV_ORIGIMG.fits, its background
    map, the published flux, the application's kwargs (stop rule 3, tol 1e-5)
    -- inputs, and the reference's outputs of fixture set `variant`."""
    fx = golden(f"ref_{name}{variant}.npz")
    z = golden("crowded_inputs.npz")
    _, psf = __import__("fits_io").read_fits(os.path.join(GOLDEN, "psfccfbrd210048_1_1_img.fits"))
    kw = ref_kwargs(fx)
    kw["flux"] = np.float64(z["flux_beta"] if str(fx["fn"]) == "sgp_betaDiv" else z["flux_kl"])
    return z["img"], psf, z["bkg"], kw, str(fx["fn"]), fx


def satellite_case(name):
    """simulation_test_sgp.py's satellite runs (make_golden.py satellite):
    image, psf, background, ground truth, kwargs, function name, reference
    outputs (x, discr, rel_err and the FFT-swap spread of rel_err)."""
    d = golden("satellite_inputs.npz")
    fx = golden(f"ref_{name}.npz")
    return (d["gn"], d["psf"], d["bg"][0][0], d["obj"], ref_kwargs(fx), str(fx["fn"]), fx)


APP_CASES = ["app_beta0", "app_beta1", "app_beta2", "app_beta3", "app_beta4", "app_kl",
             "app_beta2_flux32", "app_crop_beta"]


def konst_shift(gn, kw, fx):
    """Discrepancy offset between the device and an SVML-set (variant "")
    float32-image reference run that comes only from numpy's float32 power.
    The beta objective's constant K = np.sum(s * gn**beta) is a float32 sum of
    float32 terms (sgp.py:458); numpy evaluates float32 ** on AVX-512 CPUs
    with SVML, while the device computes the C library's powf.  Both then sum
    in numpy's order (tests/test_oracle.py::test_numpy_f32_sum_model), so
    their K differ by at most an ulp or two of float32, and the discrepancy
    2/N*scaling*f by that constant.  Returns 2/N*scaling*(K_device -
    K_reference), K_device restated here with libm's powf; 0 for KL runs and
    for the "_libm" set (where it is 0 by construction: checked)."""
    if str(fx["fn"]) != "sgp_betaDiv" or "konst" not in fx:
        return 0.0
    import sgp_oracle
    g = np.asarray(gn).astype(np.float32).reshape(-1)
    sc = np.max(g)
    gs = g / sc
    b = float(kw["betaParam"])
    p = sgp_oracle._libm_call("bsgp_orc_powf", gs, __import__("ctypes").c_float(np.float32(b)))
    k_dev = np.sum(np.float32(1 / (b * (b - 1))) * p)
    return 2 / g.size * float(sc) * (float(k_dev) - float(fx["konst"]))


_STAMPS = {}


def stamp_case(j, i, variant=LIBM):
    """Inputs and reference outputs of one star-stamp run (make_golden.py
    stamps; application_sgp_star_stamps.py:56-105): the 31x31 float32 cutout,
    the >f8 DIAPL PSF, the float64 scalar background and flux, the kwargs with
    this seed's betaParam, and the reference's x / iters / discr / trials /
    final beta (fixture set `variant`, see LIBM)."""
    if variant not in _STAMPS:
        _STAMPS[variant] = golden(f"ref_stamps31{variant}.npz")
    z = _STAMPS[variant]
    import fits_io
    _, psf = fits_io.read_fits(os.path.join(GOLDEN, "psfccfbrd210048_1_1_img.fits"))
    kw = ref_kwargs(z)
    kw.update(flux=np.float64(z[f"flux{j}"]), betaParam=float(z["betas"][i]))
    ref = {k: z[f"{k}{j}_{i}"] for k in ("x", "iters", "discr", "trials", "beta")}
    return z[f"cut{j}"], psf, np.float64(z[f"bkg{j}"]), kw, ref


def stamp_kl_case(j, variant=LIBM):
    """Inputs and reference outputs of one KL star-stamp run (make_golden.py
    stamps_kl; application_sgp_star_stamps.py:107-112, the USE_BETADIV=False
    branch): the 31x31 float32 cutout, the >f8 DIAPL PSF, the float64 median
    background, the kwargs with the star's flux, and the reference's x / iters /
    discr / line-search trials per iteration (fixture set `variant`)."""
    key = "kl" + variant
    if key not in _STAMPS:
        _STAMPS[key] = golden(f"ref_stamps31_kl{variant}.npz")
    z = _STAMPS[key]
    import fits_io
    _, psf = fits_io.read_fits(os.path.join(GOLDEN, "psfccfbrd210048_1_1_img.fits"))
    kw = ref_kwargs(z)
    kw.update(flux=np.float64(z[f"flux{j}"]))
    ref = {k: z[f"{k}{j}"] for k in ("x", "iters", "discr", "trials")}
    return z[f"cut{j}"], psf, np.float64(z[f"bkg{j}"]), kw, ref


def stamp_kl_exact(x, it, discr, trials, ref, xtol=1e-5, drtol=1e-7):
    """The KL stamp bar: the reference's iteration count and its line-search
    trial count in every iteration, x within the north-star 1e-5, the
    discrepancy at rtol 1e-7 (no float32 power enters the KL objective)."""
    assert it == int(ref["iters"]), (it, int(ref["iters"]))
    np.testing.assert_array_equal(np.asarray(trials, dtype=np.int64),
                                  np.asarray(ref["trials"], dtype=np.int64))
    r = float(np.linalg.norm(x - ref["x"]) / np.linalg.norm(ref["x"]))
    assert r < xtol, r
    np.testing.assert_allclose(discr, ref["discr"], rtol=drtol)
    return r


def konst_ulp_discr(gn, beta, n_ulp=4):
    """Discrepancy change of n_ulp float32 ulps of K = sum(s*gn**beta) on a
    float32 image: numpy's float32 power is not correctly rounded (SVML), the
    device's is, so their K differ by an ulp now and then (conftest.konst_shift
    removes that offset exactly for fixed beta; with adaptive beta K is
    re-summed at every trial's beta, so it enters as a bound)."""
    g = np.asarray(gn, dtype=np.float32).reshape(-1)
    sc = float(np.max(g))
    gs = (g / np.float32(sc)).astype(np.float64)
    gs = np.where(gs > 0, gs, 0.0)
    k = abs(1 / (beta * (beta - 1))) * np.sum(gs ** beta)
    return 2.0 / g.size * sc * n_ulp * float(np.spacing(np.float32(k)))


def stamp_parity(x, it, discr, trials, beta, ref, atol=0.0):
    """The star-stamp bar against a reference run made with ANOTHER float32
    power (the SVML set).  These adaptive-beta float32 runs are chaotic near
    their end (stop rule 3 decides on a relative decrease of 1e-4, the
    float32 K = sum(s*gn**beta) is re-summed at every trial's beta): an ulp
    of numpy's vectorised float32 power can flip a late line-search test,
    after which the trajectories part.  Up to the first iteration whose trial
    count differs the discrepancy matches at rtol 1e-5 (plus `atol`:
    konst_ulp_discr); a run whose trial counts all agree must stop at the
    reference's iteration and reproduce x within the north-star 1e-5 and the
    final beta within 1e-7 (relative).  Returns (agreed, x rel, first
    differing iteration or None)."""
    rt = np.asarray(ref["trials"], dtype=np.int64)
    dt = np.asarray(trials, dtype=np.int64)
    m = min(len(rt), len(dt))
    bad = np.nonzero(dt[:m] != rt[:m])[0]
    k = int(bad[0]) if bad.size else m  # iterations 1..k agree in their trials
    np.testing.assert_allclose(discr[:k + 1], ref["discr"][:k + 1], rtol=1e-5, atol=atol)
    r = float(np.linalg.norm(x - ref["x"]) / np.linalg.norm(ref["x"]))
    if bad.size == 0 and it == int(ref["iters"]):
        assert r < 1e-5, r
        assert abs(beta - float(ref["beta"])) <= 1e-7 * abs(float(ref["beta"])), \
            (beta, float(ref["beta"]))
        return True, r, None
    return False, r, k + 1


_STAMP_ORC = {}


def stamp_oracle(j, i):
    """The oracle's run of star-stamp case (j, i) with the C library's float32
    power and log (sgp_oracle.LIBM_F32): the device's arithmetic, and the
    reference's under the "_libm" fixture setting."""
    if (j, i) not in _STAMP_ORC:
        import sgp_oracle as orc
        gn, psf, bkg, kw, _ = stamp_case(j, i)
        old, orc.LIBM_F32 = orc.LIBM_F32, True
        try:
            st = {}
            x, it, discr, _, _ = orc.sgp_betaDiv(gn, psf, bkg, stats=st, **kw)
        finally:
            orc.LIBM_F32 = old
        _STAMP_ORC[(j, i)] = dict(x=x, iters=int(it), discr=np.asarray(discr),
                                  trials=np.asarray(st["ls_trials"], dtype=np.int64),
                                  beta=float(st["beta"]))
    return _STAMP_ORC[(j, i)]


def stamp_exact(x, it, discr, trials, beta, ref, drtol=1e-5):
    """The star-stamp bar against a run with the same float32 arithmetic (the
    "_libm" reference set, or stamp_oracle): the same iteration count and
    line-search trial count in every iteration, x within the north-star 1e-5,
    the final beta within 1e-9 and the discrepancy at rtol `drtol` (the
    north-star 1e-5: star 0 / seed 1 amplifies last-bit differences of the
    float64 FFT and sums to 1e-6 in the discrepancy, 7e-6 in x).
    Returns None when the run meets it, else (first iteration whose trial count
    differs, iters, reference iters, x rel) -- a parting, which the caller
    must name -- after checking the discrepancy up to that iteration."""
    rt = np.asarray(ref["trials"], dtype=np.int64)
    dt = np.asarray(trials, dtype=np.int64)
    m = min(len(rt), len(dt))
    bad = np.nonzero(dt[:m] != rt[:m])[0]
    k = int(bad[0]) if bad.size else m  # iterations 1..k agree in their trials
    r = float(np.linalg.norm(x - ref["x"]) / np.linalg.norm(ref["x"]))
    np.testing.assert_allclose(discr[:k + 1], ref["discr"][:k + 1], rtol=drtol)
    if bad.size == 0 and it == int(ref["iters"]):
        assert r < 1e-5, r
        assert abs(beta / float(ref["beta"]) - 1) <= 1e-9, (beta, float(ref["beta"]))
        return None
    return (k + 1, int(it), int(ref["iters"]), round(r, 6))
