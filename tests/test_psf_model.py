"""DIAPL PSF model on the device and per-image PSFs in the solver.

CPU: the oracle (oracle/psf_oracle.py) against the reference's PSF class
(tests/golden/ref_psf_model.npz, make_golden_psf.py) and against the
reference's own normalised stamp psf/psfccfbrd210048_1_1_img.fits; the
drop-in's file parsing.
GPU: bsgp_psf_stamps against the same vectors (exp() may differ by an ulp:
rtol 1e-14), spatial stamps against the oracle's expansion, and
bsgp_plan_set_psfs: a batch with per-image PSFs gives, image by image, the
bits of solving each image with its own plan."""
import os

import numpy as np
import pytest

from conftest import GOLDEN, golden

import fits_io
import psf_oracle

TXT = os.path.join(GOLDEN, "psfccfbrd210048_1_1.bin.txt")


def _atol(a):
    return 1e-15 * np.abs(a).max()


def _cases():
    z = golden("ref_psf_model.npz")
    n = len([k for k in z if k.startswith("file")])
    return [(z[f"file{i}"], z[f"raw{i}"], z[f"norm{i}"]) for i in range(n)]


def test_oracle_matches_reference_psf_class():
    for vals, raw, norm in _cases():
        hdr, coef = psf_oracle.read_model(vals)
        # exp() may differ by an ulp between numpy builds; pixels where the
        # local polynomial cancels carry that as a larger relative error
        np.testing.assert_allclose(psf_oracle.stamp(hdr, coef), raw, rtol=1e-14, atol=_atol(raw))
        np.testing.assert_allclose(psf_oracle.stamp(hdr, coef, True), norm, rtol=1e-14,
                                   atol=_atol(norm))


def test_oracle_matches_reference_fits_stamp():
    hdr, coef = psf_oracle.read_model(TXT)
    _, ref = fits_io.read_fits(os.path.join(GOLDEN, "psfccfbrd210048_1_1_img.fits"))
    np.testing.assert_allclose(psf_oracle.stamp(hdr, coef, True), ref, rtol=1e-14, atol=_atol(ref))


def test_oracle_spatial_expansion_at_origin_is_local_model():
    hdr, coef = psf_oracle.read_model(TXT)
    loc = psf_oracle.local_coeffs(hdr, coef, hdr["x_orig"], hdr["y_orig"])
    assert loc == list(coef[:12])


def test_dropin_parses_like_reference():
    import psf_calculate
    p = psf_calculate.PSF(TXT)
    vals = [float(l) for l in open(TXT)]
    assert (p.hw, p.ndeg_spat, p.ndeg_local, p.ngauss) == (15, 1, 2, 2)
    assert p.coeffs == vals[14:] and p.ntot == 36.0
    hdr, coef = psf_oracle.read_model(TXT)
    assert p.local_coeffs(300.0, 150.0) == psf_oracle.local_coeffs(hdr, coef, 300.0, 150.0)


# ------------------------------------------------------------------- GPU
@pytest.mark.gpu
def test_device_stamps_match_reference(tmp_path):
    import psf_calculate
    for i, (vals, raw, norm) in enumerate(_cases()):
        path = tmp_path / f"psf_case{i}.bin.txt"
        path.write_text("".join(f"{float(v)!r}\n" for v in vals))
        p = psf_calculate.PSF(str(path))
        np.testing.assert_allclose(p.get_psf_mat(), raw, rtol=1e-14, atol=_atol(raw))
        np.testing.assert_allclose(p.normalize_psf_mat(), norm, rtol=1e-14, atol=_atol(norm))
    _, ref = fits_io.read_fits(os.path.join(GOLDEN, "psfccfbrd210048_1_1_img.fits"))
    got = psf_calculate.PSF(TXT).normalize_psf_mat()
    np.testing.assert_allclose(got, ref, rtol=1e-14, atol=_atol(ref))
    print("bit-identical pixels vs the reference's FITS stamp:", int((got == ref).sum()), "/ 961")


@pytest.mark.gpu
def test_calc_psf_pix_matches_stamp():
    import psf_calculate
    p = psf_calculate.PSF(TXT)
    mat = p.get_psf_mat()
    for x, y in [(0, 0), (3, -2), (-15, 15), (7, 11)]:
        assert p.calc_psf_pix(p.coeffs, x, y) == mat[y + 15, x + 15]


@pytest.mark.gpu
def test_device_spatial_stamps_match_oracle():
    import psf_calculate
    p = psf_calculate.PSF(TXT)
    hdr, coef = psf_oracle.read_model(TXT)
    rng = np.random.default_rng(5)
    xy = np.concatenate([[[hdr["x_orig"], hdr["y_orig"]]], rng.uniform(0, 2048, (40, 2))])
    got = p.stamps(xy)
    ref = psf_oracle.spatial_stamps(hdr, coef, xy)
    np.testing.assert_allclose(got, ref, rtol=1e-13, atol=_atol(ref))
    # at the origin the spatial stamp is the reference's normalize_psf_mat
    np.testing.assert_array_equal(got[0], p.normalize_psf_mat())


def _stars(rng, n, k, nstar=60):
    import cpu_bench
    from scipy.signal import fftconvolve
    out = []
    for _ in range(n):
        f = np.zeros((96, 96))
        p = rng.integers(0, 96, (nstar, 2))
        np.add.at(f, (p[:, 0], p[:, 1]), rng.pareto(1.5, nstar) * 800 + 100)
        out.append(rng.poisson(np.clip(fftconvolve(f, cpu_bench.gaussian_psf(k), "same"), 0, None)
                               + 100.0).astype(float))
    return np.stack(out)


@pytest.mark.gpu
@pytest.mark.parametrize("linear", [True, False])
def test_per_image_psfs_match_single_image_solves(linear):
    """B images, B different PSFs in one batch == each image solved alone with its PSF
    (bitwise: the device placement reproduces the host's, and results are batch invariant)."""
    import psf_calculate
    import sgp
    rng = np.random.default_rng(9)
    gns = _stars(rng, 5, 31)
    p = psf_calculate.PSF(TXT)
    psfs = p.stamps(rng.uniform(0, 450, (5, 2)))
    if not linear:  # circular A needs psf.shape == image shape: embed the stamp
        big = np.zeros((5, 96, 96))
        big[:, 48 - 15:48 + 16, 48 - 15:48 + 16] = psfs
        psfs = big / big.sum(axis=(1, 2), keepdims=True)
    kw = dict(init_recon=2, proj_type=1, stop_criterion=1, MAXIT=12, alpha=10.0,
              ccd_sat_level=65000.0, use_original_SGP_Afunction=not linear, schedule_lr=True,
              adapt_beta=False, betaParam=1.05, verbose=False)
    out = sgp.sgp_betaDiv_batch(gns, psfs, 100.0, **kw)
    for i in range(5):
        one = sgp.sgp_betaDiv_batch(gns[i:i + 1], psfs[i], 100.0, **kw)
        np.testing.assert_array_equal(out["x"][i], one["x"][0])
        np.testing.assert_array_equal(out["discr"][i], one["discr"][0])
    # and the per-image plan differs from a shared PSF (the TFs are really per image)
    shared = sgp.sgp_betaDiv_batch(gns, psfs[0], 100.0, **kw)
    np.testing.assert_array_equal(shared["x"][0], out["x"][0])
    assert not np.array_equal(shared["x"][1], out["x"][1])


@pytest.mark.gpu
def test_per_image_psf_rejects_unnormalized_and_wrong_batch():
    import _bsgp
    import sgp
    rng = np.random.default_rng(1)
    gns = _stars(rng, 2, 15)
    import cpu_bench
    psfs = np.stack([cpu_bench.gaussian_psf(15)] * 2)
    bad = psfs.copy()
    bad[1] *= 1.01
    with pytest.raises(_bsgp.BsgpError, match="not normalized"):
        sgp.sgp_batch(gns, bad, 100.0, MAXIT=2, use_original_SGP_Afunction=False, verbose=False)
    with pytest.raises(ValueError, match="one PSF per image"):
        sgp.sgp_batch(gns, psfs[:1], 100.0, MAXIT=2, use_original_SGP_Afunction=False,
                      verbose=False)
