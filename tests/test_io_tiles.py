"""Subdivision tiling/mosaic and FITS I/O.

CPU: the box calculation (product and oracle) against the reference's own
calculate_slice_bboxes (restoration/utils.py:332-372), the oracle cutouts
against astropy Cutout2D, the FITS reader against astropy on the reference's
data files, and the writer byte for byte against those files.
GPU: tile extraction, co-add and the device FITS decode bit for bit against
the oracle / host reader, and the whole subdivision chain against the oracle
solving every tile on the CPU."""
import hashlib
import os

import numpy as np
import pytest

from conftest import GOLDEN, golden

import fits_io
import subdivisions
import tiles_oracle


def _cases():
    z = golden("ref_slice_bboxes.npz")
    n = len([k for k in z if k.startswith("case")])
    return [(z[f"case{i}"], z[f"boxes{i}"]) for i in range(n)]


@pytest.mark.parametrize("fn", [subdivisions.calculate_slice_bboxes,
                                tiles_oracle.calculate_slice_bboxes])
def test_slice_bboxes_match_reference(fn):
    for case, boxes in _cases():
        H, W, sh, sw, ov = (int(v) for v in case)
        got = np.array(fn(H, W, sh, sw, ov / sh, ov / sw), dtype=np.int32)
        np.testing.assert_array_equal(got, boxes)


def test_subdivision_boxes_round_overlap_like_reference():
    # 29/100*100 == 28.999999999999996: the reference's int() drops a pixel
    b = subdivisions.subdivision_boxes((600, 700), (100, 100), 29)
    assert b[1][0] == 100 - 28
    np.testing.assert_array_equal(b, _cases()[8][1])


def test_oracle_cutouts_match_astropy():
    z = golden("ref_cutouts.npz")
    np.testing.assert_array_equal(tiles_oracle.extract_tiles(z["img"], z["boxes"]), z["cutouts"])


def _native_sha(a):
    return hashlib.sha256(np.asarray(a, dtype=np.float64).tobytes()).hexdigest()


@pytest.mark.parametrize("tag", ["psf", "subdiv"])
def test_fits_reader_matches_astropy(tag):
    z = golden("ref_fits_io.npz")
    hdr, data = fits_io.read_fits(os.path.join(GOLDEN, str(z[f"{tag}_file"])))
    assert hdr["BITPIX"] == int(z[f"{tag}_bitpix"])
    assert data.shape == tuple(z[f"{tag}_shape"])
    assert _native_sha(data) == str(z[f"{tag}_sha256"])
    np.testing.assert_array_equal(np.asarray(data, dtype=np.float64)[0], z[f"{tag}_row0"])


@pytest.mark.parametrize("name", ["psfccfbrd210048_1_1_img.fits", "SUBDIV_ORIGIMG.fits"])
def test_fits_writer_reproduces_reference_files(name, tmp_path):
    src = os.path.join(GOLDEN, name)
    _, data = fits_io.read_fits(src)
    dst = tmp_path / name
    fits_io.write_fits(str(dst), data)
    assert open(dst, "rb").read() == open(src, "rb").read()


def test_fits_scaled_integer_roundtrip(tmp_path):
    a = (np.arange(12, dtype=np.int16) - 6).reshape(3, 4)
    p = tmp_path / "i16.fits"
    fits_io.write_fits(str(p), a)
    hdr, b = fits_io.read_fits(str(p))
    assert hdr["BITPIX"] == 16 and b.dtype == np.int16
    np.testing.assert_array_equal(a, b)


# ------------------------------------------------------------------- GPU
@pytest.mark.gpu
def test_extract_and_coadd_bitwise_vs_oracle():
    rng = np.random.default_rng(11)
    img = rng.normal(100, 5, (700, 900))
    boxes = subdivisions.subdivision_boxes(img.shape, (256, 256), 40)
    tiles = subdivisions.extract_tiles(img, boxes, (256, 256)).cpu().numpy()
    np.testing.assert_array_equal(tiles, tiles_oracle.extract_tiles(img, boxes))
    tiles2 = tiles * rng.uniform(0.9, 1.1, tiles.shape)
    mean, foot = subdivisions.coadd_tiles(tiles2, boxes, img.shape)
    m_ref, c_ref = tiles_oracle.coadd_mean(tiles2, boxes, img.shape)
    np.testing.assert_array_equal(mean.cpu().numpy(), m_ref)
    np.testing.assert_array_equal(foot.cpu().numpy(), c_ref)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["psfccfbrd210048_1_1_img.fits", "SUBDIV_ORIGIMG.fits"])
def test_fits_device_decode_bitwise(name):
    src = os.path.join(GOLDEN, name)
    _, host = fits_io.read_fits(src)
    _, dev = fits_io.read_fits_device(src)
    np.testing.assert_array_equal(dev.cpu().numpy(), np.asarray(host, dtype=np.float64))


@pytest.mark.gpu
def test_fits_device_decode_integer_bscale(tmp_path):
    rng = np.random.default_rng(2)
    for dt in (np.uint8, np.int16, np.int32, np.int64):
        a = rng.integers(0, 120, (33, 17)).astype(dt)
        p = tmp_path / f"{np.dtype(dt).name}.fits"
        fits_io.write_fits(str(p), a, overwrite=True)
        # add BSCALE/BZERO cards by rewriting the header in place
        raw = bytearray(open(p, "rb").read())
        end = raw.find(b"END" + b" " * 77)
        cards = (b"BSCALE  = " + b"0.5".rjust(20)).ljust(80) + \
                (b"BZERO   = " + b"32768.0".rjust(20)).ljust(80)
        raw[end:end + 240] = cards + b"END".ljust(80)  # same header length
        open(p, "wb").write(bytes(raw))
        hdr, host = fits_io.read_fits(str(p))
        _, dev = fits_io.read_fits_device(str(p))
        np.testing.assert_array_equal(host, 32768.0 + 0.5 * a.astype(np.float64))
        np.testing.assert_array_equal(dev.cpu().numpy(), host)


@pytest.mark.gpu
def test_subdivision_chain_matches_oracle_per_tile():
    """Field -> 9 overlapping 256^2 subdivisions -> batched beta-SGP (linear A,
    projection) -> mean mosaic, against the numpy oracle solving each tile and
    co-adding on the CPU."""
    import cpu_bench
    import sgp_oracle
    rng = np.random.default_rng(4)
    field = np.zeros((600, 600))
    p = rng.integers(0, 600, (400, 2))
    np.add.at(field, (p[:, 0], p[:, 1]), rng.pareto(1.5, 400) * 1000 + 100)
    psf = cpu_bench.gaussian_psf(25)
    from scipy.signal import fftconvolve
    gn = rng.poisson(np.clip(fftconvolve(field, psf, mode="same"), 0, None) + 100.0).astype(float)
    kw = dict(init_recon=2, proj_type=1, stop_criterion=1, MAXIT=6, alpha=10.0,
              ccd_sat_level=65000.0, use_original_SGP_Afunction=False, schedule_lr=True,
              adapt_beta=False, betaParam=1.05, verbose=False)
    mosaic, foot, out = subdivisions.sgp_subdivisions(gn, psf, 100.0, (256, 256), 84, **kw)
    boxes = subdivisions.subdivision_boxes(gn.shape, (256, 256), 84)
    assert len(boxes) == 9
    ref = np.stack([sgp_oracle.sgp_betaDiv(t, psf, np.float64(100.0), **kw)[0]
                    for t in tiles_oracle.extract_tiles(gn, boxes)])
    rel = np.linalg.norm(out["x"] - ref) / np.linalg.norm(ref)
    assert rel < 1e-5, rel
    m_ref, c_ref = tiles_oracle.coadd_mean(ref, boxes, gn.shape)
    np.testing.assert_array_equal(foot, c_ref)
    assert np.linalg.norm(mosaic - m_ref) / np.linalg.norm(m_ref) < 1e-5


@pytest.mark.gpu
def test_subdivision_chain_with_spatial_psf_model():
    """Each 128^2 subdivision solved with the DIAPL model's stamp at its centre
    (bsgp_psf_stamps -> bsgp_plan_set_psfs), against the oracle solving every
    tile with the oracle's stamp for that centre."""
    import cpu_bench
    import psf_calculate
    import psf_oracle
    import sgp_oracle
    txt = os.path.join(GOLDEN, "psfccfbrd210048_1_1.bin.txt")
    model = psf_calculate.PSF(txt)
    rng = np.random.default_rng(6)
    field = np.zeros((300, 300))
    p = rng.integers(0, 300, (150, 2))
    np.add.at(field, (p[:, 0], p[:, 1]), rng.pareto(1.5, 150) * 1000 + 100)
    from scipy.signal import fftconvolve
    gn = rng.poisson(np.clip(fftconvolve(field, cpu_bench.gaussian_psf(31), mode="same"), 0, None)
                     + 100.0).astype(float)
    kw = dict(init_recon=2, proj_type=1, stop_criterion=1, MAXIT=5, alpha=10.0,
              ccd_sat_level=65000.0, use_original_SGP_Afunction=False, schedule_lr=True,
              adapt_beta=False, betaParam=1.05, verbose=False)
    mosaic, foot, out = subdivisions.sgp_subdivisions(gn, model, 100.0, (128, 128), 40, **kw)
    boxes = subdivisions.subdivision_boxes(gn.shape, (128, 128), 40)
    hdr, coef = psf_oracle.read_model(txt)
    stamps = psf_oracle.spatial_stamps(hdr, coef, subdivisions.tile_centres(boxes))
    assert not np.allclose(stamps[0], stamps[-1])  # the PSF really varies over the field
    tiles = tiles_oracle.extract_tiles(gn, boxes)
    ref = np.stack([sgp_oracle.sgp_betaDiv(t, s, np.float64(100.0), **kw)[0]
                    for t, s in zip(tiles, stamps)])
    rel = np.linalg.norm(out["x"] - ref) / np.linalg.norm(ref)
    assert rel < 1e-5, rel
    m_ref, c_ref = tiles_oracle.coadd_mean(ref, boxes, gn.shape)
    np.testing.assert_array_equal(foot, c_ref)
    assert np.linalg.norm(mosaic - m_ref) / np.linalg.norm(m_ref) < 1e-5


def test_float32_field_needs_float64_background():
    """A float32 field with a float32 (or integer) background map raises
    before any tile is cut (the background's float32 share of the prelude
    would otherwise be lost in the float64 tiles); float64 maps and Python /
    float64 scalars pass (host-side guard, no GPU)."""
    import subdivisions
    with pytest.raises(ValueError, match="float64 backgrounds"):
        subdivisions._check_bkg_dtype(True, np.ones((8, 8), np.float32))
    with pytest.raises(ValueError, match="float64 backgrounds"):
        subdivisions._check_bkg_dtype(True, np.int32(3))
    subdivisions._check_bkg_dtype(True, np.ones((8, 8)))
    subdivisions._check_bkg_dtype(True, 100.0)
    subdivisions._check_bkg_dtype(False, np.ones((8, 8), np.float32))
