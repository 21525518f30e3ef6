"""TEST INFRASTRUCTURE — pure-Python/numpy restatement of the DIAPL PSF model
(SURVEY §8f row 4), the checker for bsgp_psf_stamps / beta-sgp_amd/psf_calculate.py.
Only tests/, __graft_entry__.smoke() and bench.py's CPU leg use it; the product
never imports it.

Follows psf/psf_calculate.py: the coefficient file layout (:10-47), calc_psf_pix
(:52-87), get_psf_mat's pixel placement (:89-107), normalize_psf_mat (:129-137)
and the spatial expansion of init_psf (:140-165, restated as it is meant: the
reference's own version raises TypeError on ``[0.0] * ncomp`` with a float
ncomp and returns nothing).

Pinned by tests/golden/make_golden_psf.py (the reference's PSF class on its
coefficient file and on synthetic files) and by the reference's own output
psf/psfccfbrd210048_1_1_img.fits.  Spatial stamps away from (x_orig, y_orig)
have no reference vector (parity unpinned beyond this restatement).
"""
import numpy as np

LDEG = 2  # psf_calculate.py:24
SDEG = 1  # psf_calculate.py:25


def read_model(path_or_values):
    """(header dict, coefficient list) of a psf*.bin.txt file (:27-43)."""
    if isinstance(path_or_values, str):
        with open(path_or_values) as f:
            data = [float(l.rstrip("\n")) for l in f]
    else:
        data = [float(v) for v in path_or_values]
    hdr = dict(hw=int(data[0]), ndeg_spat=int(data[1]), ndeg_local=int(data[2]),
               ngauss=int(data[3]), recenter=data[4], cos=data[5], sin=data[6], ax=data[7],
               ay=data[8], sigma_inc=data[9], sigma_mscale=data[10], fitrad=data[11],
               x_orig=data[12], y_orig=data[13])
    return hdr, data[14:]


def calc_psf_pix(hdr, coeffs, x, y, ldeg=LDEG):
    """psf_calculate.py:52-87 (same operation order)."""
    x1 = hdr["cos"] * x - hdr["sin"] * y
    y1 = hdr["sin"] * x + hdr["cos"] * y
    rr = hdr["ax"] * x1 * x1 + hdr["ay"] * y1 * y1
    pix = 0.0
    icomp = 0
    for _ in range(hdr["ngauss"]):
        f = float(np.exp(rr))  # numpy's exp, as the reference
        a1 = 1.0
        for m in range(ldeg + 1):
            a2 = 1.0
            for _n in range(ldeg - m + 1):
                pix += float(coeffs[icomp]) * f * a1 * a2
                icomp += 1
                a2 *= y
            a1 *= x
        rr *= hdr["sigma_inc"] * hdr["sigma_inc"]
    return pix


def local_coeffs(hdr, coeffs, x, y, ldeg=LDEG, sdeg=SDEG):
    """init_psf's spatial expansion (:151-165) at field position (x, y)."""
    ncomp = hdr["ngauss"] * (ldeg + 1) * (ldeg + 2) // 2
    loc = [0.0] * ncomp
    itot = 0
    a1 = 1.0
    for m in range(sdeg + 1):
        a2 = 1.0
        for _n in range(sdeg - m + 1):
            for icomp in range(ncomp):
                loc[icomp] += coeffs[itot] * a1 * a2
                itot += 1
            a2 *= y - hdr["y_orig"]
        a1 *= x - hdr["x_orig"]
    return loc


def stamp(hdr, coeffs, normalize=False):
    """get_psf_mat (:89-107) / normalize_psf_mat (:129-137) for local
    coefficients `coeffs`; (2hw+1)^2 (31x31 for hw = 15, as the reference hard-codes)."""
    hw = hdr["hw"]
    S = 2 * hw + 1
    mat = np.zeros((S, S))
    for i in range(-hw, hw + 1):
        for j in range(-hw, hw + 1):
            mat[i + hw, j + hw] = calc_psf_pix(hdr, coeffs, j, i)
    if normalize:
        mat = mat / np.sum(mat)
    return mat


def spatial_stamps(hdr, coeffs, xy, normalize=True):
    return np.stack([stamp(hdr, local_coeffs(hdr, coeffs, x, y), normalize) for x, y in xy])
