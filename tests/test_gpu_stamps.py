"""The star-stamp application path (application_sgp_star_stamps.py:56-105) on
the MI355X through the C ABI, against the reference's own runs
(tests/golden/make_golden.py stamps): 31x31 float32 cutouts of
results/SUBDIV_ORIGIMG.fits around 8 bright stars, the 31x31 DIAPL PSF with
the default circular A (odd-size fftshift), adaptive beta, stop rule 3, the
application's five seeds -- 40 solves.

Adaptive beta on a float32 image re-sums s*gn**beta in float32 at every
trial and rounds the float32 terms of betaDivDeriv to float32 (numpy 1.x;
include/bsgp.h gn_f32): the device reproduces both with correctly rounded
float32 power and log, where the reference's numpy uses its own vectorised
float32 power/log (not correctly rounded).  Two bars:

* against the oracle with correctly rounded float32 power/log
  (conftest.stamp_oracle_cr, the device's arithmetic): every iteration --
  equal iteration and line-search trial counts, discrepancy at rtol 1e-6,
  x within 1e-5, final beta within 1e-10 -- except that at most
  MAX_PARTED_CR runs may part in their last 5 iterations (float64
  rounding of the FFT and sums flips a stagnating Armijo test);
* against the reference (conftest.stamp_parity): the discrepancy up to the
  first iteration whose trial count differs, and x / final beta where all
  trial counts agree.  The runs that part from the reference are exactly the
  runs in which that oracle parts from it (12 of 40: an ulp of numpy's float32
  power flips a late line-search test; the oracle with numpy's own power
  parts in 1).
"""
import numpy as np
import pytest

from conftest import konst_ulp_discr, stamp_case, stamp_matches_cr, stamp_oracle_cr, stamp_parity

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def sgpmod():
    import _bsgp
    _bsgp.require_gpu()
    import sgp
    return sgp


def trials_of(out, i, it):
    return (np.asarray(out["flags"][i, 1:it + 1]) >> 8).astype(np.int64)


# runs allowed to part from the correctly rounded oracle late in the run
# (conftest.stamp_matches_cr: float64 FFT / summation-order rounding flips a
# late stagnating Armijo test)
MAX_PARTED_CR = 4


def check_run(j, i, x, it, discr, trials, beta, gn, ref, parted, worst, parted_cr):
    cr = stamp_oracle_cr(j, i)
    *w, p_cr = stamp_matches_cr(x, it, discr, trials, beta, cr)
    worst[:] = np.maximum(worst, w)
    ok, r, k = stamp_parity(x, it, discr, trials, beta, ref, atol=konst_ulp_discr(gn, beta))
    ok_cr = stamp_parity(cr["x"], cr["iters"], cr["discr"], cr["trials"], cr["beta"], ref,
                         atol=konst_ulp_discr(gn, cr["beta"]))[0]
    if p_cr:
        parted_cr.append((j, i, it, int(cr["iters"])))
    else:
        assert ok == ok_cr, (j, i)
    if not ok:
        parted.append((j, i, k, it, int(ref["iters"]), round(r, 6)))


def test_star_stamps_each_alone(sgpmod):
    """Each of the 40 runs as a one-image solve (automatic team size)."""
    parted, worst, parted_cr = [], np.zeros(3), []
    for j in range(8):
        for i in range(5):
            gn, psf, bkg, kw, ref = stamp_case(j, i)
            out = sgpmod.sgp_betaDiv_batch(gn[None], psf, bkg, betaParams=[kw.pop("betaParam")],
                                           **kw)
            it = int(out["iters"][0])
            check_run(j, i, out["x"][0], it, out["discr"][0, :it + 1], trials_of(out, 0, it),
                      float(out["beta_final"][0]), gn, ref, parted, worst, parted_cr)
    print("vs the correctly rounded oracle: worst x rel %.2e, discrepancy rel %.2e, beta rel %.2e"
          % tuple(worst))
    print("parted from the reference (star, seed, first differing iteration, iters, reference "
          "iters, x rel):", parted)
    print("parted late from the correctly rounded oracle (star, seed, iters, oracle iters):",
          parted_cr)
    assert len(parted) <= 12 + len(parted_cr), parted
    assert len(parted_cr) <= MAX_PARTED_CR, parted_cr


def test_star_stamps_batched_multistart(sgpmod, monkeypatch):
    """All 8 stars x 5 seeds in ONE batched launch (float32 images, per-image
    scalar backgrounds and fluxes): bitwise equal to the single-image
    drop-in at the same team size, and both bars."""
    cases = [stamp_case(j, i) for j in range(8) for i in range(5)]
    gns = np.stack([c[0] for c in cases])
    assert gns.dtype.itemsize == 4
    psf = cases[0][1]
    bkgs = np.array([c[2] for c in cases])
    flux = np.array([c[3]["flux"] for c in cases])
    betas = [c[3]["betaParam"] for c in cases]
    kw = {k: v for k, v in cases[0][3].items() if k not in ("flux", "betaParam")}
    out = sgpmod.sgp_betaDiv_batch(gns, psf, bkgs, betaParams=betas, flux=flux, team=1, **kw)
    monkeypatch.setattr(sgpmod, "TEAM_DEFAULT", 1)
    parted, worst, parted_cr = [], np.zeros(3), []
    for n, (gn, p, b, k, ref) in enumerate(cases):
        it = int(out["iters"][n])
        check_run(n // 5, n % 5, out["x"][n], it, out["discr"][n, :it + 1], trials_of(out, n, it),
                  float(out["beta_final"][n]), gn, ref, parted, worst, parted_cr)
        if n % 7 == 0:  # a sample against the single-image drop-in, bit for bit
            x1, it1, d1, _, _ = sgpmod.sgp_betaDiv(gn, p, b, **k)
            assert it1 == it
            np.testing.assert_array_equal(x1, out["x"][n])
            np.testing.assert_array_equal(d1, out["discr"][n, :it + 1])
    print("batched vs the correctly rounded oracle: worst x rel %.2e, discrepancy rel %.2e, "
          "beta rel %.2e" % tuple(worst))
    print("batched parted from the reference:", parted)
    print("parted late from the correctly rounded oracle (star, seed, iters, oracle iters):",
          parted_cr)
    assert len(parted) <= 12 + len(parted_cr), parted
    assert len(parted_cr) <= MAX_PARTED_CR, parted_cr
