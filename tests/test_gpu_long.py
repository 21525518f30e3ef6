"""The timed workload's own regime, pinned to the reference (SURVEY §8d C3:
256x256, 25x25 PSF, linear A, beta = 1.05, flux-conserving projection,
MAXIT = 100, stop rule 1; tests/golden/make_golden.py long).

From iteration ~40 on these solves stagnate: 20-32 line-search trials per
iteration, most of which the engine evaluates with its closed-form moment
series ("Line search") instead of the reference's direct pow
sums.  The reference's trials per iteration are recorded in the fixtures
(its betaDiv calls between two projectDF calls, sgp.py:763/782); the device
reports its own in bits 8..23 of flags (include/bsgp.h).  Checked on the
bench path (one workgroup per image, compact gn, projection pixel lists):
equal iteration counts, x within the north-star 1e-5, discrepancy rtol
1e-7, every non-stagnating iteration's trial count equal to the
reference's, and every stagnating one stagnating here too (the count inside
the stagnation regime follows rounding; conftest.compare_trials; the
mismatches are printed).
"""
import numpy as np
import pytest

from conftest import STAGNATION_TRIALS, compare_trials, golden, ref_kwargs

pytestmark = pytest.mark.gpu

LONG = ["c3long_s0", "c3long_s1", "c3long_s2"]


@pytest.fixture(scope="module")
def sgpmod():
    import _bsgp
    _bsgp.require_gpu()
    import sgp
    return sgp


def rel(a, b):
    return np.linalg.norm(np.asarray(a) - np.asarray(b)) / np.linalg.norm(np.asarray(b))


def trials_of(out, i):
    it = int(out["iters"][i])
    return (np.asarray(out["flags"][i, 1:it + 1]) >> 8).astype(np.int64)


# Seed 2's reference trajectory is itself unstable around iteration 55: the
# oracle (the reference's formulas under numpy 2 and another FFT, pinned to
# 1e-11 on seeds 0 and 1) parts from it there, ending 5.6e-5 away in x and
# 5.5e-6 in the discrepancy.  The reference itself, fed the image changed by
# one ulp per pixel (make_golden.py long_ens, 6 seeds), ends up to 0.73 away
# in x and 1.4e-2 in the discrepancy on that seed (8.9e-11 / 1.7e-11 on seeds
# 0 and 1).  That fixture is held to what a faithful restatement reaches,
# 1e-4 / 1e-5: far inside the reference's own rounding-level spread.
TOL = {"c3long_s2": (1e-4, 1e-5)}


def check_against(out, i, fx, what):
    it = int(out["iters"][i])
    assert it == int(fx["iters"]), (what, it, int(fx["iters"]))
    xt, dtol = TOL.get(what, (1e-5, 1e-7))
    r = rel(out["x"][i], fx["x"])
    assert r < xt, (what, r)
    np.testing.assert_allclose(out["discr"][i, :it + 1], fx["discr"], rtol=dtol, err_msg=what)
    diff = compare_trials(trials_of(out, i), fx["trials"], what)
    print(f"{what}: x rel {r:.2e}; stagnating iterations "
          f"({int(np.sum(fx['trials'] >= STAGNATION_TRIALS))}) with another trial count: "
          f"{len(diff)} {diff}")
    return r


def test_c3_maxit100_stagnation_matches_reference(sgpmod):
    fxs = [golden(f"ref_{n}.npz") for n in LONG]
    kw = ref_kwargs(fxs[0])
    assert kw["MAXIT"] == 100 and kw["stop_criterion"] == 1
    # the pinned window holds the stagnation regime the bench times
    assert all(int(np.sum(fx["trials"] >= 20)) >= 40 for fx in fxs)
    gns = np.stack([fx["gn"].astype(np.float64) for fx in fxs])
    out = sgpmod.sgp_betaDiv_batch(gns, fxs[0]["psf"], 100.0, team=1, **kw)
    assert np.all(out["counters"][:, 5] == 1) and np.all(out["counters"][:, 3] == 0)
    for i, (name, fx) in enumerate(zip(LONG, fxs)):
        check_against(out, i, fx, name)
        # most stagnating trials come from the series (the regime being pinned)
        assert out["counters"][i, 4] > 0.5 * np.sum(fx["trials"][fx["trials"] >= 20])
    # E_ls = the sum of the per-iteration counts
    for i in range(len(LONG)):
        assert out["counters"][i, 1] == trials_of(out, i).sum()


def test_c3_stop3_matches_reference(sgpmod):
    """The stop-3 (tol 1e-5) variant of the same workload (the
    application's own stop rule, application_sgp_subdivisions.py:87-90)."""
    fx = golden("ref_c3stop3_s0.npz")
    kw = ref_kwargs(fx)
    out = sgpmod.sgp_betaDiv_batch(fx["gn"].astype(np.float64)[None], fx["psf"], 100.0, team=1,
                                   **kw)
    check_against(out, 0, fx, "c3stop3_s0")


@pytest.mark.parametrize("team", [0, 4])
def test_c3_maxit100_team_solves(sgpmod, team):
    """The same 100-iteration run as a team solve (T workgroups per image,
    team reductions in another summation order): the same bar."""
    fx = golden("ref_c3long_s0.npz")
    kw = ref_kwargs(fx)
    out = sgpmod.sgp_betaDiv_batch(fx["gn"].astype(np.float64)[None], fx["psf"], 100.0, team=team,
                                   **kw)
    assert out["counters"][0, 5] > 1 and out["counters"][0, 3] == 0
    check_against(out, 0, fx, f"c3long_s0 team {int(out['counters'][0, 5])}")
