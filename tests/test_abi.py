"""CPU-side checks of the drop-in boundary: the C-ABI library loads and exports
every symbol include/bsgp.h declares; the Python drop-in modules import and
expose the reference's names with the reference's signatures; the product
path refuses to run without a GPU (no CPU fallback)."""
import inspect
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import PKG, ROOT

HEADER = os.path.join(ROOT, "include", "bsgp.h")
LIB = os.path.join(PKG, "libbsgp.so")


def header_functions():
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"^\w[\w\s\*]*?\b(bsgp_\w+)\s*\(", txt, flags=re.M)))


def test_header_declares_entry_points():
    fns = header_functions()
    for f in ["bsgp_plan_create", "bsgp_solve_device", "bsgp_project_df", "bsgp_beta_div"]:
        assert f in fns


def test_library_exports_every_header_symbol():
    assert os.path.exists(LIB), "libbsgp.so not built (run __graft_entry__.build())"
    out = subprocess.run(["nm", "-D", "--defined-only", LIB], capture_output=True, text=True,
                         check=True).stdout
    exported = set(l.split()[-1] for l in out.splitlines() if l.strip())
    missing = [f for f in header_functions() if f not in exported]
    assert not missing, missing


def test_ctypes_load_and_version():
    import _bsgp
    L = _bsgp.lib()
    assert L.bsgp_abi_version() == 3
    for f in _bsgp.EXPORTED:
        assert hasattr(L, f)
    # argument validation runs on the host without a device
    h = __import__("ctypes").c_void_p()
    psf = np.ones((3, 3)) / 9.0
    rc = L.bsgp_plan_create(8, 8, psf.ctypes.data, 3, 3, 0, 0, 0, __import__("ctypes").byref(h))
    assert rc == -1 and b"psf.shape" in L.bsgp_last_error()
    bad = np.ones((8, 8))
    rc = L.bsgp_plan_create(8, 8, bad.ctypes.data, 8, 8, 0, 0, 0, __import__("ctypes").byref(h))
    assert rc == -4 and b"normalized" in L.bsgp_last_error()
    rc = L.bsgp_plan_create(8, 8, psf.ctypes.data, 3, 3, 1, 7, 0, __import__("ctypes").byref(h))
    assert rc == -1 and b"storage" in L.bsgp_last_error()


def test_dropin_signatures_match_reference():
    import flux_conserve_proj as fcp
    import sgp
    s = inspect.signature(sgp.sgp)
    assert list(s.parameters)[:8] == ["gn", "psf", "bkg", "init_recon", "proj_type",
                                      "stop_criterion", "MAXIT", "gamma"]
    assert s.parameters["alpha"].default == 1.3 and s.parameters["MAXIT"].default == 500
    assert s.parameters["use_original_SGP_Afunction"].default is True
    b = inspect.signature(sgp.sgp_betaDiv)
    names = list(b.parameters)
    # beta kwargs sit after errflag and before tol_convergence (sgp.py:510-512)
    assert names.index("adapt_beta") == names.index("errflag") + 1
    assert names[-2:] == ["tol_convergence", "use_original_SGP_Afunction"]
    assert b.parameters["betaParam"].default == 1.005 and b.parameters["adapt_beta"].default is True
    assert sgp.DEFAULT_PARAMS == (1000, 1e-4, 0.4, 1e-5, 1e5, 1e1, 3, 0.5, 1)
    assert len(sgp.DEFAULT_COLUMNS) == 20
    p = inspect.signature(fcp.projectDF)
    assert list(p.parameters) == ["b", "c", "dia", "scaling", "ccd_sat_level", "lambda_",
                                  "dlambda_", "tol_lam", "biter", "siter", "max_projs"]
    assert fcp.EPSILON == np.finfo(float).eps


def test_dropin_errors_like_reference():
    import sgp
    gn = np.ones((8, 8))
    with pytest.raises(ValueError, match="PSF is not normalized"):
        sgp.sgp(gn, np.ones((8, 8)), np.float64(1.0))
    with pytest.raises(ValueError, match="errflag"):
        sgp.sgp(gn, np.ones((8, 8)) / 64, np.float64(1.0), errflag=True)
    # sgp_betaDiv never checks errflag/obj (sgp.py:506-895 has no err path): the
    # call goes on to the device, which is absent here
    import _bsgp
    if not (_bsgp.torch is not None and _bsgp.torch.cuda.is_available()):
        with pytest.raises(_bsgp.BsgpError):
            sgp.sgp_betaDiv(gn, np.ones((8, 8)) / 64, np.float64(1.0), errflag=True, MAXIT=2)
    assert sgp.lr_schedule(1e-3, 0.1, 3) == pytest.approx(1e-3 * np.exp(-0.3))
    assert sgp.betaDivDeriv(gn, gn, 1) == 0 and sgp.betaDivDeriv(gn, gn, 0) == 0


def test_no_cpu_fallback_without_gpu():
    import _bsgp
    import sgp
    if _bsgp.torch is not None and _bsgp.torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    with pytest.raises(_bsgp.BsgpError):
        sgp.sgp(np.ones((8, 8)), np.ones((8, 8)) / 64, np.float64(1.0), MAXIT=2)
    with pytest.raises(_bsgp.BsgpError):
        sgp.betaDiv(np.ones(4), np.ones(4), 1.5)


def test_product_never_imports_oracle():
    for fn in os.listdir(PKG):
        if fn.endswith(".py"):
            assert "sgp_oracle" not in open(os.path.join(PKG, fn)).read(), fn


def test_check_status_raises_on_status_bits():
    """counters[:, 3]: bit 4 (team barrier timed out) and bit 1 (line search
    cap, only for a backtracking factor outside (0, 1)) are errors."""
    import _bsgp
    c = np.zeros((3, 8), np.int64)
    _bsgp.check_status(c)
    c[1, 3] = 4
    with pytest.raises(_bsgp.BsgpError, match="barrier"):
        _bsgp.check_status(c)
    c[1, 3] = 1
    with pytest.raises(_bsgp.BsgpError, match="line search"):
        _bsgp.check_status(c)
    c[1, 3] = 8  # no positive entry in the scaling bound: the reference's ValueError
    with pytest.raises(ValueError, match="zero-size array"):
        _bsgp.check_status(c)
    assert _bsgp.BSGP_ERR_HIP == -2 and _bsgp.BSGP_ERR_ARG == -1


def _f32_psf_sum_exact(seed):
    """A float32 PSF normalised in float32 whose float32 sum is exactly 1 while
    its float64 sum is not within the reference's 1e4*eps."""
    rng = np.random.default_rng(seed)
    for _ in range(200):
        p = rng.random((25, 25), dtype=np.float32)
        p = (p / np.sum(p)).astype(np.float32)
        if np.sum(p) == np.float32(1) and abs(np.sum(p.astype(np.float64)) - 1) > 1e4 * np.finfo(float).eps:
            return p
    pytest.skip("no such PSF found")


def test_shared_psf_checked_in_its_own_dtype():
    """The batch API checks a shared PSF as the reference does (sgp.py:97-102:
    np.sum in the PSF's own dtype), on the caller's array, once per content."""
    import _bsgp
    import sgp
    p = _f32_psf_sum_exact(0)
    calls = []

    def check(a):
        calls.append(a.dtype)
        sgp._check_psf(a)

    _bsgp.check_psf_once(p, check)        # float32 sum == 1: accepted
    _bsgp.check_psf_once(p.copy(), check)  # same bytes, same dtype: not re-run
    assert calls == [np.float32]
    with pytest.raises(ValueError, match="not normalized"):  # the float64 sum is off by >2e-12
        _bsgp.check_psf_once(p.astype(np.float64), check)
    bad = p.copy()
    bad[0, 0] += np.float32(1e-3)
    with pytest.raises(ValueError, match="not normalized"):
        _bsgp.check_psf_once(bad, check)
