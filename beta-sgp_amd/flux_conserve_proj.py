"""Drop-in replacement for ``restoration/flux_conserve_proj.py``.

``projectDF`` keeps the reference signature (flux_conserve_proj.py:7) and
returns the same projected vector; the bracketing + secant search on the
multiplier runs in one workgroup on the MI355X (``bsgp_project_df`` in
include/bsgp.h), each x(lambda) evaluation being a fused clip + workgroup
reduction.  Inside ``sgp``/``sgp_betaDiv`` the projection never leaves the
solver kernel; this module serves direct callers.

Differences: the device caps the bracketing loop at 200000 evaluations where
the reference's ``while r < 0`` (flux_conserve_proj.py:38) never ends when
``b`` exceeds the saturation capacity; a plain float ``b`` is accepted.
"""
import numpy as np

import _bsgp as _B

EPSILON = np.finfo(float).eps  # flux_conserve_proj.py:5


def projectDF(b, c, dia, scaling, ccd_sat_level=None, lambda_=0, dlambda_=1, tol_lam=1e-11,
              biter=0, siter=0, max_projs=1000):
    """min 0.5 x'diag(dia)x - c'x  s.t. sum(x) = b, 0 <= x (<= sat/scaling - eps)."""
    _B.require_gpu()
    c = np.asarray(c)
    shape = c.shape
    cd = _B.to_dev(c.astype(np.float64, copy=False).ravel())
    dd = _B.to_dev(np.asarray(dia).astype(np.float64, copy=False).ravel())
    x, _ = _B.project_df_dev(np.float64(b), cd, dd, scaling, ccd_sat_level, lambda_, dlambda_,
                             tol_lam, biter, siter, max_projs)
    return x.cpu().numpy().reshape(shape)
