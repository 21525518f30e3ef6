"""Offline replay of the projection's first-pass bracket rules (analysis, not a
test; test infrastructure, so it may run the oracle).

The device evaluates projectDF's multiplier search (flux_conserve_proj.py:7-144)
with pixel lists (bsgp_kernels.hpp cached_projection): the first evaluation is
a full pass over the image that also splits the pixels for a bracket [qL, qU]
(pixels that change state inside it go to a list); an evaluation inside the
current bracket reads only the list, one outside is a full pass ("miss") that
splits for a new bracket.  The bracket never changes results, only the cost.
This script runs the oracle's sgp_betaDiv on a bench image, records every
projection's multiplier sequence (and the step length alpha it was called
at), and replays the sequences through the split / list / miss rules for the
first-pass bracket policies:

  guess30     the previous root +/- 30 % (rounds 2-5)
  alpha(w1,w2) alpha * (previous root / previous alpha) +/- w1, widened to
              cover kappa times that, +/- w2 (kappa: the previous search's first
              multiplier off the first pass over its root) -- round 6

    python tests/proj_bracket_replay.py c3 0      # C3 image 0 (bench generator), MAXIT 100
    python tests/proj_bracket_replay.py c4        # the 2048^2 field, MAXIT 24

Output: full passes and list entries read (in units of N) per projection.
"""
import contextlib
import io
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, ROOT)


def record(which, seed):
    """The oracle's solve with every projectDF evaluation's multiplier and
    each call's (y, X, flux, saturation) and alpha recorded."""
    import cpu_bench
    src = open(os.path.join(ROOT, "oracle", "sgp_oracle.py")).read()
    src = src.replace('''    def xof(lam):
        nev[0] += 1''', '''    def xof(lam):
        nev[0] += 1
        REC[-1]["lams"].append(float(lam))''')
    src = src.replace('''    x = xof(lambda_)  # :22-25''', '''    REC.append({"lams": [], "y": c / dia, "X": 1 / dia, "b": float(b),
                "sat": None if ccd_sat_level is None else ccd_sat_level / scaling - EPSILON})
    x = xof(lambda_)  # :22-25''')
    src = src.replace('''        y = x - alpha * np.multiply(X, g)\n''',
                      '''        y = x - alpha * np.multiply(X, g)\n        ALPHA.append(float(alpha))\n''')
    ns = {"__name__": "oracle_replay", "REC": [], "ALPHA": []}
    exec(compile(src, "sgp_oracle_replay", "exec"), ns)
    if which == "c3":
        gn, psf = cpu_bench.make_stamp(seed, 256, 25, 200, circular=False)
        kw = dict(MAXIT=100, use_original_SGP_Afunction=False)
    else:
        gn, psf = cpu_bench.make_stamp(0, 2048, 64, 5000, circular=True)
        kw = dict(MAXIT=24, use_original_SGP_Afunction=True)
    with contextlib.redirect_stdout(io.StringIO()):
        ns["sgp_betaDiv"](gn, psf, np.float64(100.0), init_recon=2, proj_type=1, stop_criterion=1,
                          alpha=10.0, ccd_sat_level=65000.0, schedule_lr=True, adapt_beta=False,
                          betaParam=1.05, lr=1e-3, lr_exp_param=0.1, **kw)
    rec = ns["REC"][1:]  # (the setup's projection has no history)
    for r, a in zip(rec, ns["ALPHA"]):
        r["alpha"] = a
    return rec


def n_list(y, X, sat, qL, qU):
    """Pixels whose x(lambda) changes state inside [qL, qU] (the list)."""
    vL, vU = np.maximum(0, y + qL * X), np.maximum(0, y + qU * X)
    if sat is not None:
        vL, vU = np.minimum(sat, vL), np.minimum(sat, vU)
    keep = (vU == 0.0) | ((vL > 0.0) & ((vU < sat) if sat is not None else True))
    if sat is not None:
        keep |= vL == sat
    return int(np.count_nonzero(~keep))


def replay(rec, policy):
    passes = lists = 0
    hist = {}
    for d in rec:
        y, X, sat, lams, b = d["y"], d["X"], d["sat"], d["lams"], d["b"]
        lam0, root = lams[0], lams[-1]
        qL, qU = policy(d, hist)
        passes += 1
        have = qL is not None
        cL, cU, nl = qL, qU, (n_list(y, X, sat, qL, qU) if qL is not None else 0)
        v0 = y + lam0 * X
        inside = (v0 > 0) & ((v0 < sat) if sat is not None else True)
        slope = X[inside].sum()
        S0 = np.maximum(0, v0)
        S0 = (np.minimum(sat, S0) if sat is not None else S0).sum()
        lamN = lam0 - (S0 - b) / slope if slope > 0 else np.nan
        first_miss, Lk, Uk, first = True, -np.inf, np.inf, None
        free = {lam0, lam0 - 1.0, lam0 + 1.0}
        for lam in lams[1:]:
            if lam in free:
                continue
            first = lam if first is None else first
            if have and cL <= lam <= cU:
                lists += nl
            else:
                passes += 1
                if first_miss and np.isfinite(lamN):
                    cL, cU, have = min(lam, lamN), max(lam, lamN), True
                elif np.isfinite(Lk) and np.isfinite(Uk):
                    cL, cU, have = min(Lk, Uk), max(Lk, Uk), True
                else:
                    have = False
                first_miss = False
                nl = n_list(y, X, sat, cL, cU) if have else 0
            v = np.maximum(0, y + lam * X)
            r = (np.minimum(sat, v) if sat is not None else v).sum() - b
            Lk = lam if (r < 0 and lam > Lk) else Lk
            Uk = lam if (r > 0 and lam < Uk) else Uk
        hist = {"root": root, "ratio": root / d["alpha"] if d["alpha"] else 0.0,
                "kappa": first / root if (first is not None and root) else 0.0}
    return passes / len(rec), lists / len(rec) / rec[0]["y"].size


def guess30(d, h):
    lp = h.get("root")
    if not lp:
        return None, None
    return lp - 0.3 * abs(lp), lp + 0.3 * abs(lp)


def alpha_policy(w1, w2):
    def pol(d, h):
        lh = d["alpha"] * h.get("ratio", 0.0)
        if not lh:
            return guess30(d, h)
        lo, hi = lh - w1 * abs(lh), lh + w1 * abs(lh)
        pk = h.get("kappa", 0.0) * lh
        if pk:
            lo, hi = min(lo, pk - w2 * abs(pk)), max(hi, pk + w2 * abs(pk))
        return lo, hi
    return pol


if __name__ == "__main__":
    which = sys.argv[1] if len(sys.argv) > 1 else "c3"
    seed = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    rec = record(which, seed)
    print(f"{which} seed {seed}: {len(rec)} projections of N = {rec[0]['y'].size}")
    for name, pol in [("guess30", guess30), ("alpha(0.1,0.2)", alpha_policy(0.1, 0.2)),
                      ("alpha(0.15,0.15)", alpha_policy(0.15, 0.15))]:
        p, l = replay(rec, pol)
        print(f"  {name:18s} full passes {p:.3f}  list reads {l:.4f} N  pass-equivalents {p + l:.3f}")
