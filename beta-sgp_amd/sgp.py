"""Drop-in replacement for the hot path of ``restoration/sgp.py`` (Yash-10/beta-sgp).

Put ``beta-sgp_amd/`` on ``sys.path`` in place of ``restoration/`` and the
reference's callers keep working unchanged::

    from sgp import sgp, sgp_betaDiv, DEFAULT_PARAMS, DEFAULT_COLUMNS     # application_sgp_*.py:5,18
    from sgp import betaDiv, betaDivDeriv, betaDivDerivwrtY                # tests.py:1

Same names, argument order/meaning, return tuples and error behaviour as
sgp.py:41-47 (``sgp``) and sgp.py:506-513 (``sgp_betaDiv``); the iteration
itself runs on the MI355X through ``libbsgp.so`` (include/bsgp.h): one
persistent workgroup per image executes setup, every SGP iteration, the
flux-conserving projection, the Armijo line search, the Barzilai-Borwein
update and the stop rules on the device.  There is no CPU fallback: without
the library or a GPU every entry point raises ``_bsgp.BsgpError``.

Kept from the reference: ``sgp.log`` in the cwd with the same per-iteration
lines (sgp.py:104, 291-298, 351-352, 399-411), the final prints of
``sgp_betaDiv`` (sgp.py:892-893), ``ValueError`` for a non-normalised PSF
(sgp.py:97-102) and for ``errflag`` without ``obj`` (sgp.py:237-238), the
revert-to-previous-iterate on stop (sgp.py:424-425) and the returned tuple
``(x, iters, discr, times, None)``.

Deliberate differences: ``save=True`` (per-iteration FITS
dumps) and ``errflag=True`` raise ``NotImplementedError``; a plain Python
float ``bkg`` is accepted (the reference crashes on ``bkg.flatten()``).

Extra: :func:`sgp_betaDiv_batch` / :func:`sgp_batch` solve
many images or beta candidates in one launch.
"""
import logging
import math

import numpy as np

import _bsgp as _B

DEFAULT_PARAMS = (1000, 1e-4, 0.4, 1e-5, 1e5, 1e1, 3, 0.5, 1)  # sgp.py:34
DEFAULT_COLUMNS = ['label', 'xcentroid', 'ycentroid', 'sky_centroid',
                   'bbox_xmin', 'bbox_xmax', 'bbox_ymin', 'bbox_ymax',
                   'area', 'semimajor_sigma', 'semiminor_sigma',
                   'orientation', 'eccentricity', 'min_value', 'max_value',
                   'local_background', 'segment_flux', 'segment_fluxerr', 'ellipticity',
                   'fwhm']  # sgp.py:35-39

LS_SPEC_DEFAULT = 2  # line-search trial lambdas evaluated per pass over the data
LS_SERIES_DEFAULT = 1  # small line-search steps from the moment series (general beta)
STREAMS_DEFAULT = 3  # sub-batch streams of a batched solve (+ the caller's = 4 HW queues; 4 sub-streams collapse under the default GPU_MAX_HW_QUEUES=4)
TEAM_DEFAULT = 0  # workgroups per image: 0 = auto (spread small batches over the CUs)
PROJ_CACHE_DEFAULT = 1  # projectDF evaluations inside a known root bracket read a pixel list
GN_COMPACT_DEFAULT = 1  # f32-exact observed images stored in f32 (bit-identical results)


# ------------------------------------------------------------------ helpers
def _check_psf(psf):
    checkPSF = np.abs(np.sum(psf.flatten()) - 1.)
    tolCheckPSF = 1e4 * np.finfo(float).eps
    if checkPSF > tolCheckPSF:
        errmsg = f"\n\tsum(psf) - 1. = {checkPSF}, tolerance = {tolCheckPSF}"
        raise ValueError(f'PSF is not normalized! Provide a normalized PSF! {errmsg}')


def _bkg_kind(bkg, shape):
    b = np.asarray(bkg)
    if b.size == 1:
        return "scalar", b
    if b.size == int(np.prod(shape)):
        return "map", b.reshape(shape)
    raise ValueError(f"bkg of shape {b.shape} does not broadcast to the image shape {shape}")


def _prelude_host(gn, bkg, init_recon, flux, stop_criterion, scale_data):
    """sgp.py:166-199 in the input dtype (used for non-float64 images so the
    scaling rounds exactly like the reference's numpy code)."""
    if init_recon == 0:
        x = np.zeros_like(gn)
    elif init_recon == 1:
        np.random.seed(42)
        x = np.random.randn(*gn.shape)
    elif init_recon == 2:
        x = gn.copy()
    else:
        if flux is None:
            x = np.sum(gn - bkg) / gn.size * np.ones_like(gn)
        else:
            x = flux / gn.size * np.ones_like(gn)
    gn = gn.flatten()
    x = x.flatten()
    bkg = np.asarray(bkg).flatten()
    tol4 = 1 + 1 / np.mean(gn) if stop_criterion == 4 else 0.0
    if scale_data:
        scaling = np.max(gn)
        gn = gn / scaling
        bkg = bkg / scaling
        x = x / scaling
    else:
        scaling = 1.
    return gn, bkg, x, float(scaling), float(tol4)


def _params(variant, init_recon, proj_type, stop_criterion, MAXIT, gamma, beta, alpha, alpha_min,
            alpha_max, M_alpha, tau, M, max_projs, verbose, ccd_sat_level, scale_data,
            tol_convergence, adapt_beta=False, betaParam=1.005, lr=1e-3, lr_exp_param=0.1,
            schedule_lr=False, bkg_is_map=False, ls_spec=None, ls_series=None, streams=None,
            team=None, proj_cache=None, gn_compact=None):
    p = _B.Params()
    p.variant = variant
    p.init_recon = int(init_recon)
    p.proj_type = int(proj_type)
    p.stop_criterion = int(stop_criterion)
    p.MAXIT = int(MAXIT)
    p.M_alpha = int(M_alpha)
    p.M = int(M)
    p.max_projs = int(max_projs)
    p.gamma, p.beta, p.alpha = float(gamma), float(beta), float(alpha)
    p.alpha_min, p.alpha_max, p.tau = float(alpha_min), float(alpha_max), float(tau)
    p.has_sat = int(ccd_sat_level is not None)
    p.ccd_sat_level = float(ccd_sat_level) if ccd_sat_level is not None else 0.0
    p.betaParam, p.lr, p.lr_exp_param = float(betaParam), float(lr), float(lr_exp_param)
    p.tol_convergence = float(tol_convergence)
    p.scale_data = int(bool(scale_data))
    p.verbose = int(bool(verbose))
    p.adapt_beta = int(bool(adapt_beta))
    p.schedule_lr = int(bool(schedule_lr))
    p.bkg_is_map = int(bool(bkg_is_map))
    ls = LS_SPEC_DEFAULT if ls_spec is None else int(ls_spec)
    p.ls_spec = 1 if (variant == _B.BSGP_VARIANT_BETA and adapt_beta) else ls
    p.ls_series = LS_SERIES_DEFAULT if ls_series is None else int(bool(ls_series))
    p.streams = STREAMS_DEFAULT if streams is None else int(streams)
    p.team = TEAM_DEFAULT if team is None else int(team)
    p.proj_cache = PROJ_CACHE_DEFAULT if proj_cache is None else int(bool(proj_cache))
    p.gn_compact = GN_COMPACT_DEFAULT if gn_compact is None else int(bool(gn_compact))
    return p


def _write_log(stop_criterion, verbose, discr, crit, flags, MAXIT, tol):
    """The reference's sgp.log lines (sgp.py:291-298, 351-352, 399-411)."""
    log = logging.getLogger()
    n = len(discr)
    if verbose:
        if stop_criterion == 2:
            log.info('it 0 || x_k - x_(k-1) ||^2 / || x_k ||^2 0 \n')
        elif stop_criterion == 3:
            log.info('it 0 | f_k - f_(k-1) | / | f_k | 0 \n')
        elif stop_criterion == 4:
            log.info(f'it 0 D_k {discr[0]} \n')
    for k in range(1, n):
        if verbose and flags[k] & 1:
            log.warning("\tWarning, fv >= fr")
        if stop_criterion == 1:
            log.info(f'it {k} of  {MAXIT}\n')
        elif stop_criterion == 2:
            log.info(f'it {k} || x_k - x_(k-1) ||^2 / || x_k ||^2 {crit[k]} tol {tol}\n')
        elif stop_criterion == 3:
            log.info(f'it {k} | f_k - f_(k-1) | / | f_k | {crit[k]} tol {tol}\n')
        elif stop_criterion == 4:
            log.info(f'it {k} D_k {discr[k]} tol {tol}\n')


def _run(variant, gn, psf, bkg, init_recon, proj_type, stop_criterion, MAXIT, gamma, beta,
         alpha, alpha_min, alpha_max, M_alpha, tau, M, max_projs, save, obj, verbose, flux,
         ccd_sat_level, scale_data, errflag, tol_convergence, use_original_SGP_Afunction,
         beta_kw):
    _check_psf(psf)
    logging.basicConfig(filename='sgp.log', level=logging.INFO, force=True)
    if errflag and obj is None:
        raise ValueError("errflag was set to True but no ground-truth was passed.")
    if save:
        raise NotImplementedError("save=True (per-iteration FITS dumps) is not supported by the "
                                  "device engine")
    if errflag:
        raise NotImplementedError("errflag=True (per-iteration error vs obj) is not supported by "
                                  "the device engine")
    gn = np.asarray(gn)
    psf = np.asarray(psf)
    _shape = gn.shape
    if gn.ndim != 2:
        raise ValueError("gn must be a 2-D image")
    if use_original_SGP_Afunction:
        if psf.shape != _shape:
            raise ValueError(f"cannot reshape array of size {gn.size} into shape {psf.shape}: "
                             "use_original_SGP_Afunction=True needs psf.shape == gn.shape")
        mode = _B.BSGP_CONV_CIRCULAR
    else:
        mode = _B.BSGP_CONV_LINEAR_FILL
    kind, b = _bkg_kind(bkg, _shape)
    bkg_is_map = kind == "map"
    prm = _params(variant, init_recon, proj_type, stop_criterion, MAXIT, gamma, beta, alpha,
                  alpha_min, alpha_max, M_alpha, tau, M, max_projs, verbose, ccd_sat_level,
                  scale_data, tol_convergence, bkg_is_map=bkg_is_map, **beta_kw)
    x0 = None
    native_f64 = gn.dtype == np.float64
    if native_f64:
        g = gn
        bk = b
        if init_recon == 1:
            np.random.seed(42)
            x0 = np.random.randn(*gn.shape)
    else:
        # reference scaling in the input dtype (sgp.py:193-197), done on the host
        g, bk, x0, scaling, tol4 = _prelude_host(gn, b if bkg_is_map else b.reshape(()),
                                                 init_recon, flux, stop_criterion, scale_data)
        prm.scale_data = 2
        prm.prescaled_scaling = scaling
        prm.prescaled_tol4 = tol4
    plan = _B.get_plan(_shape[0], _shape[1], psf, mode)
    gd = _B.to_dev(np.asarray(g, dtype=np.float64).reshape(1, *_shape))
    bd = _B.to_dev(np.asarray(bk, dtype=np.float64).reshape((1, *_shape) if bkg_is_map else (1,)))
    fd = None if flux is None else _B.to_dev(np.array([float(flux)]))
    xd = None if x0 is None else _B.to_dev(np.asarray(x0, dtype=np.float64).reshape(1, *_shape))
    out = plan.solve(gd, bd, prm, flux=fd, x0=xd)
    _B.torch.cuda.current_stream().synchronize()
    _B.check_status(out["counters"])
    it = int(out["iters"][0])
    discr = out["discr"][0, :it + 1].cpu().numpy()
    times = out["times"][0, :it + 1].cpu().numpy()
    if verbose or stop_criterion in (1, 2, 3, 4):
        tol = tol_convergence
        if stop_criterion == 4:
            tol = 1 + 1 / np.mean(np.asarray(gn, dtype=np.float64))
        if stop_criterion == 2 and verbose:
            tol = tol * tol
        _write_log(stop_criterion, verbose, discr, out["crit"][0].cpu().numpy(),
                   out["flags"][0].cpu().numpy(), MAXIT, tol)
    x = out["x"][0].cpu().numpy().reshape(_shape)
    extra = {"beta": float(out["beta_final"][0]), "counters": out["counters"][0].cpu().numpy()}
    return x, it, discr, times, extra


# ---------------------------------------------------------------- public API
def sgp(gn, psf, bkg, init_recon=0, proj_type=0, stop_criterion=0, MAXIT=500, gamma=1e-4,
        beta=0.4, alpha=1.3, alpha_min=1e-5, alpha_max=1e5, M_alpha=3, tau=0.5, M=1,
        max_projs=1000, save=False, obj=None, verbose=True, flux=None, ccd_sat_level=None,
        scale_data=True, errflag=False, tol_convergence=1e-4, use_original_SGP_Afunction=True):
    """Scaled Gradient Projection with the KL objective (sgp.py:41-438)."""
    x, it, discr, times, _ = _run(_B.BSGP_VARIANT_KL, gn, psf, bkg, init_recon, proj_type,
                                  stop_criterion, MAXIT, gamma, beta, alpha, alpha_min,
                                  alpha_max, M_alpha, tau, M, max_projs, save, obj, verbose,
                                  flux, ccd_sat_level, scale_data, errflag, tol_convergence,
                                  use_original_SGP_Afunction, {})
    return x, it, discr, times, None


def sgp_betaDiv(gn, psf, bkg, init_recon=0, proj_type=0, stop_criterion=0, MAXIT=500,
                gamma=1e-4, beta=0.4, alpha=1.3, alpha_min=1e-5, alpha_max=1e5, M_alpha=3,
                tau=0.5, M=1, max_projs=1000, save=False, obj=None, verbose=True, flux=None,
                ccd_sat_level=None, scale_data=True, errflag=False, adapt_beta=True,
                betaParam=1.005, lr=1e-3, lr_exp_param=0.1, schedule_lr=False,
                tol_convergence=1e-4, use_original_SGP_Afunction=True):
    """Scaled Gradient Projection with the beta-divergence objective (sgp.py:506-895)."""
    bkw = dict(adapt_beta=adapt_beta, betaParam=betaParam, lr=lr, lr_exp_param=lr_exp_param,
               schedule_lr=schedule_lr)
    x, it, discr, times, extra = _run(_B.BSGP_VARIANT_BETA, gn, psf, bkg, init_recon, proj_type,
                                      stop_criterion, MAXIT, gamma, beta, alpha, alpha_min,
                                      alpha_max, M_alpha, tau, M, max_projs, save, obj, verbose,
                                      flux, ccd_sat_level, scale_data, errflag, tol_convergence,
                                      use_original_SGP_Afunction, bkw)
    print(f'Beta parameter in beta-divergence (final value): {extra["beta"]}')
    print(f'No. of iterations: {it}')
    return x, it, discr, times, None


def _dev1(a):
    return _B.to_dev(np.asarray(a, dtype=np.float64).ravel())


def betaDiv(y, x, betaParam):
    """sgp.py:441-458, evaluated on the device."""
    _B.require_gpu()
    out = _B.beta_div_dev(_dev1(y), _dev1(x), float(betaParam))
    return np.float64(out.cpu().numpy()[0])


def betaDivDeriv(y, x, betaParam):
    """sgp.py:462-495 (elementwise d betaDiv / d beta), evaluated on the device."""
    if betaParam == 0 or betaParam == 1:  # special cases (sgp.py:493-494)
        return 0
    _B.require_gpu()
    shape = np.shape(y)
    out = _B.beta_div_deriv_dev(_dev1(y), _dev1(x), float(betaParam))
    return out.cpu().numpy().reshape(shape)


def betaDivDerivwrtY(AT, den_arg, gn_arg, betaParam):
    """sgp.py:498-499: den**(beta-1) - AT(gn*den**(beta-2)); the elementwise
    parts run on the device, ``AT`` is the caller's operator."""
    _B.require_gpu()
    shape = np.shape(den_arg)
    p1, w = _B.grad_parts_dev(_dev1(den_arg), _dev1(gn_arg), float(betaParam))
    return p1.cpu().numpy().reshape(shape) - AT(x=w.cpu().numpy().reshape(shape))


def lr_schedule(init_lr, k, epoch):
    """sgp.py:502-503 (host scalar)."""
    return init_lr * math.exp(-k * epoch)


# ------------------------------------------------------------------- batched
def _solve_batch(variant, gns, psf, bkgs, betaParams=None, flux=None, init_recon=0, proj_type=0,
                 stop_criterion=0, MAXIT=500, gamma=1e-4, beta=0.4, alpha=1.3, alpha_min=1e-5,
                 alpha_max=1e5, M_alpha=3, tau=0.5, M=1, max_projs=1000, verbose=True,
                 ccd_sat_level=None, scale_data=True, tol_convergence=1e-4,
                 use_original_SGP_Afunction=True, adapt_beta=False, betaParam=1.005, lr=1e-3,
                 lr_exp_param=0.1, schedule_lr=False, ls_spec=None, ls_series=None,
                 streams=None, team=None, proj_cache=None, gn_compact=None,
                 device_out=False):
    torch = _B.torch
    per_image = (psf.dim() if torch.is_tensor(psf) else np.ndim(psf)) == 3
    if not per_image:
        _check_psf(np.asarray(psf))
    _B.require_gpu()
    if not torch.is_tensor(gns):
        gns = _B.to_dev(np.asarray(gns, dtype=np.float64))
    Bn, H, W = gns.shape
    mode = _B.BSGP_CONV_CIRCULAR if use_original_SGP_Afunction else _B.BSGP_CONV_LINEAR_FILL
    if not torch.is_tensor(bkgs):
        bk = np.asarray(bkgs, dtype=np.float64)
        bk = np.broadcast_to(bk, (Bn,)) if bk.ndim <= 1 and bk.size in (1, Bn) else bk
        bkgs = _B.to_dev(np.ascontiguousarray(bk))
    bkg_is_map = bkgs.dim() == 3
    prm = _params(variant, init_recon, proj_type, stop_criterion, MAXIT, gamma, beta, alpha,
                  alpha_min, alpha_max, M_alpha, tau, M, max_projs, verbose, ccd_sat_level,
                  scale_data, tol_convergence, adapt_beta=adapt_beta, betaParam=betaParam, lr=lr,
                  lr_exp_param=lr_exp_param, schedule_lr=schedule_lr, bkg_is_map=bkg_is_map,
                  ls_spec=ls_spec, ls_series=ls_series, streams=streams,
                  team=team, proj_cache=proj_cache, gn_compact=gn_compact)
    x0 = None
    if init_recon == 1:
        np.random.seed(42)
        x0 = _B.to_dev(np.broadcast_to(np.random.randn(H, W), (Bn, H, W)))
    b0 = None if betaParams is None else _B.to_dev(np.broadcast_to(
        np.asarray(betaParams, dtype=np.float64), (Bn,)))
    fl = None if flux is None else _B.to_dev(np.broadcast_to(np.asarray(flux, dtype=np.float64),
                                                            (Bn,)))
    if per_image:  # psf [B, kh, kw]: image i uses psf[i] (each checked as sgp.py:97-102)
        if len(psf) != Bn:
            raise ValueError("one PSF per image: psf must be [B, kh, kw]")
        plan = _B.per_image_plan(H, W, psf, mode)
    else:
        plan = _B.get_plan(H, W, np.asarray(psf), mode)
    out = plan.solve(gns, bkgs, prm, flux=fl, x0=x0, beta0=b0)
    if device_out:
        return out
    torch.cuda.current_stream().synchronize()
    _B.check_status(out["counters"])
    return {k: (v.cpu().numpy() if v is not None else None) for k, v in out.items()}


def sgp_batch(gns, psf, bkgs, **kw):
    """KL-SGP on a batch [B, H, W] (one launch); psf is one [kh, kw] PSF or
    [B, kh, kw] (a PSF per image).  Returns a dict of arrays:
    x [B,H,W], iters [B], discr [B,MAXIT+1], times, crit, flags, counters."""
    return _solve_batch(_B.BSGP_VARIANT_KL, gns, psf, bkgs, **kw)


def sgp_betaDiv_batch(gns, psf, bkgs, betaParams=None, **kw):
    """beta-SGP on a batch [B, H, W] with per-image initial betaParam (the
    multi-start beta search of application_sgp_subdivisions.py:70-107 as one
    launch).  Returns the dict of :func:`sgp_batch` plus beta_final [B]."""
    return _solve_batch(_B.BSGP_VARIANT_BETA, gns, psf, bkgs, betaParams=betaParams, **kw)
