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

``save=True`` writes the reference's per-iteration FITS files
(SGP_reconstructed_images/, sgp.py:223-231, 416-422) from device snapshots of
every iterate; ``errflag=True`` (``sgp`` only, as in the reference) returns
the per-iteration error as the fifth element (sgp.py:240-257, 394-396).
A float32 image is solved with the reference's float32 arithmetic
reproduced on the device, its float32 prelude (scaling, null-pixel fill,
start, flux) included (numpy 1.x rules; include/bsgp.h ``gn_f32``), in the
single-image drop-in and in the batched calls alike.

Deliberate differences: a plain Python float ``bkg`` is
accepted (the reference crashes on ``bkg.flatten()``); errflag at MAXIT
returns the error array instead of the reference's IndexError.

Extra: :func:`sgp_betaDiv_batch` / :func:`sgp_batch` solve
many images or beta candidates in one launch.
"""
import errno
import logging
import math
import os

import numpy as np

import _bsgp as _B
import fits_io

DEFAULT_PARAMS = (1000, 1e-4, 0.4, 1e-5, 1e5, 1e1, 3, 0.5, 1)  # sgp.py:34
DEFAULT_COLUMNS = ['label', 'xcentroid', 'ycentroid', 'sky_centroid',
                   'bbox_xmin', 'bbox_xmax', 'bbox_ymin', 'bbox_ymax',
                   'area', 'semimajor_sigma', 'semiminor_sigma',
                   'orientation', 'eccentricity', 'min_value', 'max_value',
                   'local_background', 'segment_flux', 'segment_fluxerr', 'ellipticity',
                   'fwhm']  # sgp.py:35-39

LS_SPEC_DEFAULT = 2  # line-search trial lambdas evaluated per pass over the data
LS_SERIES_DEFAULT = 1  # small line-search steps from the moment series (general beta)
def _hw_queues():
    try:
        return int(os.environ.get("GPU_MAX_HW_QUEUES", "4"))
    except ValueError:
        return 4


# Sub-batches of a batched solve, each on its own stream (the caller's + plan
# streams) so that kernels of different phases overlap.  One per hardware queue
# HIP opens for the process (GPU_MAX_HW_QUEUES, 4 by default): C3 A/B with 4
# queues: 4 > 3 > 2 sub-batches (8 collapse to 164 k); with 8 queues 8
# sub-batches are +2.8 % over 4; 16 queues with 12 or 16 sub-batches: no gain.
STREAMS_DEFAULT = 8 if _hw_queues() >= 8 else 4
TEAM_DEFAULT = 0  # workgroups per image: 0 = auto (spread small batches over the CUs)
PROJ_CACHE_DEFAULT = 1  # projectDF evaluations inside a known root bracket read a pixel list
GN_COMPACT_DEFAULT = 1  # f32-exact observed images stored in f32 (bit-identical results)
PERSIST_DEFAULT = 1  # one-workgroup batches: all iterations in one persistent launch (C3 +1.4 %, A/B)


# ------------------------------------------------------------------ helpers
def _check_psf(psf):
    # (np.sum of a C-contiguous array is np.sum of its flatten(): the same
    # pairwise order over the same buffer, without the copy)
    total = np.sum(psf) if isinstance(psf, np.ndarray) and psf.flags.c_contiguous \
        else np.sum(psf.flatten())
    checkPSF = np.abs(total - 1.)
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


def _scalar_dtype(v):
    if isinstance(v, (np.generic, np.ndarray)):
        return np.asarray(v).dtype
    return np.dtype(np.float64) if isinstance(v, float) else np.dtype(np.int64)


def _np1_scalar_div(a, b):
    """a / b of two scalars as numpy 1.x computes it (the reference's numpy:
    the golden fixtures come from numpy 1.26): scalar-with-scalar operations
    promote by type, a Python float counting as float64, so float32 / float32
    stays float32 and a Python float over a float32 scaling is float64."""
    rt = np.promote_types(_scalar_dtype(a), _scalar_dtype(b))
    if rt.kind != "f":
        rt = np.dtype(np.float64)
    return rt.type(np.asarray(a, dtype=rt) / np.asarray(b, dtype=rt))


def _prelude_host(gn, bkg, init_recon, flux, stop_criterion, scale_data):
    """sgp.py:166-211 (= 619-666) for a float32 image, in float32 with numpy
    1.x promotion: an array never widens for a Python or 0-d operand, scalars
    promote by type.  Returns the scaled, null-pixel-fixed float32 image, the
    scaled background (its own dtype), the scaled start x, the scaling, the
    stop-rule-4 tolerance and the scaled flux (None: the device sums it)."""
    gn = np.asarray(gn)
    gn = gn.astype(gn.dtype.newbyteorder("="), copy=True)  # native order, same values
    dt = gn.dtype
    bk = np.asarray(bkg)
    bk = bk.astype(bk.dtype.newbyteorder("="))
    if init_recon == 0:
        x = np.zeros_like(gn)
    elif init_recon == 1:
        np.random.seed(42)
        x = np.random.randn(*gn.shape)
    elif init_recon == 2:
        x = gn.copy()
    else:
        if flux is None:
            v = _np1_scalar_div(np.sum(gn - (bk.astype(dt) if bk.ndim == 0 else bk)), gn.size)
        else:
            v = _np1_scalar_div(flux, gn.size)
        x = np.full(gn.shape, v).astype(dt)  # v * ones_like(gn) runs in gn's dtype
    gn = gn.flatten()
    x = x.flatten()
    bkf = bk.flatten()
    tol4 = 1 + 1 / float(np.mean(gn)) if stop_criterion == 4 else 0.0
    if scale_data:
        scaling = np.max(gn)
        gn = gn / scaling
        bkf = bkf / scaling
        x = x / scaling
    else:
        scaling = 1.
    vmin = np.min(gn[gn > 0])
    gn[gn <= 0] = np.float64(vmin) * np.finfo(float).eps * np.finfo(float).eps
    if flux is not None:
        flux_s = _np1_scalar_div(flux, scaling)
    elif bkf.dtype != np.float64:
        flux_s = np.sum(gn - bkf)  # float32 background: numpy's float32 reduction (sgp.py:209)
    else:
        flux_s = None  # float64 sum, on the device
    return gn, bkf, x, float(scaling), float(tol4), flux_s


def _f32_on_device(init_recon, flux, bkg):
    """A float32 image's prelude (sgp.py:620-666) runs on the device
    (include/bsgp.h gn_f32 with scale_data 0/1) unless numpy would compute part
    of it in float32 from the background too: a float32 (or integer)
    background, or init_recon 3 without a flux and with a scalar background
    (np.sum(gn - bkg) of a float32 array, sgp.py:629).  Those few cases keep
    the host prelude (_prelude_host)."""
    b = np.asarray(bkg)
    if not (b.dtype.kind == "f" and b.dtype.itemsize == 8):  # any byte order
        return False
    return not (init_recon == 3 and flux is None and b.size == 1)


def _flux_is_f32(flux):
    return flux is not None and np.asarray(flux).dtype == np.float32


def _gn_scaled_host(gn, scale_data):
    """The scaled, null-pixel-fixed float64 image of sgp.py:193-204, for the
    FITS files of save=True only (orig.fits, res_k.fits)."""
    g = np.asarray(gn, dtype=np.float64).flatten()
    if scale_data:
        g = g / np.max(g)
    vmin = np.min(g[g > 0])
    g[g <= 0] = vmin * np.finfo(float).eps * np.finfo(float).eps
    return g


def _params(variant, init_recon, proj_type, stop_criterion, MAXIT, gamma, beta, alpha, alpha_min,
            alpha_max, M_alpha, tau, M, max_projs, verbose, ccd_sat_level, scale_data,
            tol_convergence, adapt_beta=False, betaParam=1.005, lr=1e-3, lr_exp_param=0.1,
            schedule_lr=False, bkg_is_map=False, ls_spec=None, ls_series=None, streams=None,
            team=None, proj_cache=None, gn_compact=None, betaParams=None, persistent=None):
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
    p.gn_f32 = 0
    p.persistent = PERSIST_DEFAULT if persistent is None else int(bool(persistent))
    if betaParams is not None:
        b0 = np.asarray(betaParams, dtype=np.float64)
        p.beta0_general = int(bool(np.all((b0 != 0.0) & (b0 != 1.0))))
    return p


def _log_records(stop_criterion, verbose, discr, crit, flags, MAXIT, tol):
    """The reference's sgp.log records (sgp.py:291-298, 351-352, 399-411), in
    order, as (level, message)."""
    I, W = logging.INFO, logging.WARNING
    recs = []
    if verbose:
        if stop_criterion == 2:
            recs.append((I, 'it 0 || x_k - x_(k-1) ||^2 / || x_k ||^2 0 \n'))
        elif stop_criterion == 3:
            recs.append((I, 'it 0 | f_k - f_(k-1) | / | f_k | 0 \n'))
        elif stop_criterion == 4:
            recs.append((I, f'it 0 D_k {discr[0]} \n'))
    for k in range(1, len(discr)):
        if verbose and flags[k] & 1:
            recs.append((W, "\tWarning, fv >= fr"))
        if stop_criterion == 1:
            recs.append((I, f'it {k} of  {MAXIT}\n'))
        elif stop_criterion == 2:
            recs.append((I, f'it {k} || x_k - x_(k-1) ||^2 / || x_k ||^2 {crit[k]} tol {tol}\n'))
        elif stop_criterion == 3:
            recs.append((I, f'it {k} | f_k - f_(k-1) | / | f_k | {crit[k]} tol {tol}\n'))
        elif stop_criterion == 4:
            recs.append((I, f'it {k} D_k {discr[k]} tol {tol}\n'))
    return recs


def _write_log(stop_criterion, verbose, discr, crit, flags, MAXIT, tol):
    """The reference's sgp.log lines.  With the logging set-up the reference
    itself makes (sgp.py:104 / :564: basicConfig(filename='sgp.log'), one
    FileHandler, the default format, nothing filtered) the lines go to the
    file in ONE write, byte for byte what one logging call per line writes
    (~20 us per record through the logging machinery: 0.7 ms of a 32-iteration
    call of the application's); any other set-up gets one logging call per
    record."""
    recs = _log_records(stop_criterion, verbose, discr, crit, flags, MAXIT, tol)
    log = logging.getLogger()
    hs = log.handlers
    h = hs[0] if len(hs) == 1 else None
    fast = (h is not None and type(h) is logging.FileHandler and not h.filters
            and not log.filters and h.formatter is not None
            and h.formatter._fmt == logging.BASIC_FORMAT and h.level <= logging.INFO
            and log.isEnabledFor(logging.INFO) and not logging.root.manager.disable
            and h.stream is not None)
    if not fast:
        for lvl, msg in recs:
            log.log(lvl, msg)
        return
    text = "".join(f"{logging.getLevelName(lvl)}:{log.name}:{msg}{h.terminator}"
                   for lvl, msg in recs)
    h.acquire()
    try:
        h.stream.write(text)
        h.flush()
    finally:
        h.release()


SAVE_DIR = "SGP_reconstructed_images/"


def _save_setup(gs, shape):
    """sgp.py:223-231 / 678-686: the directory, and orig.fits when it is new."""
    try:
        os.mkdir(SAVE_DIR)
        fits_io.write_fits(f"{SAVE_DIR}/orig.fits", gs.reshape(shape))
    except OSError as exc:
        if exc.errno != errno.EEXIST:
            raise OSError("Directory already exists!")


def _save_iterates(x_iter, gs, shape):
    """sgp.py:416-422 / 870-876: rec_k.fits (the scaled iterate after iteration
    k, before the revert) and res_k.fits = (x - gn) / sqrt(x)."""
    for k in range(x_iter.shape[0]):
        x = x_iter[k].reshape(-1)
        fits_io.write_fits(f"SGP_reconstructed_images/rec_{k + 1}.fits", x.reshape(shape),
                           overwrite=True)
        with np.errstate(all="ignore"):
            res = np.divide(x - gs, np.sqrt(x))
        fits_io.write_fits(f"SGP_reconstructed_images/res_{k + 1}.fits", res.reshape(shape),
                           overwrite=True)


def _err_layout(e, it):
    """The reference's err array (sgp.py:241, 257, 394-396, 431-432): err[0]
    after the initial projection, then the error after iteration k stored at
    index k+1 (the increment comes first), cut to iters+1 entries, so err[1]
    stays 0 and the last iteration's error is dropped.  At MAXIT the
    reference's store overruns its array (IndexError); this returns what the
    array would have held."""
    err = np.zeros(it + 1)
    err[0] = e[0]
    if it >= 2:
        err[2:] = e[1:it]
    return err


def _run(variant, gn, psf, bkg, init_recon, proj_type, stop_criterion, MAXIT, gamma, beta,
         alpha, alpha_min, alpha_max, M_alpha, tau, M, max_projs, save, obj, verbose, flux,
         ccd_sat_level, scale_data, errflag, tol_convergence, use_original_SGP_Afunction,
         beta_kw, betas=None):
    """One drop-in solve; with ``betas`` (beta variant) the same image is solved
    for every initial betaParam in one batched launch and a list of results is
    returned (the multi-start of application_sgp_subdivisions.py:83-99)."""
    _check_psf(psf)
    logging.basicConfig(filename='sgp.log', level=logging.INFO, force=True)
    # sgp_betaDiv has no error path: errflag / obj are accepted and ignored
    errflag = bool(errflag) and variant == _B.BSGP_VARIANT_KL
    if errflag and obj is None:
        raise ValueError("errflag was set to True but no ground-truth was passed.")
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
                  scale_data, tol_convergence, bkg_is_map=bkg_is_map, betaParams=betas,
                  **beta_kw)
    x0 = None
    fl = None if flux is None else np.array([float(flux)])
    f32 = gn.dtype.kind == "f" and gn.dtype.itemsize == 4
    dev32 = f32 and _f32_on_device(init_recon, flux, b if bkg_is_map else bkg)
    if dev32:
        # float32 image: the device runs the reference's float32 prelude
        # (scaling, null-pixel fill, start, flux; include/bsgp.h ABI 3)
        g = np.asarray(gn, dtype=np.float64)  # the float32 values, exact
        bk = b
        prm.gn_f32 = 1
        prm.scale_data = 1 if scale_data else 0
        prm.flux_f32 = int(_flux_is_f32(flux))
        if init_recon == 1:
            np.random.seed(42)
            x0 = np.random.randn(*gn.shape)
    elif f32:
        # the reference computes in the image's float32 (sgp.py:193-211): scale
        # on the host in float32, and let the device reproduce the float32
        # parts of the beta objective (include/bsgp.h gn_f32)
        g, bk, x0, scaling, tol4, flux_s = _prelude_host(
            gn, b if bkg_is_map else np.asarray(bkg).reshape(()), init_recon, flux,
            stop_criterion, scale_data)
        prm.scale_data = 2
        prm.prescaled_scaling = scaling
        prm.prescaled_tol4 = tol4
        prm.gn_f32 = 1
        fl = None if flux_s is None else np.array([float(flux_s)])
    else:
        # float64 in any byte order (and integer images, which numpy's
        # true division turns into float64 at the scaling, sgp.py:195)
        g = np.asarray(gn, dtype=np.float64)
        bk = b
        if init_recon == 1:
            np.random.seed(42)
            x0 = np.random.randn(*gn.shape)
    _B.require_gpu()  # the product path runs on the device or not at all
    # inputs through page-locked memory, enqueued without waiting (_B.to_dev_async)
    gd = _B.to_dev_async(np.asarray(g, dtype=np.float64).reshape(1, *_shape))
    bd = _B.to_dev_async(np.asarray(bk, dtype=np.float64).reshape((1, *_shape) if bkg_is_map
                                                                  else (1,)))
    fd = None if fl is None else _B.to_dev_async(fl)
    xd = None if x0 is None else _B.to_dev_async(np.asarray(x0, dtype=np.float64).reshape(1, *_shape))
    od = None if not errflag else _B.to_dev_async(np.asarray(obj, dtype=np.float64).reshape(1,
                                                                                           *_shape))
    gs = None
    if save:
        g_f = g
        if dev32:  # the scaled float32 image of the FITS files, restated on the host
            g_f = _prelude_host(gn, b if bkg_is_map else np.asarray(bkg).reshape(()), init_recon,
                                flux, stop_criterion, scale_data)[0]
        gs = np.asarray(g_f, dtype=np.float64).reshape(-1) if f32 else _gn_scaled_host(g, scale_data)
        _save_setup(np.asarray(g_f).reshape(-1) if f32 else gs, _shape)
    b0 = None
    if betas is not None:
        nb = len(betas)
        gd, bd, xd, od = (None if t is None else t.expand(nb, *t.shape[1:]).contiguous()
                          for t in (gd, bd, xd, od))
        fd = None if fd is None else fd.expand(nb).contiguous()
        b0 = _B.to_dev_async(np.asarray(betas, dtype=np.float64))
    with _B.lease_plan(_shape[0], _shape[1], psf, mode) as plan:
        dout = plan.solve(gd, bd, prm, flux=fd, x0=xd, obj=od, beta0=b0, want_iterates=bool(save))
    # every output the caller gets, in one round of copies and one stream sync
    # (each .cpu() had waited for the stream on its own)
    out = _B.to_host({k: dout[k] for k in ("x", "iters", "discr", "times", "crit", "flags",
                                           "beta_final", "counters", "err")})
    _B.check_status(out["counters"])
    def log_run(i, discr):
        if verbose or stop_criterion in (1, 2, 3, 4):
            tol = tol_convergence
            if stop_criterion == 4:  # sgp.py:644, in the image's dtype
                tol = 1 + 1 / float(np.mean(gn if f32 else np.asarray(gn, dtype=np.float64)))
            if stop_criterion == 2 and verbose:
                tol = tol * tol
            _write_log(stop_criterion, verbose, discr, out["crit"][i],
                       out["flags"][i], MAXIT, tol)

    if betas is not None:
        res = []
        for i in range(len(betas)):
            it = int(out["iters"][i])
            discr = out["discr"][i, :it + 1]
            log_run(i, discr)  # each candidate is one sgp_betaDiv call in the application
            res.append((out["x"][i].reshape(_shape), it, discr,
                        out["times"][i, :it + 1],
                        {"beta": float(out["beta_final"][i]),
                         "counters": out["counters"][i], "err": None,
                         "log": lambda i=i, d=discr: log_run(i, d)}))
        return res
    it = int(out["iters"][0])
    discr = out["discr"][0, :it + 1]
    times = out["times"][0, :it + 1]
    log_run(0, discr)
    if save:
        _save_iterates(dout["x_iter"][0, :it].cpu().numpy(), gs, _shape)  # (can be large)
    x = out["x"][0].reshape(_shape)
    extra = {"beta": float(out["beta_final"][0]), "counters": out["counters"][0],
             "err": _err_layout(out["err"][0], it) if errflag else None}
    return x, it, discr, times, extra


# ---------------------------------------------------------------- public API
def sgp(gn, psf, bkg, init_recon=0, proj_type=0, stop_criterion=0, MAXIT=500, gamma=1e-4,
        beta=0.4, alpha=1.3, alpha_min=1e-5, alpha_max=1e5, M_alpha=3, tau=0.5, M=1,
        max_projs=1000, save=False, obj=None, verbose=True, flux=None, ccd_sat_level=None,
        scale_data=True, errflag=False, tol_convergence=1e-4, use_original_SGP_Afunction=True):
    """Scaled Gradient Projection with the KL objective (sgp.py:41-438)."""
    x, it, discr, times, extra = _run(_B.BSGP_VARIANT_KL, gn, psf, bkg, init_recon, proj_type,
                                      stop_criterion, MAXIT, gamma, beta, alpha, alpha_min,
                                      alpha_max, M_alpha, tau, M, max_projs, save, obj, verbose,
                                      flux, ccd_sat_level, scale_data, errflag, tol_convergence,
                                      use_original_SGP_Afunction, {})
    return x, it, discr, times, extra["err"]


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
def _bkg_batch(bkgs, Bn, H, W):
    """Backgrounds of a batch as the device expects them: [B] scalars or
    [B, H, W] maps, float64, contiguous.  Accepted: a scalar, [1] or [B]
    scalars, one [H, W] (or [1, H, W]) map for every image, or [B, H, W]."""
    torch = _B.torch
    t = (bkgs.to(device="cuda", dtype=torch.float64) if torch.is_tensor(bkgs)
         else _B.to_dev(np.asarray(bkgs, dtype=np.float64)))
    shape = tuple(t.shape)
    if t.dim() == 0 or (t.dim() == 1 and shape[0] in (1, Bn)):
        return t.reshape(-1).expand(Bn).contiguous()
    if shape in ((H, W), (1, H, W)):
        return t.reshape(1, H, W).expand(Bn, H, W).contiguous()
    if shape == (Bn, H, W):
        return t.contiguous()
    raise ValueError(f"bkg of shape {shape} fits neither [B]={Bn} scalars nor [B, H, W] maps "
                     f"of {H}x{W} images")


def _solve_batch(variant, gns, psf, bkgs, betaParams=None, flux=None, init_recon=0, proj_type=0,
                 stop_criterion=0, MAXIT=500, gamma=1e-4, beta=0.4, alpha=1.3, alpha_min=1e-5,
                 alpha_max=1e5, M_alpha=3, tau=0.5, M=1, max_projs=1000, verbose=True,
                 ccd_sat_level=None, scale_data=True, tol_convergence=1e-4,
                 use_original_SGP_Afunction=True, adapt_beta=False, betaParam=1.005, lr=1e-3,
                 lr_exp_param=0.1, schedule_lr=False, ls_spec=None, ls_series=None,
                 streams=None, team=None, proj_cache=None, gn_compact=None,
                 device_out=False, profile=False, storage="f64", gn_f32=None, save=False,
                 errflag=False, obj=None, persistent=None):
    torch = _B.torch
    if save or errflag:  # sgp()/sgp_betaDiv() keywords: per-image files / err arrays
        raise ValueError("save / errflag are single-image options: use sgp / sgp_betaDiv")
    per_image = (psf.dim() if torch.is_tensor(psf) else np.ndim(psf)) == 3
    _B.require_gpu()
    if not per_image:  # a shared PSF is checked in its own dtype before any upload
        psf = np.asarray(psf.cpu().numpy() if torch.is_tensor(psf) else psf)
        _B.check_psf_once(psf, _check_psf)
    # float32 images (the application's FITS data): the reference's float32
    # prelude on the device, per image (include/bsgp.h gn_f32, ABI 3)
    if gn_f32 is None:
        gn_f32 = (gns.dtype == torch.float32) if torch.is_tensor(gns) else \
            np.asarray(gns).dtype.kind == "f" and np.asarray(gns).dtype.itemsize == 4
    if gn_f32:
        f64b = (bkgs.dtype == torch.float64) if torch.is_tensor(bkgs) else \
            (np.asarray(bkgs).dtype.kind == "f" and np.asarray(bkgs).dtype.itemsize == 8)
        bnd = bkgs.dim() if torch.is_tensor(bkgs) else np.ndim(bkgs)
        if not f64b or (init_recon == 3 and flux is None and bnd <= 1):
            raise ValueError("float32 images in a batch need float64 backgrounds, and a flux for "
                             "init_recon=3 with scalar backgrounds (numpy computes those parts "
                             "in float32 from the background; solve such images one at a time "
                             "with sgp_betaDiv / sgp)")
    if torch.is_tensor(gns):
        gns = gns.to(device="cuda", dtype=torch.float64).contiguous()
    else:
        gns = _B.to_dev(np.asarray(gns, dtype=np.float64))
    if gns.dim() != 3:
        raise ValueError("gns must be a batch [B, H, W]")
    Bn, H, W = gns.shape
    mode = _B.BSGP_CONV_CIRCULAR if use_original_SGP_Afunction else _B.BSGP_CONV_LINEAR_FILL
    bkgs = _bkg_batch(bkgs, Bn, H, W)
    bkg_is_map = bkgs.dim() == 3
    prm = _params(variant, init_recon, proj_type, stop_criterion, MAXIT, gamma, beta, alpha,
                  alpha_min, alpha_max, M_alpha, tau, M, max_projs, verbose, ccd_sat_level,
                  scale_data, tol_convergence, adapt_beta=adapt_beta, betaParam=betaParam, lr=lr,
                  lr_exp_param=lr_exp_param, schedule_lr=schedule_lr, bkg_is_map=bkg_is_map,
                  ls_spec=ls_spec, ls_series=ls_series, streams=streams,
                  team=team, proj_cache=proj_cache, gn_compact=gn_compact, betaParams=betaParams,
                  persistent=persistent)
    if gn_f32:
        prm.gn_f32 = 1
        prm.scale_data = 1 if scale_data else 0
        prm.flux_f32 = int(_flux_is_f32(flux) if not torch.is_tensor(flux)
                           else flux.dtype == torch.float32)
    x0 = None
    if init_recon == 1:
        np.random.seed(42)
        x0 = _B.to_dev(np.broadcast_to(np.random.randn(H, W), (Bn, H, W)))
    b0 = None if betaParams is None else _B.to_dev(np.broadcast_to(
        np.asarray(betaParams, dtype=np.float64), (Bn,)))
    if flux is None:
        fl = None
    elif torch.is_tensor(flux):
        fl = flux.to(device="cuda", dtype=torch.float64).reshape(-1).expand(Bn).contiguous()
    else:
        fl = _B.to_dev(np.broadcast_to(np.asarray(flux, dtype=np.float64), (Bn,)))
    if per_image:  # psf [B, kh, kw]: image i uses psf[i] (each checked as sgp.py:97-102)
        if len(psf) != Bn:
            raise ValueError("one PSF per image: psf must be [B, kh, kw]")
        plan = _B.per_image_plan(H, W, psf, mode, storage=storage)
        out = plan.solve(gns, bkgs, prm, flux=fl, x0=x0, beta0=b0, profile=profile)
    else:
        with _B.lease_plan(H, W, psf, mode, storage=storage) as plan:
            out = plan.solve(gns, bkgs, prm, flux=fl, x0=x0, beta0=b0, profile=profile)
    if device_out:
        return out
    prof = {k: out.pop(k) for k in ("kernel_ms", "launches") if k in out}
    torch.cuda.current_stream().synchronize()
    _B.check_status(out["counters"])
    res = {k: (v.cpu().numpy() if v is not None else None) for k, v in out.items()}
    res.update(prof)
    return res


def on_devices(devices, n, work):
    """Shard n independent items over GPUs: contiguous shards [lo, hi), one
    host thread per device, ``work(device, lo, hi)`` run with that device
    current (images and beta candidates are independent, so no
    collective; the C library holds no Python lock while a solve runs).
    Returns the per-shard results in device order."""
    import threading
    devices = list(devices)
    k = len(devices)
    if k == 0:
        raise ValueError("devices is empty")
    bounds = [(n * j // k, n * (j + 1) // k) for j in range(k)]
    res, errs = [None] * k, [None] * k

    def run(j):
        try:
            with _B.torch.cuda.device(devices[j]):
                res[j] = work(devices[j], *bounds[j])
                _B.torch.cuda.current_stream().synchronize()
        except BaseException as e:  # re-raised in the caller
            errs[j] = e

    threads = [threading.Thread(target=run, args=(j,)) for j in range(k)
               if bounds[j][1] > bounds[j][0]]
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    for e in errs:
        if e is not None:
            raise e
    return [r for r, (lo, hi) in zip(res, bounds) if hi > lo]


def _shard(v, lo, hi, Bn):
    """The [lo, hi) part of a per-image argument (scalars and shared maps pass)."""
    if v is None:
        return None
    shape = tuple(v.shape) if hasattr(v, "shape") else np.shape(v)
    if len(shape) in (1, 3) and shape[0] == Bn and Bn > 1:  # [B] values or [B, H, W] maps
        return v[lo:hi]
    return v


def _solve_sharded(variant, gns, psf, bkgs, devices, betaParams=None, flux=None, **kw):
    Bn = gns.shape[0]
    if kw.get("device_out"):
        raise ValueError("devices=... returns host arrays (device_out is per device)")
    if len(set(devices)) < len(list(devices)):
        # several shards on one GPU run concurrently: team solves size their
        # teams for the whole device and spin on co-resident members, so
        # shards that share a GPU use one workgroup per image
        kw["team"] = 1
    per_image_psf = (psf.dim() if _B.torch.is_tensor(psf) else np.ndim(psf)) == 3

    def work(dev, lo, hi):
        return _solve_batch(variant, gns[lo:hi], psf[lo:hi] if per_image_psf else psf,
                            _shard(bkgs, lo, hi, Bn),
                            betaParams=_shard(betaParams, lo, hi, Bn),
                            flux=_shard(flux, lo, hi, Bn), **kw)

    parts = on_devices(devices, Bn, work)
    return {k: (np.concatenate([p[k] for p in parts]) if parts[0][k] is not None else None)
            for k in parts[0]}


def sgp_batch(gns, psf, bkgs, devices=None, **kw):
    """KL-SGP on a batch [B, H, W] (one launch); psf is one [kh, kw] PSF or
    [B, kh, kw] (a PSF per image).  Returns a dict of arrays:
    x [B,H,W], iters [B], discr [B,MAXIT+1], times, crit, flags, counters.
    ``devices=[0, 1, ...]`` shards the batch over those GPUs (contiguous
    shards, one host thread per GPU, results concatenated in batch order).
    ``storage='f32'`` keeps the iteration vectors in float32 in HBM (every sum
    and scalar stays float64; SURVEY config C4); the default 'f64' is the
    reference's arithmetic."""
    if devices is not None:
        return _solve_sharded(_B.BSGP_VARIANT_KL, gns, psf, bkgs, devices, **kw)
    return _solve_batch(_B.BSGP_VARIANT_KL, gns, psf, bkgs, **kw)


def sgp_betaDiv_batch(gns, psf, bkgs, betaParams=None, devices=None, **kw):
    """beta-SGP on a batch [B, H, W] with per-image initial betaParam (the
    multi-start beta search of application_sgp_subdivisions.py:70-107 as one
    launch).  Returns the dict of :func:`sgp_batch` plus beta_final [B].
    ``devices`` shards (image, beta) pairs over GPUs as in :func:`sgp_batch`."""
    if devices is not None:
        return _solve_sharded(_B.BSGP_VARIANT_BETA, gns, psf, bkgs, devices,
                              betaParams=betaParams, **kw)
    return _solve_batch(_B.BSGP_VARIANT_BETA, gns, psf, bkgs, betaParams=betaParams, **kw)


# --------------------------------------------------------- multi-start beta
APP_BETA_SEEDS = (0, 42, 951, 93, 810)  # application_sgp_subdivisions.py:71


def app_beta_candidates(seeds=APP_BETA_SEEDS, loc=1.0, scale=0.05):
    """The application's initial betas: one np.random.normal(1, 0.05) draw per
    seed (application_sgp_subdivisions.py:70-76)."""
    out = []
    for s in seeds:
        np.random.seed(s)
        out.append(np.random.normal(loc=loc, scale=scale))
    return out


def argmin_strict(scores):
    """The application's choice among the candidates
    (application_sgp_subdivisions.py:78-99, application_sgp_star_stamps.py:
    75-98): running minimum from +inf, a candidate wins only with a score
    strictly below every earlier one, so the first of equal scores wins and a
    NaN score never does.  None when no score is below +inf (the reference is
    then left with best_beta_init = None)."""
    best, low = None, np.inf
    for i, v in enumerate(scores):
        if v < low:
            low, best = v, i
    return best


def sgp_betaDiv_multistart(gn, psf, bkg, betas=None, score=None, final_solve=True, devices=None,
                           **kwargs):
    """The beta search of application_sgp_subdivisions.py:69-107 in ONE
    batched launch: every candidate initial beta (default: the application's
    five seeds) is solved together, and the host picks the best candidate by
    ``score(x)`` with the application's strict running minimum
    (:func:`argmin_strict`).

    The application then solves the image once more with the best initial
    beta (:100-107).  The reference is deterministic, so that run repeats the
    best candidate's run exactly; here the candidate's result is returned
    instead of solving again (with final_solve=True the final run's sgp.log
    lines and its two printed lines, sgp.py:892-893, are repeated for it).

    ``score`` is the application's criterion, the photometric flux fractional
    difference 1 - sum(segment_flux(x)) / sum(segment_flux(gn)) (:92-99); it
    needs photutils, which this package does not carry, so the caller passes
    it.  Without one the candidates are ranked by their final discrepancy
    discr[-1] (a stand-in, not the application's choice).  ``kwargs`` are
    sgp_betaDiv's keyword arguments.  ``devices=[...]`` spreads the
    candidates over GPUs (one batched launch per GPU).

    Returns (x, iters, discr, times, None) of the best candidate and a dict
    with "betas", "scores", "best_beta", "best", "beta_final" (the final beta
    of every candidate) and "candidates" (each candidate's (x, iters, discr,
    times, None))."""
    betas = list(app_beta_candidates() if betas is None else betas)
    kw = dict(kwargs)
    kw.pop("betaParam", None)
    bkw = {k: kw.pop(k) for k in ["adapt_beta", "lr", "lr_exp_param", "schedule_lr"] if k in kw}
    bkw.setdefault("adapt_beta", True)  # sgp_betaDiv's default (sgp.py:510)
    args = dict(init_recon=0, proj_type=0, stop_criterion=0, MAXIT=500, gamma=1e-4, beta=0.4,
                alpha=1.3, alpha_min=1e-5, alpha_max=1e5, M_alpha=3, tau=0.5, M=1,
                max_projs=1000, save=False, obj=None, verbose=True, flux=None,
                ccd_sat_level=None, scale_data=True, errflag=False, tol_convergence=1e-4,
                use_original_SGP_Afunction=True)
    unknown = set(kw) - set(args)
    if unknown:
        raise TypeError(f"unexpected keyword arguments {sorted(unknown)}")
    args.update(kw)
    if args["save"]:
        raise ValueError("save=True writes one set of files per solve: use sgp_betaDiv")
    shared = devices is not None and len(set(devices)) < len(list(devices))

    def work(dev, lo, hi):
        extra = dict(team=1) if shared else {}  # shards sharing a GPU: no spinning teams
        return _run(_B.BSGP_VARIANT_BETA, gn, psf, bkg, args["init_recon"], args["proj_type"],
                    args["stop_criterion"], args["MAXIT"], args["gamma"], args["beta"],
                    args["alpha"], args["alpha_min"], args["alpha_max"], args["M_alpha"],
                    args["tau"], args["M"], args["max_projs"], False, None, args["verbose"],
                    args["flux"], args["ccd_sat_level"], args["scale_data"], False,
                    args["tol_convergence"], args["use_original_SGP_Afunction"],
                    dict(bkw, betaParam=betas[lo], **extra), betas=betas[lo:hi])

    if devices is None:
        runs = work(None, 0, len(betas))
    else:
        runs = [r for part in on_devices(devices, len(betas), work) for r in part]
    cands = [(x, it, d, t, None) for x, it, d, t, _ in runs]
    scores = [float(score(c[0])) if score is not None else float(c[2][-1]) for c in cands]
    best = argmin_strict(scores)
    if best is None:
        raise ValueError(f"no candidate has a finite score below +inf: {scores} (the reference "
                         "would call sgp_betaDiv with betaParam=None)")
    info = {"betas": betas, "scores": scores, "best_beta": betas[best], "best": best,
            "beta_final": [r[4]["beta"] for r in runs], "candidates": cands}
    if final_solve:
        # the application's final sgp_betaDiv call repeats the best candidate's
        # run: its sgp.log lines (sgp.py:748-882) and its two prints (:892-893)
        runs[best][4]["log"]()
        print(f'Beta parameter in beta-divergence (final value): {runs[best][4]["beta"]}')
        print(f'No. of iterations: {cands[best][1]}')
    return cands[best], info
