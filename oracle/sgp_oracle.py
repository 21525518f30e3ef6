"""CPU ORACLE — numpy restatement of the reference beta-SGP hot path.

TEST INFRASTRUCTURE ONLY.  Only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may import this module, and only as the
checker / the timed CPU baseline.  The product path (``beta-sgp_amd/``) never
imports it: it runs on the HIP library and fails loudly without it.

Pinned against golden vectors produced by the reference itself
(``tests/golden/make_golden.py``; checked by ``tests/test_oracle.py``):
NGC7027 KL/beta solves (rel. diff <= 1e-9), projectDF KATs with full line
coverage, betaDiv-family KATs, and astropy-4.3.1 ``convolve_fft`` A/AT
vectors for the linear operator.

Every function cites the reference lines it restates
(``/root/reference/restoration/...``).  The reference's own quirks are kept:
revert to ``prev_x`` on stop (sgp.py:424-425), ``fftshift`` on odd sizes
(sgp.py:109), AT = convolution with ``psf.conj().T`` in linear mode
(sgp.py:157), the approximate beta gradient (sgp.py:499), the
``x =`` / ``s =`` slip of flux_conserve_proj.py:122, ``tol**2`` only when
``verbose`` (sgp.py:291-294).
"""
import math

import numpy as np

EPSILON = np.finfo(float).eps  # flux_conserve_proj.py:5
DEFAULT_PARAMS = (1000, 1e-4, 0.4, 1e-5, 1e5, 1e1, 3, 0.5, 1)  # sgp.py:34


# ----------------------------------------------------------------- operators
def next_fast_len(n):
    """5-smooth size >= n (scipy next_fast_len for complex input)."""
    m = max(int(n), 1)
    while True:
        t = m
        for f in (2, 3, 5):
            while t % f == 0:
                t //= f
        if t == 1:
            return m
        m += 1


def convolve_fft_fill(array, kernel):
    """Restates astropy.convolution.convolve_fft(array, kernel,
    normalize_kernel=True, normalization_zero_tol=1e-4) with its defaults
    boundary='fill', fill_value=0, nan_treatment='interpolate', psf_pad=True,
    fft_pad=True (astropy 4.3.1 convolve.py:646-829), for finite inputs:
    kernel normalised by its sum, both padded to next_fast_len(shape sum),
    array centred, kernel ifftshift-ed, result divided by the weight image
    (ones convolved with the kernel) and cropped back.
    Called from sgp.py:138 (A) and sgp.py:157 (AT, kernel = psf.conj().T)."""
    array = np.asarray(array, dtype=complex)
    kernel = np.asarray(kernel, dtype=complex)
    kernel = kernel / kernel.sum()
    ash, ksh = array.shape, kernel.shape
    newshape = [next_fast_len(a + k) for a, k in zip(ash, ksh)]
    asl, ksl = [], []
    for nd, ad, kd in zip(newshape, ash, ksh):
        center = nd - (nd + 1) // 2
        asl.append(slice(center - ad // 2, center + (ad + 1) // 2))
        ksl.append(slice(center - kd // 2, center + (kd + 1) // 2))
    asl, ksl = tuple(asl), tuple(ksl)
    bigarray = np.zeros(newshape, dtype=complex)
    bigarray[asl] = array
    bigkernel = np.zeros(newshape, dtype=complex)
    bigkernel[ksl] = kernel
    kernfft = np.fft.fftn(np.fft.ifftshift(bigkernel))
    fftmult = np.fft.fftn(bigarray) * kernfft
    bigimwt = np.ones(newshape, dtype=complex)
    wtsm = np.fft.ifftn(np.fft.fftn(bigimwt) * kernfft)
    bigimwt[asl] = wtsm.real[asl]
    rifft = np.fft.ifftn(fftmult) / bigimwt
    return rifft[asl].real


def make_operators(psf, shape, circular):
    """A / AT of sgp.py:108-161 (identical at sgp.py:570-615)."""
    if circular:
        TF = np.fft.fftn(np.fft.fftshift(psf))  # sgp.py:109
        CTF = np.conj(TF)  # sgp.py:110

        def afun(x, tf):  # sgp.py:111-117
            x = np.reshape(x, psf.shape)
            return np.real(np.fft.ifftn(np.multiply(tf, np.fft.fftn(x)))).flatten()

        return (lambda x: afun(x, TF)), (lambda x: afun(x, CTF))

    def A(x):  # sgp.py:122-139
        return convolve_fft_fill(np.reshape(x, shape), psf).ravel()

    def AT(x):  # sgp.py:141-158 — transpose, not a flip
        return convolve_fft_fill(np.reshape(x, shape), psf.conj().T).ravel()

    return A, AT


# ------------------------------------------------------------ beta-divergence
# Test hook: when True, the float32 terms x**beta and log(x) of a float32 image
# come from the C library's powf / logf (oracle/f32libm.c): the arithmetic of
# numpy 1.26 with its SIMD float32 kernels disabled, under which the reference
# made the ``_libm`` fixtures (tests/golden/make_golden.py), and the device's
# (bsgp_math.hpp libm_powf / libm_logf).  False (the default) is this numpy's
# own float32 power/log.
LIBM_F32 = False
_LIBM = []


def _is_f32(x):
    return isinstance(x, np.ndarray) and x.dtype.kind == "f" and x.dtype.itemsize == 4


def libm_lib():
    """oracle/_build/libf32libm.so (built by __graft_entry__.build(), or here
    with gcc when missing)."""
    if not _LIBM:
        import ctypes
        import os
        import subprocess
        here = os.path.dirname(os.path.abspath(__file__))
        so = os.path.join(here, "_build", "libf32libm.so")
        if not os.path.exists(so):
            os.makedirs(os.path.dirname(so), exist_ok=True)
            subprocess.run(["gcc", "-O2", "-shared", "-fPIC", os.path.join(here, "f32libm.c"),
                            "-o", so, "-lm"], check=True)
        lib = ctypes.CDLL(so)
        fp = ctypes.POINTER(ctypes.c_float)
        lib.bsgp_orc_powf.argtypes = [fp, ctypes.c_float, fp, ctypes.c_long]
        lib.bsgp_orc_logf.argtypes = [fp, fp, ctypes.c_long]
        _LIBM.append((lib, fp))
    return _LIBM[0]


def _libm_call(name, x, *extra):
    import ctypes
    lib, fp = libm_lib()
    xc = np.ascontiguousarray(x, dtype=np.float32)
    out = np.empty_like(xc)
    getattr(lib, name)(xc.ctypes.data_as(fp), *extra, out.ctypes.data_as(fp),
                       ctypes.c_long(xc.size))
    return out.reshape(np.shape(x))


def _pow(x, b):
    if LIBM_F32 and _is_f32(x):
        import ctypes
        return _libm_call("bsgp_orc_powf", x, ctypes.c_float(float(np.float32(b))))
    return x ** b


def _log(x):
    if LIBM_F32 and _is_f32(x):
        return _libm_call("bsgp_orc_logf", x)
    return np.log(x)


def betaDiv(y, x, betaParam):
    """sgp.py:441-458.  betaParam enters as a Python float: numpy 1.x (the
    reference's) casts a float64 SCALAR to a float32 array's dtype (value-based
    casting), as numpy 2 does for a Python float -- after an adaptive update
    (sgp.py:800) the reference's betaParam is a numpy float64, and the
    float32 terms of a float32 image (x ** betaParam) must stay float32."""
    betaParam = float(betaParam)
    if betaParam == 0:
        return np.sum(x / y) - np.sum(np.log(x / y)) - x.size
    elif betaParam == 1:
        return np.sum(np.multiply(x, np.log(np.divide(x, y)))) - np.sum(x) + np.sum(y)
    scal = 1 / (betaParam * (betaParam - 1))
    return (np.sum(scal * _pow(x, betaParam)) + np.sum(scal * (betaParam - 1) * y ** betaParam)
            - np.sum(scal * betaParam * x * y ** (betaParam - 1)))


def betaDivDeriv(y, x, betaParam):
    """sgp.py:462-495 (d betaDiv / d beta, elementwise)."""
    if betaParam == 0 or betaParam == 1:
        return 0
    b = float(betaParam)  # numpy 1.x scalar casting (see betaDiv)
    xb = _pow(x, b)
    return (-x * y ** (b - 1) * np.log(y) / (b - 1) + x * y ** (b - 1) / (b - 1) ** 2
            + xb * _log(x) / (b * (b - 1)) - xb / (b * (b - 1) ** 2)
            + y ** b * np.log(y) / b - xb / (b ** 2 * (b - 1)) - y ** b / b ** 2)


def betaDivDerivwrtY(AT, den_arg, gn_arg, betaParam):
    """sgp.py:498-499 (no AT on the first term)."""
    return den_arg ** (betaParam - 1) - AT(gn_arg * den_arg ** (betaParam - 2))


def lr_schedule(init_lr, k, epoch):
    """sgp.py:502-503."""
    return init_lr * math.exp(-k * epoch)


# ------------------------------------------------------------------ projection
def projectDF(b, c, dia, scaling, ccd_sat_level=None, lambda_=0, dlambda_=1, tol_lam=1e-11,
              biter=0, siter=0, max_projs=1000, stats=None):
    """flux_conserve_proj.py:7-144.  ``stats`` (optional dict) receives the
    number of x(lambda) evaluations under key 'evals'."""
    c = c.astype(np.float64, copy=False)
    dia = dia.astype(np.float64, copy=False)
    b = np.float64(b)
    tol_r = 1e-11 * b
    nev = [0]

    def xof(lam):
        nev[0] += 1
        x = np.maximum(0, np.divide(c + lam, dia))
        if ccd_sat_level is not None:
            x = np.minimum(ccd_sat_level / scaling - EPSILON, x)
        return x

    def done(x):
        if stats is not None:
            stats["evals"] = nev[0]
        return x

    x = xof(lambda_)  # :22-25
    r = np.sum(x) - b
    if abs(r) < tol_r:  # :27-28
        return done(x)
    if r < 0:  # :30-53
        lambdal = lambda_
        rl = r
        lambda_ = lambda_ + dlambda_
        x = xof(lambda_)
        r = np.sum(x) - b
        while r < 0:
            biter = biter + 1
            lambdal = lambda_
            s = np.max([rl / r - 1, 0.1])
            dlambda_ = dlambda_ + dlambda_ / s
            lambda_ = lambda_ + dlambda_
            rl = r
            x = xof(lambda_)
            r = np.sum(x) - b
        lambdau = lambda_
        ru = r
    else:  # :55-81
        lambdau = lambda_
        ru = r
        lambda_ = lambda_ - dlambda_
        x = xof(lambda_)
        r = np.sum(x) - b
        while r > 0:
            biter = biter + 1
            lambdau = lambda_
            s = np.max([ru / r - 1, 0.1])
            try:
                with np.errstate(all="raise"):
                    dlambda_ = dlambda_ + dlambda_ / s
            except Exception:
                break
            lambda_ = lambda_ - dlambda_
            ru = r
            x = xof(lambda_)
            r = np.sum(x) - b
        lambdal = lambda_
        rl = r
    if abs(ru) < tol_r:  # :84-88
        return done(xof(lambdau))
    if abs(rl) < tol_r:  # :89-93
        return done(xof(lambdal))
    s = 1 - rl / ru  # :96-102
    with np.errstate(divide="ignore", invalid="ignore"):
        dlambda_ = dlambda_ / s
    lambda_ = lambdau - dlambda_
    x = xof(lambda_)
    r = np.sum(x) - b
    maxit_s = max_projs - biter
    while abs(r) > tol_r and dlambda_ > tol_lam * (1 + abs(lambda_)) and siter < maxit_s:
        siter = siter + 1  # :106-142
        if r > 0:
            if s <= 2:
                lambdau = lambda_
                ru = r
                s = 1 - rl / ru
                dlambda_ = (lambdau - lambdal) / s
                lambda_ = lambdau - dlambda_
            else:
                s = np.max([ru / r - 1, 0.1])
                dlambda_ = (lambdau - lambda_) / s
                lambda_new = np.max([lambda_ - dlambda_, 0.75 * lambdal + 0.25 * lambda_])
                lambdau = lambda_
                ru = r
                lambda_ = lambda_new
                # :122 assigns x (immediately overwritten), leaving s as set above
        else:
            if s >= 2:
                lambdal = lambda_
                rl = r
                s = 1 - rl / ru
                dlambda_ = (lambdau - lambdal) / s
                lambda_ = lambdau - dlambda_
            else:
                s = np.max([rl / r - 1, 0.1])
                dlambda_ = (lambda_ - lambdal) / s
                lambda_new = np.min([lambda_ + dlambda_, 0.75 * lambdau + 0.25 * lambda_])
                lambdal = lambda_
                rl = r
                lambda_ = lambda_new
                s = (lambdau - lambdal) / (lambdau - lambda_)
        x = xof(lambda_)
        r = np.sum(x) - b
    return done(x)


# ---------------------------------------------------------------------- solver
def _np1_scalar_div(a, b):
    """Scalar a / b under numpy 1.x promotion (the reference's numpy; this
    module may run under numpy 2, whose NEP 50 rules differ for Python
    scalars): scalar-with-scalar promotes by type, a Python float is float64."""
    def dt(v):
        if isinstance(v, (np.generic, np.ndarray)):
            return np.asarray(v).dtype
        return np.dtype(np.float64) if isinstance(v, float) else np.dtype(np.int64)
    rt = np.promote_types(dt(a), dt(b))
    if rt.kind != "f":
        rt = np.dtype(np.float64)
    return rt.type(np.asarray(a, dtype=rt) / np.asarray(b, dtype=rt))


def _solve(gn, psf, bkg, *, variant, init_recon=0, proj_type=0, stop_criterion=0, MAXIT=500,
           gamma=1e-4, beta=0.4, alpha=1.3, alpha_min=1e-5, alpha_max=1e5, M_alpha=3, tau=0.5,
           M=1, max_projs=1000, verbose=True, flux=None, ccd_sat_level=None, scale_data=True,
           adapt_beta=True, betaParam=1.005, lr=1e-3, lr_exp_param=0.1, schedule_lr=False,
           tol_convergence=1e-4, use_original_SGP_Afunction=True, stats=None):
    """Shared body of sgp (sgp.py:41-438, variant 'kl') and sgp_betaDiv
    (sgp.py:506-895, variant 'beta').  Returns (x, iters, discr, times, None)
    plus, when ``stats`` is a dict, total projection evaluations 'E_p' and
    line-search evaluations 'E_ls'."""
    import time
    checkPSF = np.abs(np.sum(psf.flatten()) - 1.0)  # :97-102
    if checkPSF > 1e4 * np.finfo(float).eps:
        raise ValueError("PSF is not normalized! Provide a normalized PSF!")
    _shape = gn.shape
    init_lr = lr
    A, AT = make_operators(psf, _shape, use_original_SGP_Afunction)
    t0 = time.perf_counter()
    if init_recon == 0:  # :166-177
        x = np.zeros_like(gn)
    elif init_recon == 1:
        np.random.seed(42)
        x = np.random.randn(*gn.shape)
    elif init_recon == 2:
        x = gn.copy()
    else:
        x = (_np1_scalar_div(np.sum(gn - bkg), gn.size) * np.ones_like(gn) if flux is None
             else _np1_scalar_div(flux, gn.size) * np.ones_like(gn))
    gn = gn.flatten()  # :180-182
    x = x.flatten()
    bkg = np.asarray(bkg).flatten()
    if stop_criterion == 1:  # :185-190
        tol = []
    elif stop_criterion in (2, 3):
        tol = tol_convergence
    elif stop_criterion == 4:
        tol = 1 + 1 / float(np.mean(gn))  # numpy 1.x: int / float32 scalar -> float64
    if scale_data:  # :193-199 (arrays divided in their own dtype)
        scaling = np.max(gn)
        gn = gn / scaling
        bkg = bkg / scaling
        x = x / scaling
    else:
        scaling = 1.0
    sc64 = float(scaling)  # numpy 1.x: Python scalars with the float32 scaling give float64
    vmin = np.min(gn[gn > 0])  # :202-204
    eps = np.finfo(float).eps
    gn[gn <= 0] = vmin * eps * eps
    N = gn.size
    if flux is None:  # :208-211
        flux = np.sum(gn - bkg)
    else:
        flux = _np1_scalar_div(flux, scaling)
    iter_ = 1
    Valpha = alpha_max * np.ones(M_alpha)
    Fold = -1e30 * np.ones(M)
    Discr_coeff = 2 / N * sc64
    discr = np.zeros(MAXIT + 1)
    times = np.zeros(MAXIT + 1)
    E_p = 0
    E_ls = 0
    ls_trials = []  # line-search trials of every iteration (stats['ls_trials'])
    pst = {}
    if proj_type == 0:  # :248-253
        x[x < 0] = 0
    else:
        x = projectDF(flux, x, np.ones_like(x), sc64, ccd_sat_level=ccd_sat_level,
                      max_projs=max_projs)
    x_tf = A(x)  # :260-265 / :702-709
    den = x_tf + bkg
    if variant == "kl":
        temp = np.divide(gn, den)
        g = 1.0 - AT(temp)
        fv = np.sum(np.multiply(gn, np.log(temp))) + np.sum(x_tf) - flux
    else:
        g = betaDivDerivwrtY(AT, den, gn, betaParam)
        fv = betaDiv(den, gn, betaParam)
    y = np.multiply((flux / (flux + bkg)), AT(gn))  # :268-273
    X_low_bound = np.min(y[y > 0])
    X_upp_bound = np.max(y)
    if X_upp_bound / X_low_bound < 50:
        X_low_bound = X_low_bound / 10
        X_upp_bound = X_upp_bound * 10
    discr[0] = Discr_coeff * fv
    if init_recon == 0:  # :279-285
        X = np.ones_like(x)
    else:
        X = x.copy()
        X[X < X_low_bound] = X_low_bound
        X[X > X_upp_bound] = X_upp_bound
    if proj_type == 1:
        D = np.divide(1, X)
    if verbose and stop_criterion == 2:  # :291-294
        tol = tol * tol
    loop = True
    epoch = 0
    while loop:  # :302-425 / :748-882
        epoch += 1
        prev_x = x.copy()
        Valpha[0:M_alpha - 1] = Valpha[1:M_alpha]
        Fold[0:M - 1] = Fold[1:M]
        Fold[M - 1] = fv
        y = x - alpha * np.multiply(X, g)
        if proj_type == 0:
            y[y < 0] = 0
        else:
            st = {}
            y = projectDF(flux, np.multiply(y, D), D, sc64, ccd_sat_level=ccd_sat_level,
                          max_projs=max_projs, stats=st)
            E_p += st["evals"]
        d = y - x
        gd = np.dot(d, g)
        lam = 1
        fcontinue = 1
        d_tf = A(d)
        fr = max(Fold)
        E_ls0 = E_ls
        while fcontinue:
            E_ls += 1
            xplus = x + lam * d
            x_tf_try = x_tf + lam * d_tf
            den = x_tf_try + bkg
            if variant == "kl":
                temp = np.divide(gn, den)
                fv = np.sum(np.multiply(gn, np.log(temp))) + np.sum(x_tf_try) - flux
            else:
                fv = betaDiv(den, gn, betaParam)
            if fv <= fr + gamma * lam * gd or lam < 1e-12:
                x = xplus.copy()
                sk = lam * d
                x_tf = x_tf_try
                gtemp = (1.0 - AT(temp)) if variant == "kl" else betaDivDerivwrtY(AT, den, gn,
                                                                                  betaParam)
                yk = gtemp - g
                g = gtemp.copy()
                fcontinue = 0
                ls_trials.append(E_ls - E_ls0)
            else:
                lam = lam * beta
                if variant == "beta" and adapt_beta:  # :798-800
                    bgrad = betaDivDeriv(den, gn, betaParam).mean()
                    betaParam = betaParam - lr * bgrad
        X = x.copy()  # :355-386
        X[X < X_low_bound] = X_low_bound
        X[X > X_upp_bound] = X_upp_bound
        D = np.divide(1, X)
        sk2 = np.multiply(sk, D)
        yk2 = np.multiply(yk, X)
        bk = np.dot(sk2, yk)
        ck = np.dot(yk2, sk)
        if bk <= 0:
            alpha1 = min(10 * alpha, alpha_max)
        else:
            alpha1 = min(alpha_max, max(alpha_min, np.sum(np.dot(sk2, sk2)) / bk))
        if ck <= 0:
            alpha2 = min(10 * alpha, alpha_max)
        else:
            alpha2 = min(alpha_max, max(alpha_min, ck / np.sum(np.dot(yk2, yk2))))
        Valpha[M_alpha - 1] = alpha2
        if iter_ <= 20:
            alpha = min(Valpha)
        elif alpha2 / alpha1 < tau:
            alpha = min(Valpha)
            tau = tau * 0.9
        else:
            alpha = alpha1
            tau = tau * 1.1
        if variant == "beta" and schedule_lr:  # :842-844
            lr = lr_schedule(init_lr, lr_exp_param, epoch)
        iter_ += 1  # :390-392
        times[iter_ - 1] = time.perf_counter() - t0
        discr[iter_ - 1] = Discr_coeff * fv
        if stop_criterion == 2:  # :399-411
            loop = np.dot(sk, sk) / np.dot(x, x) > tol
        elif stop_criterion == 3:
            reldecrease = (Fold[M - 1] - fv) / fv
            loop = reldecrease > tol and reldecrease >= 0
        elif stop_criterion == 4:
            loop = discr[iter_ - 1] > tol
        if iter_ > MAXIT:  # :413-414
            loop = False
        if not loop:  # :424-425
            x = prev_x
        if variant == "beta" and epoch == MAXIT:  # :881-882
            break
    x = x.reshape(_shape) * scaling
    if stats is not None:
        stats.update(E_p=E_p, E_ls=E_ls, beta=betaParam, ls_trials=ls_trials)
    return x, iter_ - 1, discr[0:iter_], times[0:iter_], None


def sgp(gn, psf, bkg, init_recon=0, proj_type=0, stop_criterion=0, MAXIT=500, gamma=1e-4,
        beta=0.4, alpha=1.3, alpha_min=1e-5, alpha_max=1e5, M_alpha=3, tau=0.5, M=1,
        max_projs=1000, save=False, obj=None, verbose=True, flux=None, ccd_sat_level=None,
        scale_data=True, errflag=False, tol_convergence=1e-4, use_original_SGP_Afunction=True,
        stats=None):
    """sgp.py:41-438 (KL objective)."""
    return _solve(gn, psf, bkg, variant="kl", init_recon=init_recon, proj_type=proj_type,
                  stop_criterion=stop_criterion, MAXIT=MAXIT, gamma=gamma, beta=beta,
                  alpha=alpha, alpha_min=alpha_min, alpha_max=alpha_max, M_alpha=M_alpha,
                  tau=tau, M=M, max_projs=max_projs, verbose=verbose, flux=flux,
                  ccd_sat_level=ccd_sat_level, scale_data=scale_data,
                  tol_convergence=tol_convergence,
                  use_original_SGP_Afunction=use_original_SGP_Afunction, stats=stats)


def sgp_betaDiv(gn, psf, bkg, init_recon=0, proj_type=0, stop_criterion=0, MAXIT=500,
                gamma=1e-4, beta=0.4, alpha=1.3, alpha_min=1e-5, alpha_max=1e5, M_alpha=3,
                tau=0.5, M=1, max_projs=1000, save=False, obj=None, verbose=True, flux=None,
                ccd_sat_level=None, scale_data=True, errflag=False, adapt_beta=True,
                betaParam=1.005, lr=1e-3, lr_exp_param=0.1, schedule_lr=False,
                tol_convergence=1e-4, use_original_SGP_Afunction=True, stats=None):
    """sgp.py:506-895 (beta-divergence objective)."""
    return _solve(gn, psf, bkg, variant="beta", init_recon=init_recon, proj_type=proj_type,
                  stop_criterion=stop_criterion, MAXIT=MAXIT, gamma=gamma, beta=beta,
                  alpha=alpha, alpha_min=alpha_min, alpha_max=alpha_max, M_alpha=M_alpha,
                  tau=tau, M=M, max_projs=max_projs, verbose=verbose, flux=flux,
                  ccd_sat_level=ccd_sat_level, scale_data=scale_data, adapt_beta=adapt_beta,
                  betaParam=betaParam, lr=lr, lr_exp_param=lr_exp_param,
                  schedule_lr=schedule_lr, tol_convergence=tol_convergence,
                  use_original_SGP_Afunction=use_original_SGP_Afunction, stats=stats)
