"""CPU baseline worker for bench.py (TEST/BENCH INFRASTRUCTURE: the timed CPU
leg runs the numpy oracle, a port of the reference, on the same synthetic
workload).  Imports no torch so spawned pool workers start fast."""
import os
import time

import numpy as np


def gaussian_psf(k, fwhm=None):
    fwhm = k / 4.0 if fwhm is None else fwhm
    sig = fwhm / 2.354820045030949
    c = (k - 1) / 2.0
    yy, xx = np.mgrid[0:k, 0:k]
    p = np.exp(-((yy - c) ** 2 + (xx - c) ** 2) / (2 * sig * sig))
    return p / p.sum()


def embed_psf(psf, n):
    """A k x k PSF placed in an n x n array around (n//2, n//2): the circular
    A of sgp.py:108-120 needs psf.shape == image shape."""
    k = psf.shape[0]
    full = np.zeros((n, n))
    o = n // 2 - k // 2
    full[o:o + k, o:o + k] = psf
    return full / full.sum()


def make_stamp(seed, n, k, nstars, bkg=100.0, circular=False):
    from scipy.signal import fftconvolve
    rng = np.random.default_rng(seed)
    obj = np.zeros((n, n))
    p = rng.integers(0, n, (nstars, 2))
    np.add.at(obj, (p[:, 0], p[:, 1]), rng.pareto(1.5, nstars) * 1000 + 100)
    psf = gaussian_psf(k)
    if circular:
        psf = embed_psf(psf, n)
        tf = np.fft.rfft2(np.fft.fftshift(psf))
        blurred = np.fft.irfft2(tf * np.fft.rfft2(obj), s=obj.shape)
    else:
        blurred = fftconvolve(obj, psf, mode="same")
    gn = rng.poisson(np.clip(blurred, 0, None) + bkg).astype(float)
    return gn, psf


def warm(_):
    import sgp_oracle  # noqa: F401
    import scipy.signal  # noqa: F401
    return os.getpid()


def solve_one(args):
    """One C3-style beta-SGP solve with the oracle; returns (iters, seconds)."""
    seed, n, k, nstars, kw = args
    import sgp_oracle
    gn, psf = make_stamp(seed, n, k, nstars, circular=kw["use_original_SGP_Afunction"])
    t = time.perf_counter()
    _, it, _, _, _ = sgp_oracle.sgp_betaDiv(gn, psf, np.float64(100.0), **kw)
    return it, time.perf_counter() - t


def run_pool(n, k, nstars, images, kw, workers):
    import multiprocessing as mp
    os.environ["OMP_NUM_THREADS"] = "1"
    os.environ["OPENBLAS_NUM_THREADS"] = "1"
    ctx = mp.get_context("spawn")
    with ctx.Pool(workers) as pool:
        pool.map(warm, range(workers))
        t0 = time.perf_counter()
        res = pool.map(solve_one, [(10_000 + i, n, k, nstars, kw) for i in range(images)],
                       chunksize=1)
        wall = time.perf_counter() - t0
    return sum(r[0] for r in res), wall, sum(r[1] for r in res)


def solve_job(args):
    """One star-stamp solve with the oracle (bench.py stamps31 / stamps31_kl):
    (cutout, psf, bkg, flux, beta or None for KL, kwargs) -> (iters, seconds)."""
    cut, psf, bkg, flux, beta, kw = args
    import sgp_oracle
    t = time.perf_counter()
    if beta is None:  # the KL branch (application_sgp_star_stamps.py:107-112)
        _, it, _, _, _ = sgp_oracle.sgp(cut, psf, np.float64(bkg), flux=np.float64(flux), **kw)
    else:
        _, it, _, _, _ = sgp_oracle.sgp_betaDiv(cut, psf, np.float64(bkg), flux=np.float64(flux),
                                                betaParam=beta, **kw)
    return it, time.perf_counter() - t


def run_pool_jobs(jobs, workers):
    import multiprocessing as mp
    os.environ["OMP_NUM_THREADS"] = "1"
    os.environ["OPENBLAS_NUM_THREADS"] = "1"
    ctx = mp.get_context("spawn")
    with ctx.Pool(workers) as pool:
        pool.map(warm, range(workers))
        t0 = time.perf_counter()
        res = pool.map(solve_job, jobs, chunksize=1)
        wall = time.perf_counter() - t0
    return sum(r[0] for r in res), wall, sum(r[1] for r in res)
