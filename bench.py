"""Benchmark: SGP iterations/s (fp64) on batched 256x256 images + %HBM peak.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c3|c2|c4|c5] ...

A *step* is one complete batched solve (BASELINE config C3: 1024 independent
256x256 star-field stamps per GPU, beta-SGP, fp64, 25x25 Gaussian PSF with the
astropy-semantics linear A, flux-conserving projection, MAXIT iterations with
stop_criterion=1 so every image runs exactly MAXIT iterations).
Inputs are synthetic (SURVEY §8d generator), built on the device and resident
in HBM before timing starts.  ``value`` = image-iterations of all ranks /
max-over-ranks wall time of the K timed steps.

Multi-GPU: one process per GPU.  Under torchrun the ranks come
from RANK/LOCAL_RANK/WORLD_SIZE; ``--gpus N`` without torchrun starts the N
rank processes itself (before this process touches a GPU).  Each rank solves
its own shard of independent images with no collective on the data path; the
harness's barrier and its max/sum of two scalars run over gloo (CPU).  C3 is
weak scaling (1024 images per GPU); C5 is BASELINE config 5, 8192 images
split over the ranks (strong scaling; 1024 per GPU at N=8).

roofline: from a profiled solve after the timed loop (one stream, a HIP event
pair around every kernel launch, bsgp_solve_profiled): each kernel class's
span per launch and its algorithmic bytes per launch (the HBM bytes of the
passes that kernel makes, from the device's pass counters); the
reported kernel is the one with the largest share of the solve.  traffic:
PMC-measured HBM bytes per launch of that kernel (profiles/traffic_<config>.json,
scripts/gpu_traffic.sh) when present.
cpu_baseline: the numpy oracle (oracle/sgp_oracle.py, a port of the reference)
on a bounded sample of the same workload, a process pool on this host's cores
(capped at the 16 cores a one-GPU share of the box has).
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for p in (ROOT, os.path.join(ROOT, "beta-sgp_amd"), os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402

torch = None  # imported in main() before libbsgp (one HIP runtime per process); kept
#               out of module scope so spawned CPU-baseline workers stay light

HBM_PEAK_GBS = 8000.0
CPU_CAP = 16  # host cores of a one-GPU share of the box


def gaussian_psf(k, fwhm=None):
    fwhm = k / 4.0 if fwhm is None else fwhm
    sig = fwhm / 2.354820045030949
    c = (k - 1) / 2.0
    yy, xx = np.mgrid[0:k, 0:k]
    p = np.exp(-((yy - c) ** 2 + (xx - c) ** 2) / (2 * sig * sig))
    return p / p.sum()


def embed_psf(psf, n):
    """k x k PSF placed around (n//2, n//2) of an n x n array: the circular A
    (sgp.py:108-120) needs psf.shape == image shape."""
    k = psf.shape[0]
    full = np.zeros((n, n))
    o = n // 2 - k // 2
    full[o:o + k, o:o + k] = psf
    return full / full.sum()


# SURVEY §8d configurations (C1 is the reference's own NGC7027 CPU case).
# batch: images per GPU (weak scaling); total: images of the whole job (strong).
CONFIGS = {
    "c2": dict(n=256, k=25, nstars=200, batch=1, circular=False,
               desc="single {n}x{n} synthetic image, 25x25 Gaussian PSF, linear A"),
    "c3": dict(n=256, k=25, nstars=200, batch=1024, circular=False,
               desc="{B} independent {n}x{n} stamps per GPU, 25x25 PSF, linear A"),
    "c4": dict(n=2048, k=64, nstars=5000, batch=1, circular=True,
               desc="single {n}x{n} synthetic field, 64x64 PSF embedded at the centre, "
                    "circular A (pow-2 FFT)"),
    "c5": dict(n=256, k=25, nstars=200, total=8192, circular=False,
               desc="{T} independent {n}x{n} subdivisions split over the GPUs ({B} on this "
                    "rank), 25x25 PSF, linear A"),
    # the application's subdivision tiles (application_sgp_subdivisions.py:43-107
    # cuts 375x375 tiles): a 400-point grid, cooperative transforms
    # 1024 tiles: per-wave transforms at three workgroups per CU hold 768
    # images at once, so a launch of 1024 keeps every slot busy to the end
    "sub375": dict(n=375, k=31, nstars=300, batch=1024, circular=False,
                   desc="{B} independent {n}x{n} subdivision-size tiles, 31x31 PSF, linear A"),
    # the application's CROWDED mode solves its whole 450x450 frame
    # (application_sgp_subdivisions.py:22,44-50): a 480-point grid; published
    # reference rates 4.98 beta-SGP / 3.50 KL it/s for one frame
    # (results/CROWDED_SUBDIV_EXEC_TIME*.npy, NUM_ITERS*.npy; hardware unstated)
    "sub450": dict(n=450, k=31, nstars=400, batch=512, circular=False,
                   desc="{B} independent {n}x{n} CROWDED-frame-size tiles, 31x31 PSF, linear A"),
    # application_sgp_star_stamps.py:56-105: 31x31 float32 cutouts around stars,
    # the DIAPL PSF with the default circular A, adaptive beta, stop rule 3, the
    # five seeds; the reference's only first-party throughput figure
    "stamps31": dict(n=31, k=31, nstars=0, batch=16384, circular=True, stamps=True, maxit=500,
                     desc="{B} float32 31x31 star stamps (cutouts of results/SUBDIV_ORIGIMG.fits "
                          "at bright pixels) x the application's 5 seeds, DIAPL 31x31 PSF, "
                          "circular A"),
    # the same stamps through the application's KL branch (USE_BETADIV False,
    # application_sgp_star_stamps.py:107-112): sgp(...), stop rule 3, no seeds
    "stamps31_kl": dict(n=31, k=31, nstars=0, batch=16384, circular=True, stamps=True, kl=True,
                        maxit=500,
                        desc="{B} float32 31x31 star stamps (cutouts of results/SUBDIV_ORIGIMG.fits "
                             "at bright pixels), KL SGP, DIAPL 31x31 PSF, circular A"),
}
STAMP_PUBLISHED = 1167.5  # it/s, beta-SGP star stamps (results/EXEC_TIME_BETA.npy, NUM_ITERS_BETA.npy)
STAMP_KL_PUBLISHED = 1436.7  # it/s, KL star stamps (results/EXEC_TIME.npy, NUM_ITERS.npy)
# the reference's own published single-frame rates for the subdivision application (context
# only: one image on unstated hardware, so vs_baseline stays null for these lines)
PUBLISHED_CONTEXT = {
    "sub375": "reference: one 375x375 subdivision, beta-SGP 43 iterations in 6.70 s = 6.42 it/s, "
              "KL 51 in 6.54 s = 7.80 it/s (results/SUBDIV_EXEC_TIME*.npy, SUBDIV_NUM_ITERS*.npy; "
              "hardware unstated)",
    "sub450": "reference: the 450x450 CROWDED frame, beta-SGP 51 iterations in 10.25 s = 4.98 it/s, "
              "KL 2 in 0.571 s = 3.50 it/s (results/CROWDED_SUBDIV_EXEC_TIME*.npy, "
              "CROWDED_SUBDIV_NUM_ITERS*.npy; hardware unstated)",
}


def stamp_inputs(B, seed=0):
    """B star-stamp solves as application_sgp_star_stamps.py:56-105 makes
    them: 31x31 float32 cutouts (Cutout2D at integer centres = slices) of the
    reference's float32 frame results/SUBDIV_ORIGIMG.fits around bright
    pixels (the brightest 2 % of the frame, drawn with replacement; stamps
    with flux <= 0 redrawn), each with
    its float64 median as background and sum(cutout - bkg) as flux (stand-ins
    for photutils' background_median and segment_flux), cycling through the
    application's five seeds; the 31x31 DIAPL PSF.  Returns host arrays."""
    import fits_io
    gold = os.path.join(ROOT, "tests", "golden")
    _, img = fits_io.read_fits(os.path.join(gold, "SUBDIV_ORIGIMG.fits"))
    _, psf = fits_io.read_fits(os.path.join(gold, "psfccfbrd210048_1_1_img.fits"))
    a = np.asarray(img, dtype=np.float32)
    inner = a[15:-15, 15:-15]
    thr = np.quantile(inner, 0.98)
    rows, cols = np.nonzero(inner >= thr)
    rng = np.random.default_rng(seed)
    pick = rng.integers(0, len(rows), B)

    def cut(p):
        c = np.stack([a[r:r + 31, c_:c_ + 31] for r, c_ in zip(rows[p], cols[p])])
        b = np.median(c.reshape(len(p), -1).astype(np.float64), axis=1)
        return c, b, np.sum(c.astype(np.float64) - b[:, None, None], axis=(1, 2))

    cuts, bkg, flux = cut(pick)
    # a source's segment flux is positive; a bright pixel inside a stamp whose
    # median exceeds its mean (a hot pixel on a dip) is no star: redrawn, as
    # the reference raises on it (no positive entry in flux/(flux+bkg)*AT(gn))
    bad = np.nonzero(flux <= 0)[0]
    while bad.size:
        pick[bad] = rng.integers(0, len(rows), bad.size)
        cuts[bad], bkg[bad], flux[bad] = cut(pick[bad])
        bad = bad[flux[bad] <= 0]
    seeds = (0, 42, 951, 93, 810)  # application_sgp_star_stamps.py:69-75
    betas = []
    for s_ in seeds:
        np.random.seed(s_)
        betas.append(np.random.normal(loc=1, scale=0.05))
    return cuts, np.asarray(psf, dtype=np.float64), bkg, flux, np.resize(np.asarray(betas), B)


def stamp_kwargs(maxit, kl=False):
    """application_sgp_star_stamps.py:82-90 (DEFAULT_PARAMS unpacked, sgp.py:34);
    kl: the sgp(...) call of its KL branch (:107-112), no beta keywords."""
    kw = dict(gamma=1e-4, beta=0.4, alpha_min=1e-5, alpha_max=1e5, alpha=10.0, M_alpha=3,
              tau=0.5, M=1, proj_type=1, max_projs=1000, init_recon=2, stop_criterion=3,
              MAXIT=maxit, ccd_sat_level=65000, scale_data=True, use_original_SGP_Afunction=True)
    if not kl:
        kw.update(lr=1e-3, lr_exp_param=0.1, schedule_lr=True, adapt_beta=True)
    return kw


def synth_batch(B, n, k, nstars, seed0, bkg=100.0, circular=False):
    """SURVEY §8d synthetic stamps, generated on the device: point sources
    (pareto fluxes) blurred by the engine's own A, plus Poisson noise."""
    import _bsgp
    psf = gaussian_psf(k)
    if circular:
        psf = embed_psf(psf, n)
    plan = _bsgp.get_plan(n, n, psf, _bsgp.BSGP_CONV_CIRCULAR if circular
                          else _bsgp.BSGP_CONV_LINEAR_FILL)
    pos = np.empty((B, nstars), dtype=np.int64)
    flx = np.empty((B, nstars))
    for i in range(B):
        rng = np.random.default_rng(seed0 + i)
        p = rng.integers(0, n, (nstars, 2))
        pos[i] = p[:, 0] * n + p[:, 1]
        flx[i] = rng.pareto(1.5, nstars) * 1000 + 100
    obj = torch.zeros(B, n * n, dtype=torch.float64, device="cuda")
    obj.scatter_add_(1, torch.from_numpy(pos).cuda(), torch.from_numpy(flx).cuda())
    blurred = plan.apply(obj.view(B, n, n)).clamp_min(0)
    g = torch.Generator(device="cuda")
    g.manual_seed(seed0 + 12345)
    gn = torch.poisson(blurred + bkg, generator=g)
    return gn.contiguous(), psf


def solve_kwargs(maxit, ls_spec, streams=None, team=None, circular=False, proj_cache=None,
                 storage="f64", persistent=None, stop3=False):
    max_projs, gamma, beta, alpha_min, alpha_max, alpha, M_alpha, tau, M = (
        1000, 1e-4, 0.4, 1e-5, 1e5, 1e1, 3, 0.5, 1)  # sgp.DEFAULT_PARAMS (sgp.py:34)
    return dict(init_recon=2, proj_type=1, stop_criterion=3 if stop3 else 1, MAXIT=maxit,
                tol_convergence=1e-5, gamma=gamma, beta=beta,
                alpha=alpha, alpha_min=alpha_min, alpha_max=alpha_max, M_alpha=M_alpha, tau=tau,
                M=M, max_projs=max_projs, ccd_sat_level=65000.0, scale_data=True,
                use_original_SGP_Afunction=circular, adapt_beta=False, betaParam=1.05, lr=1e-3,
                lr_exp_param=0.1, schedule_lr=True, ls_spec=ls_spec, streams=streams,
                team=team, proj_cache=proj_cache, storage=storage, persistent=persistent)


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(n, k, nstars, images, maxit, workers, circular=False):
    """Oracle (numpy port of the reference, oracle/sgp_oracle.py) on `images`
    stamps x `maxit` iterations, one image per task on `workers` processes;
    wall time of the solve phase (pool already warm, inputs built in-task)."""
    import cpu_bench
    kw = solve_kwargs(maxit, None, circular=circular)
    for key in ("ls_spec", "team", "streams", "proj_cache", "storage", "persistent"):
        kw.pop(key)
    iters, wall, cpu_s = cpu_bench.run_pool(n, k, nstars, images, kw, workers)
    ncpu = os.cpu_count() or 1
    return {"value": iters / wall, "unit": "image-iterations/s", "cores": workers,
            "kind": "port",
            "cpu_model": cpu_model(), "host_cpus": ncpu,
            "sample": f"{images} images {n}x{n} (bench generator) x {maxit} beta-SGP iterations "
                      f"with oracle/sgp_oracle.py, one image per process on {workers} processes "
                      f"({cpu_model()}; the host shows {ncpu} CPUs, a one-GPU share is "
                      f"{CPU_CAP}): {iters} image-iterations in {wall:.1f}s wall "
                      f"({iters / cpu_s:.1f} image-it/s per core)"}


def cpu_baseline_stamps(kw, images, workers, kl=False):
    """The oracle on `images` stamps of the same stamp workload, one stamp per
    task on `workers` processes."""
    import cpu_bench
    cuts, psf, bk, fl, betas = stamp_inputs(images, seed=777)
    okw = {k_: v for k_, v in kw.items() if k_ in stamp_kwargs(1, kl)}
    jobs = [(cuts[i], psf, float(bk[i]), float(fl[i]), None if kl else float(betas[i]), okw)
            for i in range(images)]
    iters, wall, cpu_s = cpu_bench.run_pool_jobs(jobs, workers)
    ncpu = os.cpu_count() or 1
    return {"value": iters / wall, "unit": "image-iterations/s", "cores": workers,
            "kind": "port", "cpu_model": cpu_model(), "host_cpus": ncpu,
            "sample": f"{images} float32 31x31 stamps of the same workload "
                      f"({'KL' if kl else 'adaptive beta'}, stop 3) with oracle/sgp_oracle.py, one stamp per process on {workers} "
                      f"processes ({cpu_model()}): {iters} image-iterations in {wall:.1f}s wall "
                      f"({iters / cpu_s:.1f} image-it/s per core)"}


def shard_seed0(rank, images_per_rank):
    """Rank r solves images [r*B, (r+1)*B) of the synthetic stream: disjoint
    shards, no data-path collective."""
    return rank * images_per_rank


def shard_bounds(total, world, rank):
    """Contiguous shard [lo, hi) of `total` images for `rank` of `world` (C5)."""
    return total * rank // world, total * (rank + 1) // world


def aggregate(dist, elapsed, iters_sum, device="cpu"):
    """Cross-rank reduction of one timed run: the max wall time over ranks and
    the total image-iterations of all ranks (the only collectives of the
    harness, on CPU tensors over gloo)."""
    t = torch.tensor([float(elapsed)], dtype=torch.float64, device=device)
    n = torch.tensor([float(iters_sum)], dtype=torch.float64, device=device)
    if dist is not None:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dist.all_reduce(n, op=dist.ReduceOp.SUM)
    return float(t.item()), float(n.item())


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n, argv, poll_s=0.2):
    """`--gpus N` without torchrun: start one rank process per GPU (this
    process has not touched a GPU) and poll them.  As soon as one rank exits
    non-zero the others are terminated (a rank that died before or after the
    gloo rendezvous would otherwise leave its peers blocked until the
    rendezvous / collective timeout) and its exit code is returned; 0 when
    every rank succeeded.  Rank 0 prints the JSON line."""
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *argv], env=env))
    live = list(procs)
    while live:
        for p in list(live):
            rc = p.poll()
            if rc is None:
                continue
            live.remove(p)
            if rc != 0:
                for q in live:
                    q.terminate()
                for q in live:
                    try:
                        q.wait(timeout=10)
                    except subprocess.TimeoutExpired:
                        q.kill()
                        q.wait()
                print(f"bench: rank {procs.index(p)} exited with {rc}; stopped the other ranks",
                      file=sys.stderr, flush=True)
                return rc
        time.sleep(poll_s)
    return 0


APP_PUBLISHED = 6.42  # it/s: the reference's one 375x375 subdivision, beta-SGP (SUBDIV_EXEC_TIME_BETA.npy)


def app375_inputs():
    """The application's own call (application_sgp_subdivisions.py:69-107): the
    375x375 big-endian float32 subdivision results/SUBDIV_ORIGIMG.fits as
    fits.getdata returns it, the >f8 31x31 DIAPL PSF, a per-pixel background
    map (photutils' Background2D is absent: the smoothed-median map of
    tests/golden/make_golden.py app) and the flux, with the application's
    keyword arguments (linear A, projection, stop rule 3 at tol 1e-5, fixed
    beta) and its five seeds.  Host arrays, from tests/golden (the copies
    the GPU box has)."""
    z = np.load(os.path.join(ROOT, "tests", "golden", "app_subdiv_inputs.npz"))
    kw = dict(gamma=1e-4, beta=0.4, alpha_min=1e-5, alpha_max=1e5, alpha=10.0, M_alpha=3,
              tau=0.5, M=1, proj_type=1, max_projs=1000, init_recon=2, stop_criterion=3,
              save=False, verbose=True, ccd_sat_level=65000, scale_data=True, lr=1e-3,
              lr_exp_param=0.1, schedule_lr=True, adapt_beta=False,
              use_original_SGP_Afunction=False, tol_convergence=1e-5,
              flux=np.float64(z["flux"]))
    return z["img"], z["psf"], z["bkg"], kw, [float(b) for b in z["betas"]]


def bench_app375(args):
    """--config app375: the drop-in at the application's real call shape, one
    subdivision at a time, end to end from host arrays (the application's own
    timing covers one sgp_betaDiv call, SUBDIV_EXEC_TIME_BETA.npy):
    (a) value: sgp_betaDiv on the one image (seed 0), iterations / wall s;
    (b) multistart: sgp_betaDiv_multistart, the five seed candidates as one
        batched launch (the application's five calls + its final re-solve,
        which repeats the best candidate's run and is returned without
        solving again), candidate iterations / wall s;
    with the GPU span of the solve (HIP events) beside the wall, the oracle
    (a port of the reference) timed on the same call on one host core, and
    the reference's published 6.42 it/s as context."""
    import contextlib
    import io
    import sgp
    torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))
    img, psf, bkg, kw, betas = app375_inputs()
    quiet = contextlib.redirect_stdout(io.StringIO())  # the drop-in prints as the reference does
    quiet.__enter__()
    kw1 = dict(kw, betaParam=betas[0])
    for _ in range(max(1, args.warmup)):
        sgp.sgp_betaDiv(img, psf, bkg, **kw1)
        sgp.sgp_betaDiv_multistart(img, psf, bkg, betas=betas, **kw)
    torch.cuda.synchronize()

    def timed(fn):
        walls, spans, its = [], [], []
        for _ in range(args.steps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            t0 = time.perf_counter()
            e0.record()
            r = fn()
            e1.record()
            torch.cuda.synchronize()
            walls.append(time.perf_counter() - t0)
            spans.append(e0.elapsed_time(e1) * 1e-3)
            its.append(r)
        return float(np.median(walls)), float(np.median(spans)), its[-1]

    w1, g1, it1 = timed(lambda: sgp.sgp_betaDiv(img, psf, bkg, **kw1)[1])

    def ms():
        _, info = sgp.sgp_betaDiv_multistart(img, psf, bkg, betas=betas, **kw)
        return sum(c[1] for c in info["candidates"])
    wm, gm, itm = timed(ms)
    res = {
        "metric": "SGP iterations/sec (fp64) of the drop-in on one 375x375 float32 subdivision "
                  "(the application's call shape)",
        "value": it1 / w1, "unit": "iterations/s", "n_gpus": 1, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": w1 * 1e3, "higher_is_better": True,
        "scaling": "none (one image: latency-bound)", "vs_baseline": None,
        "dtype": "f64 (the reference's float32 prelude on float32 data)",
        "data": "the reference's results/SUBDIV_ORIGIMG.fits (>f4, tests/golden copy), its DIAPL "
                "PSF, a smoothed-median background map, flux from the published restored image",
        "config": {"workload": "APP375: application_sgp_subdivisions.py:84-91 on one 375x375 "
                               "subdivision: sgp_betaDiv, linear A (400-point grid), proj_type=1, "
                               "init_recon=2, stop_criterion=3 (tol 1e-5), beta fixed (seed 0)",
                   "iterations": int(it1), "gpu_span_ms": g1 * 1e3,
                   "host_share": 1.0 - g1 / w1},
        "multistart": {"what": "sgp_betaDiv_multistart: the five seeds as one batched launch",
                       "candidate_iterations": int(itm), "ms": wm * 1e3, "gpu_span_ms": gm * 1e3,
                       "value": itm / wm, "unit": "candidate iterations/s"},
        "context": PUBLISHED_CONTEXT["sub375"],
        "roofline": None, "cpu_baseline": None,
    }
    if not args.no_profile:
        import _bsgp
        g = torch.from_numpy(np.asarray(img, dtype=np.float32).copy()).cuda()[None]
        b = torch.from_numpy(np.asarray(bkg, dtype=np.float64)).cuda()[None]
        bk = {k_: v for k_, v in kw.items() if k_ not in ("save", "verbose", "flux")}
        prof = sgp.sgp_betaDiv_batch(g, psf, b, betaParams=[betas[0]], profile=True,
                                     flux=np.array([kw["flux"]]), **bk)
        names = ["k_setup", "k_dir", "k_col", "k_ls", "k_bb", "k_persist"]
        kms, nl = prof["kernel_ms"], prof["launches"]
        it = int(prof["iters"][0])
        res["roofline"] = {
            "note": "one image is latency-bound: per-kernel spans of the profiled solve (one "
                    "stream, HIP events around every launch); bytes per iteration ~ 245 B/px "
                    "x 375^2 = 34 MB, i.e. ~5 us of HBM time against the span below",
            "team": int(prof["counters"][0, 5]), "iterations": it,
            "us_per_iteration": {n_: float(kms[i] / max(it, 1) * 1e3) for i, n_ in enumerate(names)
                                 if i > 0 and nl[i] > 0},
            "profiled_solve_ms": float(np.sum(kms))}
    if not args.no_cpu:
        import sgp_oracle
        t0 = time.perf_counter()
        _, ito, _, _, _ = sgp_oracle.sgp_betaDiv(img, psf, bkg, **kw1)
        el = time.perf_counter() - t0
        res["cpu_baseline"] = {"value": ito / el, "unit": "iterations/s", "cores": 1,
                               "kind": "port", "cpu_model": cpu_model(),
                               "sample": f"the same call with oracle/sgp_oracle.py on one core: "
                                         f"{ito} iterations in {el:.2f} s"}
    quiet.__exit__(None, None, None)
    print(json.dumps(res), flush=True)


def kernel_bytes(H, W, P, Qh, counters, iters, beta, series, compact, bmap, fused_at_col,
                 vb=8.0):
    """Algorithmic HBM bytes of each kernel class over one solve: the passes
    each kernel makes over the per-image vectors (counted on the device) plus
    its spectrum traffic.  N = H*W pixels; vb = bytes of a
    stored iterate element (8, or 4 for float32 storage); gn is 4 B when kept
    compact; S = 16*H*Qh bytes of stored half spectrum; TF = 16*P*Qh bytes of
    transfer function.
      k_dir: (x, g) per projection pass + 16 B per list entry read; (x, g)
             for the direction and its row transforms; writes the spectrum.
      k_col: reads and writes the spectrum, reads the TF (A; AT too if unfused).
      k_ls:  pass 1 reads the spectrum, x_tf, gn, pw (series) [, bkg map] and
             writes d_tf; every further pass reads x_tf, d_tf, gn [, bkg];
             accept reads the same, writes x_tf, pw (beta) and the spectrum;
             AT's column pass (fused for one-workgroup images).
      k_bb:  reads the spectrum, pw (beta), x, g; writes x, g."""
    N = float(H * W)
    S, TF = 16.0 * H * Qh, 16.0 * P * Qh
    gb = 4.0 if compact else 8.0
    bb = 8.0 if bmap else 0.0
    it = float(np.sum(iters))
    proj_passes, list_reads = float(np.sum(counters[:, 6])), float(np.sum(counters[:, 7]))
    ls_passes = float(np.sum(counters[:, 2]))
    b = {}
    b["k_dir"] = 2.0 * vb * N * proj_passes + 16.0 * list_reads + it * (2.0 * vb * N + S)
    col_per = 2.0 * S + TF
    b["k_ls"] = (it * (S + N * (vb + gb + (vb if series else 0.0) + bb) + vb * N)
                 + (ls_passes - it) * N * (2.0 * vb + gb + bb)
                 + it * (N * (2.0 * vb + gb + bb) + N * (2.0 * vb if beta else vb) + S)
                 + (it * col_per if fused_at_col else 0.0))
    b["k_bb"] = it * (S + N * ((vb if beta else 0.0) + 2.0 * vb) + 2.0 * vb * N)
    b["k_col"] = it * col_per * (1.0 if fused_at_col else 2.0)
    # setup (once per image, k_setup or the persistent solver's first task):
    # raw statistics 8, scale 8+8, null fill + start x 8+8+8, the start's
    # projection with one evaluation and the clip (a lower bound: the setup's
    # evaluations are not counted on the device) 8+8+8, rows of x 8, rows of
    # A(x) with f, pw 8+8+8, rows of AT(w) pw + g 8+8, rows of gn 8, compact
    # gn 8+4 = 140 B/px; spectra: 7 row passes + three column passes 3(2S+TF)
    nimg = float(counters.shape[0])
    b["k_setup"] = nimg * (140.0 * N + 12.0 * S + 3.0 * TF)
    return b


def load_traffic(config):
    f = os.path.join(ROOT, "profiles", f"traffic_{config}.json")
    if os.path.exists(f):
        try:
            return json.load(open(f))
        except Exception:
            return None
    return None


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS) + ["app375"])
    ap.add_argument("--batch", type=int, default=None, help="images per GPU (c2/c3/c4)")
    ap.add_argument("--maxit", type=int, default=None, help="default 100 (500 for stamps31)")
    ap.add_argument("--ls-spec", type=int, default=None)
    ap.add_argument("--streams", type=int, default=None)
    ap.add_argument("--team", type=int, default=None,
                    help="workgroups per image (0/None = auto, 1 = one per image)")
    ap.add_argument("--proj-cache", type=int, default=None)
    ap.add_argument("--storage", default="f64", choices=["f64", "f32"])
    ap.add_argument("--persistent", type=int, default=None,
                    help="1: every iteration in one persistent launch (task queue), 0: phase "
                         "kernels per iteration (default: sgp.PERSIST_DEFAULT)")
    ap.add_argument("--stop3", action="store_true",
                    help="stop rule 3 (tol 1e-5, the application's) instead of stop rule 1")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-e2e", action="store_true",
                    help="skip the end-to-end solve (host inputs -> host outputs)")
    ap.add_argument("--no-profile", action="store_true",
                    help="skip the profiled solve (per-kernel roofline)")
    ap.add_argument("--cpu-images", type=int, default=16)
    ap.add_argument("--cpu-maxit", type=int, default=None,
                    help="iterations per CPU-baseline image (default: --maxit)")
    ap.add_argument("--stub", action="store_true",
                    help="harness only, no GPU: a fixed CPU wait stands in for each solve "
                         "(tests of the multi-rank path)")
    ap.add_argument("--stub-fail-rank", type=int, default=None,
                    help="with --stub: this rank exits 1 before the rendezvous (test of the "
                         "fail-fast launcher)")
    return ap.parse_args(argv)


def main():
    # 8 hardware queues for this process (read by the HIP runtime when torch
    # initialises it): the solve then runs 8 sub-batches instead of 4 (+2.8 % on
    # C3).  Set here, before torch is imported, and inherited by
    # spawned ranks; importing bench (tests/bench_path.py) leaves the
    # environment alone.
    os.environ["GPU_MAX_HW_QUEUES"] = os.environ.get("BSGP_BENCH_HW_QUEUES", "8")
    args = parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    global torch
    import torch as _torch
    torch = _torch
    if args.config == "app375":
        return bench_app375(args)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.stub and args.stub_fail_rank == rank:
        sys.exit(1)
    dist = None
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        import datetime
        # a peer that never arrives (or dies mid-run) fails the rendezvous or
        # the harness's collectives after this long instead of gloo's 30 min
        tmo = float(os.environ.get("BSGP_DIST_TIMEOUT_S", "300"))
        dist.init_process_group("gloo", rank=rank, world_size=world,
                                timeout=datetime.timedelta(seconds=tmo))

    cfg = CONFIGS[args.config]
    n, k, nstars, circ = cfg["n"], cfg["k"], cfg["nstars"], cfg["circular"]
    stamps = cfg.get("stamps", False)
    kl = cfg.get("kl", False)
    if args.maxit is None:
        args.maxit = cfg.get("maxit", 100)
    strong = "total" in cfg
    if strong:
        lo, hi = shard_bounds(cfg["total"], world, rank)
        B, seed0 = hi - lo, lo
    else:
        B = args.batch if args.batch else cfg["batch"]
        seed0 = shard_seed0(rank, B)
    kw = solve_kwargs(args.maxit, args.ls_spec, args.streams, args.team, circular=circ,
                      proj_cache=args.proj_cache, storage=args.storage,
                      persistent=args.persistent, stop3=args.stop3)
    if stamps:
        kw = dict(stamp_kwargs(args.maxit, kl), ls_spec=args.ls_spec, streams=args.streams,
                  team=args.team, proj_cache=args.proj_cache, storage=args.storage,
                  persistent=args.persistent)

    if args.stub:
        def step():
            time.sleep(0.01)
            return {"iters": np.full(B, args.maxit)}

        def sync():
            pass
    else:
        # BSGP_RANK_DEVICE: every rank on this one device (the multi-rank path
        # rehearsed on a one-GPU box, tests/test_gpu_multirank.py); set before
        # any GPU call of the rank
        dev_override = os.environ.get("BSGP_RANK_DEVICE")
        torch.cuda.set_device(int(dev_override) if dev_override is not None else local)
        import _bsgp
        import sgp
        if stamps:
            cuts, psf, bk_h, fl_h, betas = stamp_inputs(B, seed=seed0)
            gn = torch.from_numpy(cuts).cuda()  # float32: the reference's float32 arithmetic
            bkg = torch.from_numpy(bk_h).cuda()
            flux = torch.from_numpy(fl_h).cuda()
            extra = dict(flux=flux) if kl else dict(betaParams=betas, flux=flux)
        else:
            gn, psf = synth_batch(B, n, k, nstars, seed0=seed0, circular=circ)
            bkg = torch.full((B,), 100.0, dtype=torch.float64, device="cuda")
            extra = {}
        kw.update(extra)
        torch.cuda.synchronize()

        solve = sgp.sgp_batch if kl else sgp.sgp_betaDiv_batch

        def step():
            return solve(gn, psf, bkg, device_out=True, **kw)

        def sync():
            torch.cuda.synchronize()

    for _ in range(args.warmup):
        out = step()
    sync()
    if dist:
        dist.barrier()
    sync()
    ev = []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        if args.stub:
            out = step()
            continue
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        out = step()
        e1.record()
        ev.append((e0, e1))
    sync()
    if dist:
        dist.barrier()
    sync()
    elapsed = time.perf_counter() - t0
    iters = out["iters"].cpu().numpy() if torch.is_tensor(out["iters"]) else out["iters"]
    elapsed_max, tot = aggregate(dist, elapsed, iters.sum())
    total_iters = tot * args.steps
    value = total_iters / elapsed_max
    if dist:
        dist.destroy_process_group()
    if rank != 0:
        return

    if stamps:
        workload = (f"{args.config.upper()}: " + cfg["desc"].format(B=B)
                    + (", KL SGP" if kl else ", adaptive beta-SGP")
                    + f", proj_type=1, init_recon=2, MAXIT={args.maxit}, stop_criterion=3 (tol 1e-4)")
    else:
        workload = (f"{args.config.upper()}: "
                    + cfg["desc"].format(n=n, B=B, T=cfg.get("total", B))
                    + f", beta-SGP (beta=1.05), proj_type=1, MAXIT={args.maxit}, "
                      f"stop_criterion={kw['stop_criterion']}")
    result = {
        "metric": ("SGP iterations/sec (fp64) on batched 31x31 float32 star stamps" if stamps
                   else f"SGP iterations/sec (fp64) on batched {n}x{n} images"),
        "value": value,
        "unit": "image-iterations/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed_max / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "strong" if strong else "weak",
        "vs_baseline": (value / (STAMP_KL_PUBLISHED if kl else STAMP_PUBLISHED)) if stamps else None,
        "dtype": "f64" if args.storage == "f64" else "f32 storage, f64 arithmetic",
        "data": ("the reference's float32 frame results/SUBDIV_ORIGIMG.fits cut into 31x31 "
                 "stamps around its brightest pixels (tests/golden copy), its DIAPL PSF; "
                 + ("vs_baseline = value / 1436.7 it/s, the reference's published star-stamp "
                    "KL rate (results/EXEC_TIME.npy, NUM_ITERS.npy; hardware unstated)" if kl else
                    "vs_baseline = value / 1167.5 it/s, the reference's published star-stamp "
                    "beta-SGP rate (results/EXEC_TIME_BETA.npy, NUM_ITERS_BETA.npy; hardware "
                    "unstated)")) if stamps else
                "synthetic (SURVEY §8d generator: pareto point sources * 25x25 Gaussian PSF "
                "+ Poisson, bkg 100), built on device",
        "config": {"workload": workload, "images_per_gpu": B,
                   "images_total": cfg.get("total", B * world), "image": [n, n], "psf": [k, k],
                   "maxit": args.maxit,
                   "iterations_per_step": tot,
                   "parallelism": f"{world} independent shards, one process per GPU "
                                  f"(no collective on the data path)"},
        "roofline": None,
        "cpu_baseline": None,
    }
    if args.config in PUBLISHED_CONTEXT:
        result["context"] = PUBLISHED_CONTEXT[args.config]
    if os.environ.get("BSGP_RANK_DEVICE") is not None and not args.stub:
        result["config"]["parallelism"] += (f"; every rank on device {os.environ['BSGP_RANK_DEVICE']}"
                                            " (BSGP_RANK_DEVICE rehearsal, not a scaling figure)")
    if args.stub:
        result["data"] = "stub: harness test without a GPU"
        print(json.dumps(result), flush=True)
        return

    import sgp
    cnt = out["counters"].cpu().numpy()
    kern_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    persistent = kw["persistent"] if kw["persistent"] is not None else sgp.PERSIST_DEFAULT
    one_wg = int(cnt[0, 5]) == 1
    result["config"].update({"ls_spec": kw["ls_spec"] or sgp.LS_SPEC_DEFAULT,
                             # sub-batches actually run: the persistent solver of
                             # one-workgroup images runs the batch as one (bsgp_api.hip)
                             "streams": 1 if (persistent and one_wg) else
                             (kw["streams"] or sgp.STREAMS_DEFAULT),
                             "team": int(cnt[0, 5]),
                             "proj_cache": kw["proj_cache"] if kw["proj_cache"] is not None
                             else sgp.PROJ_CACHE_DEFAULT,
                             "gn_compact": sgp.GN_COMPACT_DEFAULT, "storage": args.storage,
                             "persistent": persistent,
                             "stop_criterion": kw["stop_criterion"]})
    if not args.no_profile:
        result["roofline"] = roofline(args, kw, gn, psf, bkg, B, n, kern_ms)
    if not args.no_e2e:
        result["end_to_end"] = end_to_end(kw, gn, psf, bkg)
    if world == 1 and not args.no_cpu:
        workers = max(1, min(CPU_CAP, os.cpu_count() or 1))
        images = args.cpu_images if B > 1 else 1
        cpu_maxit = args.cpu_maxit if args.cpu_maxit else args.maxit
        if stamps:
            result["cpu_baseline"] = cpu_baseline_stamps(kw, args.cpu_images * 8,
                                                         min(workers, args.cpu_images * 8), kl)
        else:
            result["cpu_baseline"] = cpu_baseline(n, k, nstars, images, cpu_maxit,
                                                  min(workers, images), circular=circ)
    print(json.dumps(result), flush=True)


def end_to_end(kw, gn, psf, bkg):
    """SURVEY §8d's second figure: one solve from host buffers to host buffers
    (the drop-in's own path: the images and backgrounds copied to the device,
    the solve, x / iters / discr / times / counters copied back), outside the
    timed loop.  `value` is never this: it times the solve on resident data."""
    import sgp
    g_host = gn.cpu().numpy()
    b_host = bkg.cpu().numpy()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    kl = "betaParams" not in kw and "adapt_beta" not in kw
    host_kw = {k_: (v.cpu().numpy() if torch.is_tensor(v) else v) for k_, v in kw.items()}
    out = (sgp.sgp_batch if kl else sgp.sgp_betaDiv_batch)(g_host, psf, b_host, **host_kw)
    el = time.perf_counter() - t0
    its = float(np.sum(out["iters"]))
    h2d = g_host.nbytes + b_host.nbytes
    d2h = sum(v.nbytes for v in out.values() if isinstance(v, np.ndarray))
    return {"value": its / el, "unit": "image-iterations/s", "ms": el * 1e3,
            "h2d_bytes": int(h2d), "d2h_bytes": int(d2h),
            "note": "host float64 arrays in, host arrays out (PCIe both ways), one solve"}


def profile_kernels(kw, gn, psf, bkg, n):
    """One profiled solve (bsgp_solve_profiled: one stream, a HIP event pair
    around every kernel launch): per kernel class its span, launches and
    algorithmic bytes per launch.  The persistent solver (k_persist) is one
    launch that runs every phase of every iteration: its bytes are all of them."""
    import _bsgp
    import sgp
    kl = "betaParams" not in kw and "adapt_beta" not in kw
    prof = (sgp.sgp_batch if kl else sgp.sgp_betaDiv_batch)(gn, psf, bkg, profile=True, **kw)
    plan = _bsgp.get_plan(n, n, psf, _bsgp.BSGP_CONV_CIRCULAR if kw["use_original_SGP_Afunction"]
                          else _bsgp.BSGP_CONV_LINEAR_FILL, storage=kw["storage"])
    cnt, iters = prof["counters"], prof["iters"]
    team = int(cnt[0, 5])
    kb = kernel_bytes(n, n, plan.P, plan.Q // 2 + 1, cnt, iters, beta=not kl,
                      series=not kl and not kw.get("adapt_beta", False),
                      compact=sgp.GN_COMPACT_DEFAULT == 1, bmap=False,
                      fused_at_col=(team == 1), vb=4.0 if kw["storage"] == "f32" else 8.0)
    ms, nl = prof["kernel_ms"], prof["launches"]
    # the persistent launch holds every iteration, and the setups too when
    # they are folded into it (no k_setup launch, SolveArgs::fold_setup)
    kb["k_persist"] = float(sum(v for k, v in kb.items() if k != "k_setup" or nl[0] == 0))
    names = ["k_setup", "k_dir", "k_col", "k_ls", "k_bb", "k_persist"]
    kernels = {}
    for i, name in enumerate(names):
        if i == 0 or nl[i] == 0:
            kernels[name] = {"ms_total": float(ms[i]), "launches": int(nl[i])}
            continue
        per_ms = ms[i] / nl[i]
        per_b = kb[name] / nl[i]
        ach = per_b / (per_ms * 1e-3) / 1e9
        kernels[name] = {"ms_total": float(ms[i]), "launches": int(nl[i]),
                         "ms_per_launch": float(per_ms), "bytes_per_launch": float(per_b),
                         "achieved": float(ach), "frac": float(ach / HBM_PEAK_GBS)}
    alg_total = float(sum(v for k, v in kb.items() if k != "k_persist"))  # (setup included)
    return kernels, alg_total, cnt, iters, float(np.sum(ms))


def roofline(args, kw, gn, psf, bkg, B, n, solve_ms):
    """Per-kernel roofline from a profiled solve (outside the timed loop)."""
    kernels, alg_total, cnt, iters, prof_total = profile_kernels(kw, gn, psf, bkg, n)
    names = [k for k in kernels if k != "k_setup" and kernels[k]["launches"] > 0]
    dom = max(names, key=lambda k_: kernels[k_]["ms_total"])
    d = kernels[dom]
    traffic = load_traffic(args.config)
    tr, tr_src = None, None
    if traffic and isinstance(traffic.get("kernels"), dict) and dom in traffic["kernels"]:
        tr = traffic["kernels"][dom].get("bytes_per_launch")
        # not measured in this run: read from the committed PMC record
        tr_src = (f"profiles/traffic_{args.config}.json (committed PMC record, not this run): "
                  + str(traffic.get("note", "")))
    if dom == "k_persist":
        folded = kernels["k_setup"]["launches"] == 0
        unit = (f"one launch = the whole solve: {B} images x {int(iters.max())} iterations, "
                f"every phase (persistent task-queue kernel)"
                + (", and every image's setup as its first task" if folded else ""))
    else:
        unit = f"one launch = {B} images x one iteration of {dom} (profiled solve on one stream)"
    out = {"bound": "hbm", "kernel": dom, "achieved": d["achieved"], "peak": HBM_PEAK_GBS,
           "unit": "GB/s", "frac": d["frac"], "traffic": tr, "traffic_source": tr_src,
           "ms_per_launch": d["ms_per_launch"], "bytes_per_launch": d["bytes_per_launch"],
           "launch_unit": unit, "kernels": kernels, "profiled_solve_ms": prof_total,
           "solve": {"alg_bytes": alg_total, "ms_timed": solve_ms,
                     "achieved_timed": alg_total / (solve_ms * 1e-3) / 1e9,
                     "frac_timed": alg_total / (solve_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                     "note": "whole solve in the timed loop, same bytes"},
           "counters_per_iter": {
               "E_p": float(cnt[:, 0].sum() / iters.sum()),
               "E_ls": float(cnt[:, 1].sum() / iters.sum()),
               "proj_passes": float(cnt[:, 6].sum() / iters.sum()),
               "proj_list_frac": float(cnt[:, 7].sum() / iters.sum() / (n * n)),
               "ls_passes": float(cnt[:, 2].sum() / iters.sum()),
               "ls_series": float(cnt[:, 4].sum() / iters.sum())}}
    if dom == "k_persist":
        # where the time goes, phase by phase: the same solve on the phase kernels
        pk, _, _, _, ptot = profile_kernels(dict(kw, persistent=0), gn, psf, bkg, n)
        out["phase_kernels"] = {"note": "the same solve as one launch per phase and iteration "
                                        "(persistent=0), one stream", "profiled_solve_ms": ptot,
                                "kernels": pk}
    return out


if __name__ == "__main__":
    main()
