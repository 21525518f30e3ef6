"""Benchmark: SGP iterations/s (fp64) on batched 256x256 images + %HBM peak.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c3|c2|c1] ...

A *step* is one complete batched solve (BASELINE config C3: 1024 independent
256x256 star-field stamps, beta-SGP, fp64, 25x25 Gaussian PSF with the
astropy-semantics linear A, flux-conserving projection, MAXIT iterations with
stop_criterion=1 so every image runs exactly MAXIT iterations).
Inputs are synthetic (SURVEY §8d generator), built on the device and resident
in HBM before timing starts.  ``value`` = image-iterations of all ranks /
max-over-ranks wall time of the K timed steps.  Multi-GPU: one process per
GPU, each rank solves its own batch (seeds offset by rank): weak scaling, no
collective on the data path.

roofline: algorithmic bytes of the passes the engine makes over HBM-resident
image vectors (8*N*(23 + 2*proj_passes + 3*ls_passes) per image-iteration plus
16 B per projection-list entry read, all counted on the device; SURVEY §8d's
per-evaluation formula is reported beside it) / the solve's duration measured
with HIP events on the launch stream (the solve is the unit launched: setup +
MAXIT x five phase kernels on three sub-batch streams); peak 8.0 TB/s.
traffic: HBM bytes per solve from a rocprofv3 PMC run (profiles/), if present.
cpu_baseline: the numpy oracle (oracle/sgp_oracle.py, a port of the reference)
on a bounded sample of the same workload, process pool on this host's cores.
"""
import argparse
import json
import os
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


# SURVEY §8d configurations that fit one GPU (C1 is the reference's own
# NGC7027 CPU case; C5 is C3 sharded over 8 GPUs = `--config c3 --gpus 8`).
CONFIGS = {
    "c2": dict(n=256, k=25, nstars=200, batch=1, circular=False,
               desc="single {n}x{n} synthetic image, 25x25 Gaussian PSF, linear A"),
    "c3": dict(n=256, k=25, nstars=200, batch=1024, circular=False,
               desc="{B} independent {n}x{n} stamps per GPU, 25x25 PSF, linear A"),
    "c4": dict(n=2048, k=64, nstars=5000, batch=1, circular=True,
               desc="single {n}x{n} synthetic field, 64x64 PSF embedded at the centre, "
                    "circular A (pow-2 FFT)"),
}


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


def solve_kwargs(maxit, ls_spec, streams=None, team=None, circular=False, proj_cache=None):
    max_projs, gamma, beta, alpha_min, alpha_max, alpha, M_alpha, tau, M = (
        1000, 1e-4, 0.4, 1e-5, 1e5, 1e1, 3, 0.5, 1)  # sgp.DEFAULT_PARAMS (sgp.py:34)
    return dict(init_recon=2, proj_type=1, stop_criterion=1, MAXIT=maxit, gamma=gamma, beta=beta,
                alpha=alpha, alpha_min=alpha_min, alpha_max=alpha_max, M_alpha=M_alpha, tau=tau,
                M=M, max_projs=max_projs, ccd_sat_level=65000.0, scale_data=True,
                use_original_SGP_Afunction=circular, adapt_beta=False, betaParam=1.05, lr=1e-3,
                lr_exp_param=0.1, schedule_lr=True, ls_spec=ls_spec, streams=streams,
                team=team, proj_cache=proj_cache)


def cpu_baseline(n, k, nstars, images, maxit, workers, circular=False):
    """Oracle (numpy port of the reference, oracle/sgp_oracle.py) on `images`
    stamps x `maxit` iterations, one image per task on `workers` processes;
    wall time of the solve phase (pool already warm, inputs built in-task)."""
    import cpu_bench
    kw = solve_kwargs(maxit, None, circular=circular)
    for key in ("ls_spec", "team", "streams", "proj_cache"):
        kw.pop(key)
    iters, wall, cpu_s = cpu_bench.run_pool(n, k, nstars, images, kw, workers)
    return {"value": iters / wall, "unit": "image-iterations/s", "cores": workers,
            "kind": "port",
            "sample": f"{images} images {n}x{n} (bench generator) x {maxit} beta-SGP iterations "
                      f"with oracle/sgp_oracle.py on a pool of {workers} processes: "
                      f"{iters} image-iterations in {wall:.1f}s wall "
                      f"({iters / cpu_s:.1f} image-it/s per core)"}


def shard_seed0(rank, images_per_rank):
    """Rank r solves images [r*B, (r+1)*B) of the synthetic stream: disjoint
    shards, no data-path collective."""
    return rank * images_per_rank


def aggregate(dist, elapsed, iters_sum, device):
    """Cross-rank reduction of one timed run: the max wall time over ranks and
    the total image-iterations of all ranks (the only collectives of the
    harness).  Works with any torch.distributed backend (nccl on the GPU box,
    gloo in the CPU tests)."""
    t = torch.tensor([float(elapsed)], dtype=torch.float64, device=device)
    n = torch.tensor([float(iters_sum)], dtype=torch.float64, device=device)
    if dist is not None:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dist.all_reduce(n, op=dist.ReduceOp.SUM)
    return float(t.item()), float(n.item())


def load_traffic(config):
    f = os.path.join(ROOT, "profiles", f"traffic_{config}.json")
    if os.path.exists(f):
        try:
            return json.load(open(f))
        except Exception:
            return None
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--batch", type=int, default=None)
    ap.add_argument("--maxit", type=int, default=100)
    ap.add_argument("--ls-spec", type=int, default=None)
    ap.add_argument("--streams", type=int, default=None)
    ap.add_argument("--team", type=int, default=None,
                    help="workgroups per image (0/None = auto, 1 = one per image)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--proj-cache", type=int, default=None)
    ap.add_argument("--cpu-images", type=int, default=16)
    ap.add_argument("--cpu-maxit", type=int, default=None,
                    help="iterations per CPU-baseline image (default: --maxit)")
    args = ap.parse_args()
    global torch
    import torch as _torch
    torch = _torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl", rank=rank, world_size=world,
                                device_id=torch.device("cuda", local))

    import _bsgp
    import sgp

    cfg = CONFIGS[args.config]
    n, k, nstars, circ = cfg["n"], cfg["k"], cfg["nstars"], cfg["circular"]
    B = args.batch if args.batch else cfg["batch"]
    gn, psf = synth_batch(B, n, k, nstars, seed0=shard_seed0(rank, B), circular=circ)
    bkg = torch.full((B,), 100.0, dtype=torch.float64, device="cuda")
    kw = solve_kwargs(args.maxit, args.ls_spec, args.streams, args.team, circular=circ,
                      proj_cache=args.proj_cache)
    torch.cuda.synchronize()

    def step():
        return sgp.sgp_betaDiv_batch(gn, psf, bkg, device_out=True, **kw)

    for _ in range(args.warmup):
        out = step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    ev = []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        out = step()
        e1.record()
        ev.append((e0, e1))
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    kern_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    iters = out["iters"].cpu().numpy()
    cnt = out["counters"].cpu().numpy()
    elapsed_max, tot = aggregate(dist, elapsed, iters.sum(), "cuda")
    total_iters = tot * args.steps
    value = total_iters / elapsed_max

    # Algorithmic bytes per solve, b = 0 (scalar background).  SURVEY §8d
    # prices every projection / line-search *evaluation* as a pass over the
    # image: 8*N*(23 + 2*E_p + 3*E_ls) per image-iteration.  The engine needs
    # fewer passes (line-search trials from the moment series, several trials
    # per pass, projection evaluations from the pixel lists), so the roofline
    # uses the bytes of the passes it actually makes:
    #   8*N*(23 + 2*proj_passes + 3*ls_passes) + 16*(list entries read).
    N = n * n
    E_p, E_ls = cnt[:, 0].astype(np.float64), cnt[:, 1].astype(np.float64)
    ls_passes = cnt[:, 2].astype(np.float64)
    proj_passes, list_reads = cnt[:, 6].astype(np.float64), cnt[:, 7].astype(np.float64)
    survey_bytes = float(np.sum(8.0 * N * (23.0 * iters + 2.0 * E_p + 3.0 * E_ls)))
    alg_bytes = float(np.sum(8.0 * N * (23.0 * iters + 2.0 * proj_passes + 3.0 * ls_passes)
                             + 16.0 * list_reads))
    achieved = alg_bytes / (kern_ms * 1e-3) / 1e9
    traffic = load_traffic(args.config)
    result = {
        "metric": "SGP iterations/sec (fp64) on batched 256x256 images",
        "value": value,
        "unit": "image-iterations/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed_max / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (SURVEY §8d generator: pareto point sources * 25x25 Gaussian PSF "
                "+ Poisson, bkg 100), built on device",
        "config": {"workload": f"{args.config.upper()}: " + cfg["desc"].format(n=n, B=B)
                               + f", beta-SGP (beta=1.05), proj_type=1, "
                               f"MAXIT={args.maxit}, stop_criterion=1",
                   "images_per_gpu": B, "image": [n, n], "psf": [k, k], "maxit": args.maxit,
                   "parallelism": f"{world} independent shards (no collective)",
                   "ls_spec": kw["ls_spec"] or sgp.LS_SPEC_DEFAULT,
                   "streams": kw["streams"] or sgp.STREAMS_DEFAULT,
                   "team": int(cnt[0, 5]),
                   "proj_cache": kw["proj_cache"] if kw["proj_cache"] is not None
                   else sgp.PROJ_CACHE_DEFAULT},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS,
                     "traffic": traffic.get("bytes_per_launch") if traffic else None,
                     "kernel": "one solve = setup + MAXIT x (k_dir, k_col, k_ls, k_col, k_bb)",
                     "kernel_ms": kern_ms,
                     "alg_bytes_per_launch": alg_bytes,
                     "survey_formula_bytes_per_launch": survey_bytes,
                     "E_p_per_iter": float(E_p.sum() / iters.sum()),
                     "E_ls_per_iter": float(E_ls.sum() / iters.sum()),
                     "proj_passes_per_iter": float(proj_passes.sum() / iters.sum()),
                     "proj_list_frac_per_iter": float(list_reads.sum() / iters.sum() / N),
                     "ls_passes_per_iter": float(ls_passes.sum() / iters.sum()),
                     "ls_series_per_iter": float(cnt[:, 4].sum() / iters.sum())},
        "cpu_baseline": None,
    }
    if rank == 0 and world == 1 and not args.no_cpu:
        workers = max(1, min(16, os.cpu_count() or 1))
        images = args.cpu_images if B > 1 else 1
        cpu_maxit = args.cpu_maxit if args.cpu_maxit else args.maxit
        result["cpu_baseline"] = cpu_baseline(n, k, nstars, images, cpu_maxit,
                                              min(workers, images), circular=circ)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
