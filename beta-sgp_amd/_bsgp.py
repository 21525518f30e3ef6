"""ctypes binding of libbsgp.so (include/bsgp.h) — the only way the Python
drop-in reaches the GPU.  There is no CPU fallback: if the library or a
device is missing, every entry point raises ``BsgpError``.

PyTorch is imported *before* the library is loaded so that the process holds
exactly one HIP runtime (torch ships its own ``libamdhip64.so``; the library's
``libamdhip64.so.7`` dependency then binds to it).  Torch is used for device
memory and the current stream only; no torch type crosses the C ABI.
"""
import ctypes
import os
import threading

import numpy as np

try:  # one HIP runtime per process: torch's, loaded first
    import torch  # noqa: F401
except ImportError:  # pragma: no cover - torch is part of the image
    torch = None

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("BSGP_LIB", os.path.join(_HERE, "libbsgp.so"))

BSGP_CONV_CIRCULAR = 0
BSGP_CONV_LINEAR_FILL = 1
BSGP_VARIANT_KL = 0
BSGP_VARIANT_BETA = 1
BSGP_STORAGE_F64 = 0
BSGP_STORAGE_F32 = 1
ABI_VERSION = 3
BSGP_ERR_ARG = -1
BSGP_ERR_HIP = -2
BSGP_ERR_UNSUPPORTED = -3
BSGP_ERR_PSF = -4


class BsgpError(RuntimeError):
    """A failure reported by libbsgp (status code + bsgp_last_error())."""

    def __init__(self, code, msg):
        super().__init__(f"libbsgp error {code}: {msg}")
        self.code = code


class Params(ctypes.Structure):
    _fields_ = [
        ("variant", ctypes.c_int32), ("init_recon", ctypes.c_int32),
        ("proj_type", ctypes.c_int32), ("stop_criterion", ctypes.c_int32),
        ("MAXIT", ctypes.c_int32), ("M_alpha", ctypes.c_int32), ("M", ctypes.c_int32),
        ("max_projs", ctypes.c_int32),
        ("gamma", ctypes.c_double), ("beta", ctypes.c_double), ("alpha", ctypes.c_double),
        ("alpha_min", ctypes.c_double), ("alpha_max", ctypes.c_double), ("tau", ctypes.c_double),
        ("ccd_sat_level", ctypes.c_double), ("betaParam", ctypes.c_double),
        ("lr", ctypes.c_double), ("lr_exp_param", ctypes.c_double),
        ("tol_convergence", ctypes.c_double), ("prescaled_scaling", ctypes.c_double),
        ("prescaled_tol4", ctypes.c_double),
        ("has_sat", ctypes.c_int32), ("scale_data", ctypes.c_int32), ("verbose", ctypes.c_int32),
        ("adapt_beta", ctypes.c_int32), ("schedule_lr", ctypes.c_int32),
        ("bkg_is_map", ctypes.c_int32), ("ls_spec", ctypes.c_int32), ("ls_series", ctypes.c_int32),
        ("streams", ctypes.c_int32), ("team", ctypes.c_int32), ("proj_cache", ctypes.c_int32),
        ("gn_compact", ctypes.c_int32), ("gn_f32", ctypes.c_int32),
        ("beta0_general", ctypes.c_int32), ("flux_f32", ctypes.c_int32),
        ("persistent", ctypes.c_int32),
    ]


_P = ctypes.c_void_p


class Inputs(ctypes.Structure):
    _fields_ = [("gn", _P), ("bkg", _P), ("flux", _P), ("x0", _P), ("beta0", _P), ("obj", _P)]


class Outputs(ctypes.Structure):
    _fields_ = [("x", _P), ("iters", _P), ("discr", _P), ("times", _P), ("crit", _P),
                ("flags", _P), ("beta_final", _P), ("counters", _P), ("err", _P),
                ("x_iter", _P)]


class PsfModel(ctypes.Structure):
    """bsgp_psf_model (include/bsgp.h)."""
    _fields_ = [("hw", ctypes.c_int32), ("ngauss", ctypes.c_int32), ("ldeg", ctypes.c_int32),
                ("sdeg", ctypes.c_int32), ("cos", ctypes.c_double), ("sin", ctypes.c_double),
                ("ax", ctypes.c_double), ("ay", ctypes.c_double), ("sigma_inc", ctypes.c_double),
                ("x_orig", ctypes.c_double), ("y_orig", ctypes.c_double), ("coeffs", _P),
                ("ncoef", ctypes.c_int32)]


_lib = None
_lib_lock = threading.Lock()


def lib():
    """Load libbsgp.so once; raise loudly if it is absent."""
    global _lib
    if _lib is not None:
        return _lib
    with _lib_lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise BsgpError(-3, f"{LIB_PATH} not built — run __graft_entry__.build()")
            L = ctypes.CDLL(LIB_PATH)
            i32, i64, dbl, vp = ctypes.c_int32, ctypes.c_int64, ctypes.c_double, ctypes.c_void_p
            L.bsgp_last_error.restype = ctypes.c_char_p
            L.bsgp_abi_version.restype = i32
            L.bsgp_plan_create.argtypes = [i32, i32, vp, i32, i32, i32, i32, i32,
                                           ctypes.POINTER(vp)]
            L.bsgp_plan_create_checked.argtypes = [i32, i32, vp, i32, i32, i32, i32, i32, i32,
                                                   ctypes.POINTER(vp)]
            L.bsgp_plan_destroy.argtypes = [vp]
            L.bsgp_plan_info.argtypes = [vp, vp, vp, vp, vp]
            L.bsgp_solve_device.argtypes = [vp, i32, vp, vp, vp, vp]
            L.bsgp_solve_host.argtypes = [vp, i32, vp, vp, vp]
            L.bsgp_solve_profiled.argtypes = [vp, i32, vp, vp, vp, vp, vp, vp]
            L.bsgp_apply_operator.argtypes = [vp, i32, i32, vp, vp, vp]
            L.bsgp_project_df.argtypes = [i64, dbl, vp, vp, dbl, i32, dbl, dbl, dbl, dbl, i32,
                                          i32, i32, vp, vp, vp]
            L.bsgp_beta_div.argtypes = [i64, vp, vp, dbl, vp, vp]
            L.bsgp_beta_div_deriv.argtypes = [i64, vp, vp, dbl, vp, vp]
            L.bsgp_beta_div_grad_parts.argtypes = [i64, vp, vp, dbl, vp, vp, vp]
            L.bsgp_extract_tiles.argtypes = [vp, i32, i32, vp, i32, i32, i32, vp, vp]
            L.bsgp_coadd_tiles.argtypes = [vp, i32, i32, i32, vp, i32, i32, vp, vp, vp]
            L.bsgp_fits_to_f64.argtypes = [vp, i64, i32, dbl, dbl, vp, vp]
            L.bsgp_psf_stamps.argtypes = [ctypes.POINTER(PsfModel), vp, i32, i32, i32, vp, vp]
            L.bsgp_plan_set_psfs.argtypes = [vp, vp, i32, vp]
            for name in ["bsgp_plan_create", "bsgp_plan_create_checked", "bsgp_plan_destroy", "bsgp_plan_info",
                         "bsgp_solve_device", "bsgp_solve_host", "bsgp_solve_profiled",
                         "bsgp_apply_operator",
                         "bsgp_project_df", "bsgp_beta_div", "bsgp_beta_div_deriv",
                         "bsgp_beta_div_grad_parts", "bsgp_device_synchronize",
                         "bsgp_extract_tiles", "bsgp_coadd_tiles", "bsgp_fits_to_f64",
                         "bsgp_psf_stamps", "bsgp_plan_set_psfs"]:
                getattr(L, name).restype = ctypes.c_int
            if L.bsgp_abi_version() != ABI_VERSION:
                raise BsgpError(-3, f"{LIB_PATH} has ABI {L.bsgp_abi_version()}, this binding "
                                    f"needs {ABI_VERSION}: rebuild with __graft_entry__.build()")
            _lib = L
    return _lib


EXPORTED = ["bsgp_plan_create", "bsgp_plan_create_checked", "bsgp_plan_destroy", "bsgp_plan_info", "bsgp_solve_device",
            "bsgp_solve_host", "bsgp_solve_profiled", "bsgp_apply_operator", "bsgp_project_df", "bsgp_beta_div",
            "bsgp_beta_div_deriv", "bsgp_beta_div_grad_parts", "bsgp_device_synchronize",
            "bsgp_last_error", "bsgp_abi_version", "bsgp_extract_tiles", "bsgp_coadd_tiles",
            "bsgp_fits_to_f64", "bsgp_psf_stamps", "bsgp_plan_set_psfs"]


def check(rc):
    if rc != 0:
        raise BsgpError(rc, lib().bsgp_last_error().decode(errors="replace"))


def require_gpu():
    """The product path runs on the device or not at all."""
    if torch is None or not torch.cuda.is_available():
        raise BsgpError(-2, "no HIP device visible: the beta-SGP engine has no CPU fallback")


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def current_stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


class Plan:
    """A device plan: FFT geometry + PSF transfer functions (bsgp_plan_create)."""

    _leased = False  # held by a solve (lease_plan)
    _done = None  # event after the last leased solve's launches

    def __init__(self, H, W, psf, conv_mode, device=None, storage=BSGP_STORAGE_F64,
                 psf_checked=False):
        require_gpu()
        if device is None:
            device = torch.cuda.current_device()
        psf = np.ascontiguousarray(psf, dtype="<f8")
        self.H, self.W = int(H), int(W)
        self.kh, self.kw = psf.shape
        self.conv_mode = conv_mode
        self.device = device
        self.storage = storage
        h = ctypes.c_void_p()
        # psf_checked: the caller has checked the PSF's normalisation itself,
        # in its own dtype (the drop-in's pool and per-image plans, after
        # sgp._check_psf / check_psf_once), so the library's float64 check is
        # skipped; a direct construction keeps the library's check
        rc = lib().bsgp_plan_create_checked(self.H, self.W, psf.ctypes.data, self.kh, self.kw,
                                            conv_mode, storage, device, int(bool(psf_checked)),
                                            ctypes.byref(h))
        if rc != 0:
            raise BsgpError(rc, lib().bsgp_last_error().decode(errors="replace"))
        self.h = h
        P, Q, wave = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32()
        sb = ctypes.c_int64()
        check(lib().bsgp_plan_info(h, ctypes.byref(P), ctypes.byref(Q), ctypes.byref(sb),
                                   ctypes.byref(wave)))
        self.P, self.Q, self.slot_bytes, self.fft_waves = P.value, Q.value, sb.value, wave.value

    def __del__(self):
        h = getattr(self, "h", None)
        if h is not None and _lib is not None:
            try:
                _lib.bsgp_plan_destroy(h)
            except Exception:  # pragma: no cover
                pass
            self.h = None

    # -------------------------------------------------------------- operators
    def set_psfs(self, psfs):
        """Give image i of every later solve its own PSF psfs[i] ([n, kh, kw]
        float64 CUDA tensor; bsgp_plan_set_psfs builds the n TF pairs on the device)."""
        psfs = psfs.to(dtype=torch.float64).contiguous()
        if psfs.dim() != 3 or tuple(psfs.shape[1:]) != (self.kh, self.kw):
            raise ValueError(f"psfs must be [n, {self.kh}, {self.kw}]")
        check(lib().bsgp_plan_set_psfs(self.h, _ptr(psfs), psfs.shape[0], current_stream()))
        self.n_psf = psfs.shape[0]
        return self

    def apply(self, x, transpose=False):
        """A(x) / AT(x) on a [B,H,W] (or [H,W]) float64 CUDA tensor."""
        x = x.contiguous()
        out = torch.empty_like(x)
        B = 1 if x.dim() == 2 else x.shape[0]
        check(lib().bsgp_apply_operator(self.h, B, int(transpose), _ptr(x), _ptr(out),
                                        current_stream()))
        return out

    # ------------------------------------------------------------------ solve
    def solve(self, gn, bkg, params, flux=None, x0=None, beta0=None, want_times=True, obj=None,
              want_iterates=False, profile=False):
        """Batched solve on device tensors: gn [B,H,W] f64; bkg [B] or [B,H,W];
        flux/beta0 [B] or None; x0 [B,H,W] or None; obj [B,H,W] or None (then
        "err" holds the per-iteration relative error); want_iterates adds
        "x_iter" [B,MAXIT,H,W].  Asynchronous on the current stream; returns a
        dict of device output tensors.  profile=True runs bsgp_solve_profiled
        (one stream, synchronous) and adds "kernel_ms" / "launches" [6]: setup,
        k_dir, k_col, k_ls, k_bb, k_persist."""
        B = gn.shape[0]
        M1 = params.MAXIT + 1
        dev = gn.device
        f64 = dict(dtype=torch.float64, device=dev)
        if want_iterates:
            # save=True keeps every iterate of the MAXIT budget on the device
            # (copied to the host once, up to the iterations run): refuse a
            # budget that the device cannot hold beside the solve's own workspace
            need = B * params.MAXIT * self.H * self.W * 8
            free = torch.cuda.mem_get_info(dev)[0]
            if need > 0.8 * free:
                raise BsgpError(
                    f"save=True keeps {params.MAXIT} iterates of {self.H}x{self.W} on the device "
                    f"({need / 2**30:.1f} GiB, {free / 2**30:.1f} GiB free): lower MAXIT")
        # the small outputs are views of two zeroed blocks (two fill launches
        # instead of eight on the latency-bound single-image calls)
        nd = B * M1 * (2 + bool(want_times) + (obj is not None)) + B
        d64 = torch.zeros(nd, **f64)
        i32 = torch.zeros(B * (M1 + 1) + 2 * 8 * B, dtype=torch.int32, device=dev)
        parts = iter(torch.split(d64, [B * M1] * (2 + bool(want_times) + (obj is not None)) + [B]))
        discr, crit = next(parts).view(B, M1), next(parts).view(B, M1)
        times = next(parts).view(B, M1) if want_times else None
        err = next(parts).view(B, M1) if obj is not None else None
        beta_final = next(parts)
        cnt, iters, flags = torch.split(i32, [2 * 8 * B, B, B * M1])  # (int64 counters first: aligned)
        out = {
            "x": torch.empty_like(gn),
            "iters": iters,
            "discr": discr,
            "times": times,
            "crit": crit,
            "flags": flags.view(B, M1),
            "beta_final": beta_final,
            "counters": cnt.view(torch.int64).view(B, 8),
            "err": err,
            "x_iter": (torch.zeros(B, params.MAXIT, self.H, self.W, **f64) if want_iterates
                       else None),
        }
        ins = Inputs(_ptr(gn), _ptr(bkg), _ptr(flux), _ptr(x0), _ptr(beta0), _ptr(obj))
        outs = Outputs(*[_ptr(out[k]) for k in ["x", "iters", "discr", "times", "crit", "flags",
                                                 "beta_final", "counters", "err", "x_iter"]])
        self._keep = (gn, bkg, flux, x0, beta0, obj)
        if profile:
            kms = np.zeros(6, np.float64)
            nl = np.zeros(6, np.int64)
            check(lib().bsgp_solve_profiled(self.h, B, ctypes.byref(params), ctypes.byref(ins),
                                            ctypes.byref(outs), current_stream(),
                                            kms.ctypes.data, nl.ctypes.data))
            out["kernel_ms"], out["launches"] = kms, nl
            return out
        check(lib().bsgp_solve_device(self.h, B, ctypes.byref(params), ctypes.byref(ins),
                                      ctypes.byref(outs), current_stream()))
        return out


STATUS_LS_CAP = 1
STATUS_TEAM_TIMEOUT = 4
STATUS_NO_POSITIVE_BOUND = 8


def check_status(counters):
    """Raise if a solve reported a status bit in counters[:, 3]: its results
    are not valid.  Bit 1: the line search hit its trial cap, which happens
    only for a backtracking factor outside (0, 1), where the reference's
    loop (sgp.py:328-349 / 776-801) never terminates; bit 4: a team barrier
    timed out (workgroups not co-resident); bit 8: y = flux/(flux+bkg)*AT(gn)
    has no positive entry, where the reference raises numpy's ValueError
    (np.min of an empty array, sgp.py:269-270 / 711-712) -- raised here as
    ValueError too."""
    c = counters.cpu().numpy() if hasattr(counters, "cpu") else np.asarray(counters)
    st = c[:, 3]
    if np.any(st & STATUS_NO_POSITIVE_BOUND):
        bad = np.nonzero(st & STATUS_NO_POSITIVE_BOUND)[0].tolist()
        raise ValueError("zero-size array to reduction operation minimum which has no identity "
                         f"(image(s) {bad[:8]}: y = flux/(flux+bkg)*AT(gn) has no positive "
                         "entry, sgp.py:269-270)")
    if np.any(st & STATUS_TEAM_TIMEOUT):
        raise BsgpError(BSGP_ERR_HIP, "team barrier timed out (workgroups not co-resident)")
    if np.any(st & STATUS_LS_CAP):
        raise BsgpError(BSGP_ERR_ARG, "line search did not terminate: the backtracking factor "
                                      "beta must lie in (0, 1) (sgp.py:349 lam = lam * beta)")


_plan_cache = {}
_plan_cache_lock = threading.Lock()


STORAGE = {"f64": BSGP_STORAGE_F64, "f32": BSGP_STORAGE_F32}


def storage_code(storage):
    """'f64' / 'f32' (or the BSGP_STORAGE_* value) -> BSGP_STORAGE_*."""
    if storage in STORAGE.values():
        return storage
    if storage not in STORAGE:
        raise ValueError(f"storage must be 'f64' or 'f32', not {storage!r}")
    return STORAGE[storage]


# Plans are found by PSF content.  Keying the cache by the PSF's bytes cost
# every call a copy and a hash of the whole PSF (C4's circular A takes a
# 2048^2 PSF: ~20 ms of host time per call, GPU idle when the call starts
# from an idle stream); the key holds a fingerprint of a strided sample
# instead, and a plan matches only when its own copy of the PSF is
# byte-identical to the caller's (memcmp: one pass over the PSF).
_libc = ctypes.CDLL(None)
_libc.memcmp.restype = ctypes.c_int
_libc.memcmp.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]


def _same_psf(plan, psf):
    ref = plan._psf_host
    return ref.shape == psf.shape and (
        psf.nbytes == 0 or _libc.memcmp(ref.ctypes.data, psf.ctypes.data, psf.nbytes) == 0)


# plan-layout overrides read by bsgp_plan_create (A/B knobs): part of the key,
# so a pooled plan never keeps the layout of an earlier setting
_PLAN_KNOBS = ("BSGP_PERWAVE_MIN_WG", "BSGP_PERWAVE_TW", "BSGP_COOP_ELEMS")


def _plan_key(H, W, psf, conv_mode, storage):
    psf = np.ascontiguousarray(psf, dtype="<f8")
    flat = psf.reshape(-1)
    sample = flat[::max(1, flat.size // 4096)].tobytes()
    return psf, (H, W, psf.shape, hash(sample), conv_mode, storage_code(storage),
                 torch.cuda.current_device(), tuple(os.environ.get(k) for k in _PLAN_KNOBS))


def _new_plan(H, W, psf, key):
    p = Plan(H, W, psf, key[4], key[6], storage=key[5], psf_checked=True)
    p._psf_host = psf.copy()  # (the caller may rewrite its array later)
    return p


def get_plan(H, W, psf, conv_mode, storage="f64"):
    """A plan for the calling thread's own use (operators, plan queries):
    cached per (shape, psf content, mode, storage, device, host thread), since a
    plan's operator workspace serves one call at a time (include/bsgp.h: a
    plan is not thread-safe).  Entries of threads that have ended are dropped.
    Solves take their plan from the shared pool (lease_plan) instead."""
    require_gpu()
    psf, key = _plan_key(H, W, psf, conv_mode, storage)
    key = key + (threading.get_ident(),)
    with _plan_cache_lock:
        p = _plan_cache.get(key)
        if p is None or not _same_psf(p, psf):
            live = {t.ident for t in threading.enumerate()}
            for k in [k for k in _plan_cache if k[-1] not in live]:
                del _plan_cache[k]
            if len(_plan_cache) > 16:
                _plan_cache.clear()
            p = _new_plan(H, W, psf, key)
            _plan_cache[key] = p
    return p


# Solve plans: a pool per (shape, psf, mode, storage, device).  A solve leases
# an idle plan (or creates one) for the duration of its enqueue; the plan's
# workspace stays in use on the device until the solve's stream gets there, so
# the lease ends with an event on that stream and the next lessee's stream
# waits for it.  Concurrent solves (devices=[...] threads, several shards on
# one GPU) get separate plans; later calls reuse them, whichever thread runs
# them, so a new devices=[...] call re-allocates nothing.
_pool = {}
_POOL_MAX = 8  # plans kept per key


_checked = {}  # PSFs that passed a check: (check, dtype, shape, sample hash) -> copy


def check_psf_once(psf, check):
    """Run ``check(psf)`` on the caller's own array (its dtype kept: the
    reference sums the PSF in its own dtype, sgp.py:97-102 / :557-562) unless
    a byte-identical PSF of the same dtype has passed it before.  Found like
    the plans: a fingerprint of a strided sample, then memcmp."""
    psf = np.ascontiguousarray(psf)
    flat = psf.reshape(-1)
    key = (check, psf.dtype.str, psf.shape, hash(flat[::max(1, flat.size // 4096)].tobytes()))
    with _plan_cache_lock:
        ref = _checked.get(key)
        if ref is not None and (psf.nbytes == 0 or _libc.memcmp(
                ref.ctypes.data, psf.ctypes.data, psf.nbytes) == 0):
            return
    check(psf)
    with _plan_cache_lock:
        if len(_checked) > 32:
            _checked.clear()
        _checked[key] = psf.copy()


class lease_plan:
    """Context manager: ``with lease_plan(H, W, psf, mode, storage) as plan``."""

    def __init__(self, H, W, psf, conv_mode, storage="f64"):
        require_gpu()
        self.args = (H, W, psf, conv_mode, storage)
        self.plan = None

    def __enter__(self):
        H, W, psf, conv_mode, storage = self.args
        psf, key = _plan_key(H, W, psf, conv_mode, storage)
        with _plan_cache_lock:
            plans = _pool.setdefault(key, [])
            p = next((q for q in plans if not q._leased and _same_psf(q, psf)), None)
            if p is None:
                p = _new_plan(H, W, psf, key)
                p._done = None
                if len(plans) < _POOL_MAX:
                    plans.append(p)
            p._leased = True
        if p._done is not None:
            torch.cuda.current_stream().wait_event(p._done)
        self.plan = p
        return p

    def __exit__(self, *exc):
        p = self.plan
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream())
        p._done = ev
        with _plan_cache_lock:
            p._leased = False
        return False


def per_image_plan(H, W, psfs, conv_mode, storage="f64"):
    """A plan whose image i uses psfs[i] ([B, kh, kw], numpy or CUDA tensor);
    not cached (it holds B transfer-function pairs)."""
    require_gpu()
    # on the current device whatever device (or host) the stamps come from:
    # the plan-building kernels read them there
    dev = (psfs.to(device=torch.cuda.current_device(), dtype=torch.float64).contiguous()
           if torch.is_tensor(psfs) else to_dev(psfs))
    p = Plan(H, W, dev[0].cpu().numpy(), conv_mode, storage=storage_code(storage),
             psf_checked=True)
    return p.set_psfs(dev)


def to_dev(a):
    a = np.ascontiguousarray(a, dtype="<f8")
    if not a.flags.writeable:
        a = a.copy()
    return torch.from_numpy(a).to("cuda")


def to_dev_async(a):
    """Host array -> float64 device tensor through page-locked memory (torch's
    caching host allocator, which does not hand the block out again before
    the copy has run), enqueued on the current stream without waiting: the
    single-image drop-in's inputs (a pageable copy stages through the
    runtime's own buffer and blocks)."""
    a = np.asarray(a, dtype="<f8")
    h = torch.empty(a.shape, dtype=torch.float64, pin_memory=True)
    h.numpy()[...] = a
    return h.to("cuda", non_blocking=True)


def to_host(tensors):
    """Device tensors (dict; None entries kept) -> numpy arrays: every copy
    enqueued on the current stream into page-locked memory, ONE stream
    synchronisation, then plain numpy copies (nothing page-locked escapes to
    the caller)."""
    pinned = {k: (None if t is None else t.to("cpu", non_blocking=True))
              for k, t in tensors.items()}
    torch.cuda.current_stream().synchronize()
    return {k: (None if t is None else t.numpy().copy()) for k, t in pinned.items()}


def project_df_dev(b, c, dia, scaling, ccd_sat_level, lambda_, dlambda_, tol_lam, biter, siter,
                   max_projs):
    """flux_conserve_proj.projectDF on device tensors; returns (x, info[4])."""
    x = torch.empty_like(c)
    info = torch.zeros(4, dtype=torch.float64, device=c.device)
    has_sat = ccd_sat_level is not None
    check(lib().bsgp_project_df(c.numel(), float(b), _ptr(c), _ptr(dia), float(scaling),
                                int(has_sat), float(ccd_sat_level) if has_sat else 0.0,
                                float(lambda_), float(dlambda_), float(tol_lam), int(biter),
                                int(siter), int(max_projs), _ptr(x), _ptr(info),
                                current_stream()))
    return x, info


def beta_div_dev(y, x, beta):
    out = torch.zeros(1, dtype=torch.float64, device=y.device)
    check(lib().bsgp_beta_div(y.numel(), _ptr(y), _ptr(x), float(beta), _ptr(out),
                              current_stream()))
    return out


def beta_div_deriv_dev(y, x, beta):
    out = torch.empty_like(y)
    check(lib().bsgp_beta_div_deriv(y.numel(), _ptr(y), _ptr(x), float(beta), _ptr(out),
                                    current_stream()))
    return out


def grad_parts_dev(den, gn, beta):
    p1 = torch.empty_like(den)
    w = torch.empty_like(den)
    check(lib().bsgp_beta_div_grad_parts(den.numel(), _ptr(den), _ptr(gn), float(beta), _ptr(p1),
                                         _ptr(w), current_stream()))
    return p1, w
