// bsgp_api.hip — C-ABI host layer of libbsgp.so (declared in include/bsgp.h).
//
// Owns plans (FFT geometry, twiddles, PSF transfer functions built on the
// device) and per-plan workspaces; validates arguments; launches the kernels
// of bsgp_solver.hip.  No PyTorch types cross this boundary.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <cstdlib>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "bsgp_internal.hpp"
#include "bsgp_psf.hpp"

using namespace bsgp;

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

// A/B override knobs (BSGP_PERWAVE_MIN_WG, BSGP_PERWAVE_TW, BSGP_COOP_ELEMS,
// BSGP_SPIN_LIMIT): a value that is not a whole decimal number in [lo, hi]
// is ignored and the compiled default used, so a typo cannot turn into a
// zero (a spin limit of 0 fails every persistent solve with a timeout).
long long env_knob(const char* name, long long def, long long lo, long long hi) {
  const char* e = getenv(name);
  if (!e || !*e) return def;
  char* end = nullptr;
  errno = 0;
  const long long v = strtoll(e, &end, 10);
  if (errno != 0 || end == e || *end != '\0' || v < lo || v > hi) return def;
  return v;
}

#define HIP_TRY(expr)                                                                  \
  do {                                                                                 \
    hipError_t e_ = (expr);                                                            \
    if (e_ != hipSuccess)                                                              \
      return fail(BSGP_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_));    \
  } while (0)

size_t round_up(size_t v, size_t m) { return (v + m - 1) / m * m; }

// Every entry point that works on a plan's device makes it current for the
// call and gives the caller's thread its own current device back on return
// (a plan destroyed from a garbage-collector thread, or a solve on another
// GPU, must not switch the device the caller's framework is using).
struct DeviceGuard {
  int prev = -1;
  hipError_t err = hipSuccess;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    err = hipSetDevice(dev);
  }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
  DeviceGuard(const DeviceGuard&) = delete;
  DeviceGuard& operator=(const DeviceGuard&) = delete;
};
#define DEVICE_SCOPE(dev)                                                                   \
  DeviceGuard dev_guard_(dev);                                                              \
  if (dev_guard_.err != hipSuccess)                                                         \
    return fail(BSGP_ERR_HIP, std::string("hipSetDevice: ") + hipGetErrorString(dev_guard_.err))

// numpy's float32 np.sum over n contiguous elements (numpy 1.26 and 2.x,
// checked against np.sum in tests/test_oracle.py::test_numpy_f32_sum_model):
// the reduction runs over chunks of 8192 (the ufunc buffer), folding
// res = res + pairwise(chunk) from res = 0; pairwise(n) is a leaf for n <= 128
// (8 strided accumulators, or a plain loop below 8) and otherwise
// pairwise(n2) + pairwise(n - n2) with n2 = n/2 - (n/2) % 8.  The program
// lists the leaves (start, length) in order, the inner nodes (value indices
// of the two operands; values 0..L-1 are the leaves, L+k is node k) grouped
// by height so that a level can be added in parallel, and each chunk's root.
struct PwBuild {
  std::vector<int> leaves, nodes_tmp, heights, roots;
  // returns a temporary id: >= 0 leaf, < 0 node -(k+1); *h = height
  int rec(int start, int n, int* h) {
    if (n <= 128) {
      leaves.push_back(start);
      leaves.push_back(n);
      *h = 0;
      return (int)leaves.size() / 2 - 1;
    }
    int n2 = n / 2;
    n2 -= n2 % 8;
    int ha, hb;
    const int a = rec(start, n2, &ha);
    const int b = rec(start + n2, n - n2, &hb);
    nodes_tmp.push_back(a);
    nodes_tmp.push_back(b);
    *h = (ha > hb ? ha : hb) + 1;
    heights.push_back(*h);
    return -(int)(nodes_tmp.size() / 2);
  }
};

std::vector<int> pairwise_program(long n, PwProg* pp) {
  PwBuild b;
  std::vector<int> root_tmp;
  for (long c0 = 0; c0 < n; c0 += 8192) {
    int h;
    root_tmp.push_back(b.rec((int)c0, (int)std::min<long>(8192, n - c0), &h));
  }
  const int L = (int)b.leaves.size() / 2, M = (int)b.heights.size();
  int maxh = 0;
  for (int v : b.heights) maxh = std::max(maxh, v);
  // order the nodes by height (stable), then renumber the operands
  std::vector<int> order, newid(M), lev_off(maxh + 1, 0);
  for (int h = 1; h <= maxh; ++h) {
    lev_off[h - 1] = (int)order.size();
    for (int k = 0; k < M; ++k)
      if (b.heights[k] == h) order.push_back(k);
  }
  lev_off[maxh] = (int)order.size();
  for (int i = 0; i < M; ++i) newid[order[i]] = L + i;
  auto val = [&](int t) { return t >= 0 ? t : newid[-t - 1]; };
  std::vector<int> prog(b.leaves);
  for (int i = 0; i < M; ++i) {
    prog.push_back(val(b.nodes_tmp[2 * order[i]]));
    prog.push_back(val(b.nodes_tmp[2 * order[i] + 1]));
  }
  for (int v : lev_off) prog.push_back(v);
  for (int t : root_tmp) prog.push_back(val(t));
  pp->nleaf = L;
  pp->nnode = M;
  pp->nlev = maxh;
  pp->nchunk = (int)root_tmp.size();
  return prog;
}

std::vector<cd> twiddles(int n) {
  std::vector<cd> t(n);
  const long double pi = 3.141592653589793238462643383279502884L;
  for (int k = 0; k < n; ++k) {
    const long double a = -2.0L * pi * (long double)k / (long double)n;
    t[k] = cmk((double)cosl(a), (double)sinl(a));
  }
  return t;
}

}  // namespace

struct bsgp_plan_s {
  int device = 0;
  int conv_mode = 0;
  Geo g{};
  cd* tw = nullptr;     // twiddles for P then Q
  cd* tf = nullptr;     // tfA then tfAT, each Qh*P (n_tf pairs after bsgp_plan_set_psfs)
  int n_tf = 1;         // 1: one PSF for every image; else image i uses pair i (B == n_tf)
  int kh = 0, kw = 0;   // PSF stamp shape of the plan
  size_t lds_fft_bytes = 0;
  size_t lds_bytes = 0;
  int wg_per_cu = 1;
  int resident_per_cu = 1;  // workgroups of every team kernel one CU holds at once
  int ncu = 256;
  // solver workspace
  double* ws = nullptr;
  size_t ws_slots = 0;
  size_t slot_stride = 0;
  size_t vec_stride = 0;
  size_t spec_off = 0;
  ImgState* st = nullptr;
  size_t st_n = 0;
  int* active = nullptr;     // device counter of images still iterating
  int* active_h = nullptr;   // pinned host mirror for polling
  int* done_h = nullptr;     // host-mapped: the solve seq once every image has stopped
  int* done_d = nullptr;     // (its device address)
  int seq = 0;               // the last solve's sequence number (process-wide counter)
  static constexpr int kPollRing = 8;
  hipEvent_t ev_it[kPollRing] = {};  // after iteration it on stream 0 (lookahead polling)
  // sub-batch streams: phases of different sub-batches overlap on the device
  static constexpr int kMaxStreams = 16;
  hipStream_t sub[kMaxStreams] = {};
  hipEvent_t ev_fork = nullptr;
  hipEvent_t ev_join[kMaxStreams] = {};
  int nsub = 0;
  // teams: reduction partials and barrier counters (+ the timeout word)
  double* tpart = nullptr;
  size_t tpart_n = 0;
  unsigned int* tctr = nullptr;
  size_t tctr_bytes = 0;
  // projection pixel lists (proj_cache)
  double* plist = nullptr;
  size_t plist_n = 0;
  // operator workspace
  cd* opws = nullptr;
  size_t opws_slots = 0;
  int storage = BSGP_STORAGE_F64;
  // numpy's float32 reduction order over N elements (gn_f32 solves)
  int* pwprog = nullptr;
  PwProg pw{};
  // persistent solver: dequeue counter + per-image published iterations
  unsigned* pq = nullptr;
  size_t pq_n = 0;
};

// Capacity of one thread's projection list: the pixels it streams in one pass
// (stream2 in bsgp_solver.hip: T == 1 strides pixel pairs over the block; T > 1
// strides row chunks of cp = nfw*W pairs over the members).
static int proj_list_cap(const Geo& g, int T) {
  const long npair = ((long)g.H * g.W + 1) / 2;
  const int nb = plan_block(g);
  if (T == 1) return (int)(2 * ((npair + nb - 1) / nb));
  const long cp = (long)g.nfw * g.W;
  const long nch = (npair + cp - 1) / cp;
  return (int)(2 * ((nch + T - 1) / T) * ((cp + nb - 1) / nb));
}

static int ensure_plist(bsgp_plan p, size_t n) {
  if (n > p->plist_n) {
    if (p->plist) HIP_TRY(hipFree(p->plist));
    p->plist = nullptr;
    p->plist_n = 0;
    HIP_TRY(hipMalloc(&p->plist, n * sizeof(double)));
    p->plist_n = n;
  }
  return BSGP_OK;
}

static int ensure_ws(bsgp_plan p, size_t slots) {
  if (slots > p->ws_slots) {
    if (p->ws) HIP_TRY(hipFree(p->ws));
    p->ws = nullptr;
    p->ws_slots = 0;
    HIP_TRY(hipMalloc(&p->ws, slots * p->slot_stride * sizeof(double)));
    p->ws_slots = slots;
  }
  if (slots > p->st_n) {
    if (p->st) HIP_TRY(hipFree(p->st));
    p->st = nullptr;
    p->st_n = 0;
    HIP_TRY(hipMalloc(&p->st, slots * sizeof(ImgState)));
    p->st_n = slots;
  }
  return BSGP_OK;
}

// Workgroups per image.  Every member of every team must be resident at once
// (the team barriers spin): B*T never exceeds the CUs times the workgroups per
// CU the runtime reports for every team kernel of the plan's build
// (p->resident_per_cu, hipOccupancyMaxActiveBlocksPerMultiprocessor).  Each
// member keeps at least one row pair and one column per FFT wave.
// Solve sequence numbers for the lookahead poll's host-mapped word: one
// process-wide counter, so no plan (nor a reused pinned block) ever sees a
// value another solve wrote.
static std::atomic<int> g_solve_seq{0};

static int choose_team(const bsgp_plan_s* p, int B, int req) {
  if (req == 1) return 1;
  const Geo& g = p->g;
  const int rows2 = (g.H + 1) / 2;
  int tgeo = rows2 / g.nfw;
  if (g.Qh / g.nfw < tgeo) tgeo = g.Qh / g.nfw;
  const int res = p->ncu * p->resident_per_cu / B;  // resident members per image
  // auto: one workgroup per CU (cooperative plans would fit two per CU, but
  // one per CU measured faster on C4: 1262 vs 1180 it/s)
  int T = std::min(p->ncu / B, tgeo);
  if (req > 1) T = std::min(req, tgeo);
  T = std::min(T, res);
  // the barrier words and the group leaders' polls cover at most kMaxTeam
  // members (bsgp_device.hpp)
  T = std::min(T, kMaxTeam);
  return T < 1 ? 1 : T;
}

static int ensure_team(bsgp_plan p, size_t B, int T) {
  const size_t np = B * kPartBufs * (size_t)(T + 8) * kMaxRed;
  if (T > 1 && np > p->tpart_n) {
    if (p->tpart) HIP_TRY(hipFree(p->tpart));
    p->tpart = nullptr;
    p->tpart_n = 0;
    HIP_TRY(hipMalloc(&p->tpart, np * sizeof(double)));
    p->tpart_n = np;
  }
  const size_t cb = round_up((B * kTeamWords + kTeamLine) * sizeof(unsigned int), 128);
  if (cb > p->tctr_bytes) {
    if (p->tctr) HIP_TRY(hipFree(p->tctr));
    p->tctr = nullptr;
    p->tctr_bytes = 0;
    HIP_TRY(hipMalloc(&p->tctr, cb));
    p->tctr_bytes = cb;
  }
  return BSGP_OK;
}

extern "C" {

int32_t bsgp_abi_version(void) { return 3; }

// Diagnostics (not in include/bsgp.h): per-phase shader cycles of a build
// with -DBSGP_PHASE_PROF; returns BSGP_ERR_UNSUPPORTED otherwise.
int bsgp_phase_prof(uint64_t* out, int32_t n, int32_t reset) {
  hipError_t e = phase_prof(reinterpret_cast<unsigned long long*>(out), n, reset);
  if (e == hipErrorNotSupported) return fail(BSGP_ERR_UNSUPPORTED, "built without BSGP_PHASE_PROF");
  if (e != hipSuccess) return fail(BSGP_ERR_HIP, hipGetErrorString(e));
  return BSGP_OK;
}

// Diagnostics (not in include/bsgp.h): the numpy float32 reduction program the
// plans use for N = n elements (tests/test_oracle.py evaluates it against
// np.sum).  counts = {nleaf, nnode, nlev, nchunk}; returns the program length,
// copying at most cap ints to out.
int64_t bsgp_pairwise_program(int64_t n, int32_t* out, int64_t cap, int32_t* counts) {
  if (n < 1) return fail(BSGP_ERR_ARG, "n must be >= 1");
  PwProg pp{};
  const std::vector<int> prog = pairwise_program((long)n, &pp);
  if (counts) {
    counts[0] = pp.nleaf;
    counts[1] = pp.nnode;
    counts[2] = pp.nlev;
    counts[3] = pp.nchunk;
  }
  for (int64_t i = 0; out && i < cap && i < (int64_t)prog.size(); ++i) out[i] = prog[i];
  return (int64_t)prog.size();
}

const char* bsgp_last_error(void) { return g_err.c_str(); }

int bsgp_device_synchronize(void) {
  HIP_TRY(hipDeviceSynchronize());
  return BSGP_OK;
}

int bsgp_plan_create(int32_t H, int32_t W, const double* psf, int32_t kh, int32_t kw,
                     int32_t conv_mode, int32_t storage, int32_t device, bsgp_plan* out) {
  return bsgp_plan_create_checked(H, W, psf, kh, kw, conv_mode, storage, device, 0, out);
}

int bsgp_plan_create_checked(int32_t H, int32_t W, const double* psf, int32_t kh, int32_t kw,
                             int32_t conv_mode, int32_t storage, int32_t device,
                             int32_t psf_checked, bsgp_plan* out) {
  if (!out) return fail(BSGP_ERR_ARG, "out is NULL");
  if (storage != BSGP_STORAGE_F64 && storage != BSGP_STORAGE_F32)
    return fail(BSGP_ERR_ARG, "bad storage");
  *out = nullptr;
  if (H < 1 || W < 1 || kh < 1 || kw < 1 || !psf) return fail(BSGP_ERR_ARG, "bad shape or psf");
  if (conv_mode != BSGP_CONV_CIRCULAR && conv_mode != BSGP_CONV_LINEAR_FILL)
    return fail(BSGP_ERR_ARG, "bad conv_mode");
  if (conv_mode == BSGP_CONV_CIRCULAR && (kh != H || kw != W))
    return fail(BSGP_ERR_ARG,
                "circular A (use_original_SGP_Afunction=True) needs psf.shape == gn.shape");
  // PSF normalisation check (sgp.py:97-102), unless the caller has made it in
  // the PSF's own dtype (a float32 PSF sums to 1 in float32, not in float64)
  if (!psf_checked) {
    double s = 0;
    for (int i = 0; i < kh * kw; ++i) s += psf[i];
    if (std::fabs(s - 1.0) > 1e4 * 2.220446049250313e-16) {
      char b[160];
      snprintf(b, sizeof b, "PSF is not normalized! sum(psf) - 1. = %.17g", s - 1.0);
      return fail(BSGP_ERR_PSF, b);
    }
  }
  DEVICE_SCOPE(device);
  bsgp_plan p = new bsgp_plan_s();
  p->device = device;
  p->conv_mode = conv_mode;
  p->kh = kh;
  p->kw = kw;
  Geo& g = p->g;
  g.H = H;
  g.W = W;
  if (conv_mode == BSGP_CONV_CIRCULAR) {
    g.P = H;
    g.Q = W;
  } else {
    // zero-fill linear convolution on a P x Q circular grid without
    // wrap-around for either kernel (A: kh x kw, AT: kw x kh)
    const int km = kh > kw ? kh : kw;
    int pmin = H + km / 2, qmin = W + km / 2;
    if (pmin < km) pmin = km;
    if (qmin < km) qmin = km;
    g.P = next_fast_len(pmin);
    g.Q = next_fast_len(qmin);
  }
  g.Qh = g.Q / 2 + 1;
  // stored half spectrum: column k at k * sld (BSGP_SPEC_PAD rows of padding
  // break a power-of-two column stride; even, so row pairs stay 32-B aligned)
  g.sld = H + ((H & 1) ? 1 : 0) + BSGP_SPEC_PAD;
  g.fp.n = g.P;
  g.fq.n = g.Q;
  if (!plan_radices(g.P, g.fp.radix, &g.fp.ns) || !plan_radices(g.Q, g.fq.radix, &g.fq.ns)) {
    delete p;
    return fail(BSGP_ERR_UNSUPPORTED, "FFT length has too many factors");
  }
  int maxlen = g.P > g.Q ? g.P : g.Q;
  // one FFT buffer also stages a row pair's stored spectrum (2*Qh, row_inv2); odd spreads banks
  g.lpad = (maxlen + 1 > 2 * g.Qh ? maxlen + 1 : 2 * g.Qh) | 1;
  // LDS: nfw waves x 2 buffers, + reduction scratch
  size_t red_bytes = (size_t)kWaves * kMaxRed * sizeof(double) + kSharedBytes;
  int nfw = kWaves;
  size_t budget = 160 * 1024 / 4 - 256;  // four workgroups per CU
  p->wg_per_cu = 4;
  auto need = [&](int n) { return (size_t)n * 2 * g.lpad * sizeof(cd) + red_bytes; };
  g.coop = 0;
  // per-wave transforms at three workgroups per CU (12 waves/CU) before the
  // cooperative build's one 512-thread workgroup per CU (8 waves): 375^2 tiles
  // on their 400-point grid fit (52.9 KB of 54.3 KB)
  // With BSGP_PERWAVE_TW the twiddle tables must fit beside the buffers too:
  // a wave's transform that reads its twiddles from global memory waits on
  // them in every stage (375^2 tiles at 3 WG/CU: the 400-point row and column
  // transforms took 3.5x the cycles per point of C3's 270-point ones, phase
  // profile), so two workgroups per CU with LDS twiddles can beat three without.
  const size_t twb_all = (size_t)(g.P == g.Q ? g.P : g.P + g.Q) * sizeof(cd);
  {
    const int min_wg = (int)env_knob("BSGP_PERWAVE_MIN_WG", BSGP_PERWAVE_MIN_WG, 2, 4);
    const size_t tw_need = env_knob("BSGP_PERWAVE_TW", BSGP_PERWAVE_TW, 0, 1) ? twb_all : 0;
    for (int wg = 3; wg >= 2 && wg >= min_wg; --wg) {
      const size_t bw = 160 * 1024 / wg - 256;
      if (need(kWaves) > budget && need(kWaves) + tw_need <= bw) {
        budget = bw;
        p->wg_per_cu = wg;
        break;
      }
    }
  }
  if (need(kWaves) > budget) {
    // transforms too long for a wave each at four workgroups per CU: the
    // whole workgroup runs one transform at a time (cooperative passes)
    g.coop = 1;
    nfw = 1;
    budget = 160 * 1024 - 256;
    // wave partials of the cooperative build's workgroups (kCoopBlock threads)
    red_bytes = (size_t)(kCoopBlock / 64) * kMaxRed * sizeof(double) + kSharedBytes;
    if (need(1) > budget) {
      delete p;
      return fail(BSGP_ERR_UNSUPPORTED, "FFT length too large for one workgroup's LDS");
    }
    // thread groups (bsgp_device.hpp, cooperative passes): as many as the LDS
    // holds, each at least two waves and covering its transform in one load
    // batch (4 elements per thread); the 400/480-point grids take four.  A
    // transform too long for that (C4's 2048 points) takes two groups of
    // 256 threads with two load batches (BSGP_COOP_ELEMS = 8) when the LDS
    // holds both: each workgroup then runs two row pairs through the same
    // stages and barriers, and its radix-8 stages use all 512 lanes instead
    // of 256: C4 k_ls 180 -> 157 us, k_bb 72 -> 68 us, 2114 -> 2221 it/s
    // (float32 storage; f64 1868 -> 1971), the column kernel staying on one
    // group (nfc below).
    const int elems = (int)env_knob("BSGP_COOP_ELEMS", BSGP_COOP_ELEMS, 4, 8);  // (A/B override)
    auto groups = [&](int el) {
      for (int n = BSGP_COOP_GROUPS; n > 1; n /= 2)
        if (need(n) <= budget && kCoopBlock / n >= 128 && maxlen <= el * (kCoopBlock / n))
          return n;
      return 1;
    };
    nfw = groups(4);
    if (nfw == 1 && elems > 4) nfw = groups(elems);
    p->wg_per_cu = (int)(budget / need(nfw));
    if (p->wg_per_cu > 4) p->wg_per_cu = 4;
    budget = 160 * 1024 / p->wg_per_cu - 256;
  }
  g.nfw = nfw;
  // the column kernel of a cooperative plan: BSGP_COOP_COLGROUPS groups (0: as the
  // other kernels), so it may fit more workgroups per CU than they do
  // (the column kernel keeps one load batch per thread: a 2048-point column per
  // 256-thread group doubled C4's k_col, 42 -> 75 us, while the row passes gained)
  int nfc = nfw;
  while (g.coop && nfc > 1 && maxlen > 4 * (kCoopBlock / nfc)) nfc /= 2;
  g.nfc = (g.coop && BSGP_COOP_COLGROUPS > 0 && BSGP_COOP_COLGROUPS < nfc) ? BSGP_COOP_COLGROUPS
                                                                            : nfc;
  p->lds_fft_bytes = (size_t)nfw * 2 * g.lpad * sizeof(cd);
  p->lds_bytes = p->lds_fft_bytes + red_bytes;
  // the per-wave transforms' twiddle tables live in LDS when they fit the same
  // budget (one table when P == Q), else they read the global table (as the
  // cooperative workgroup-wide transforms always do)
  g.fp.lds_tw = g.fq.lds_tw = -1;
  g.fp.lds_tw2 = g.fq.lds_tw2 = -1;
  g.tw2 = 0;
  g.twmix = -1;
  // cooperative 2048-point transforms (fft_wide's static plan): their twiddles
  // as a two-level table (bsgp_fft.hpp Tw2, 1.5 KiB) at the start of every
  // kernel's LDS -- the full 32 KiB table does not fit beside the buffers, and
  // from global memory every Stockham stage waited on an L2 round trip
  // and, after them, the 2048-point column transforms' stage tables
  // (bsgp_fft.hpp TwMixL: 9 KiB, the global table's entries for the second and
  // third Stockham stages; loaded by every kernel with the two-level tables)
  if (g.coop && (BSGP_COOP_TW2 || BSGP_COL_TWMIX)) {
    size_t off = 0;
    if (BSGP_COOP_TW2) {
      if (g.P == 2048) {
        g.fp.lds_tw2 = 0;
        off += (64 + 2048 / 64) * sizeof(cd);
      }
      if (g.Q == 2048) {
        if (g.P == 2048) {
          g.fq.lds_tw2 = 0;
        } else {
          g.fq.lds_tw2 = (int)off;
          off += (64 + 2048 / 64) * sizeof(cd);
        }
      }
    }
    if (BSGP_COL_TWMIX && !BSGP_COL_TW2 && g.P == 2048) {
      g.twmix = (int)off;
      off += (64 + 512) * sizeof(cd);
    }
    g.tw2 = (int)round_up(off, 16);
    p->lds_bytes += g.tw2;
  }
  if (!g.coop) {
    const size_t twb = (size_t)(g.P == g.Q ? g.P : g.P + g.Q) * sizeof(cd);
    if (p->lds_bytes + twb <= budget) {
      g.fp.lds_tw = (int)p->lds_bytes;
      g.fq.lds_tw = g.P == g.Q ? g.fp.lds_tw : (int)(p->lds_bytes + (size_t)g.P * sizeof(cd));
      p->lds_bytes += twb;
    }
  }
  {
    int ncu = 0;
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess &&
        ncu > 0)
      p->ncu = ncu;
  }
  if (BSGP_COOP512 && (bsgp_c512_args_size() != sizeof(SolveArgs) ||
                       bsgp_c512_block() != kCoopBlock)) {
    delete p;
    return fail(BSGP_ERR_HIP, "cooperative 512-thread build does not match this library");
  }
  if (bsgp_app_args_size() != sizeof(SolveArgs)) {
    delete p;
    return fail(BSGP_ERR_HIP, "application-size persistent build does not match this library");
  }
  if (set_solver_lds_limit(p->lds_bytes) != hipSuccess) {
    delete p;
    return fail(BSGP_ERR_HIP, "hipFuncSetAttribute(MaxDynamicSharedMemorySize) failed");
  }
  if (team_resident_per_cu(g.coop != 0, storage, p->lds_bytes, &p->resident_per_cu) !=
          hipSuccess ||
      p->resident_per_cu < 1) {
    delete p;
    return fail(BSGP_ERR_HIP, "occupancy query of the team kernels failed");
  }
  // twiddles
  {
    std::vector<cd> tw = twiddles(g.P);
    std::vector<cd> twq = twiddles(g.Q);
    tw.insert(tw.end(), twq.begin(), twq.end());
    if (hipMalloc(&p->tw, tw.size() * sizeof(cd)) != hipSuccess ||
        hipMemcpy(p->tw, tw.data(), tw.size() * sizeof(cd), hipMemcpyHostToDevice) != hipSuccess) {
      bsgp_plan_destroy(p);
      return fail(BSGP_ERR_HIP, "twiddle upload failed");
    }
    g.fp.tw = p->tw;
    g.fq.tw = p->tw + g.P;
  }
  // circularly-placed kernels for A and AT on the P x Q grid
  const size_t PQ = (size_t)g.P * g.Q;
  std::vector<double> kA(PQ, 0.0), kAT(PQ, 0.0);
  if (conv_mode == BSGP_CONV_CIRCULAR) {
    // fftshift(psf): out[i][j] = psf[(i - H//2) mod H][(j - W//2) mod W]  (sgp.py:109)
    for (int i = 0; i < H; ++i)
      for (int j = 0; j < W; ++j) {
        const int si = ((i - H / 2) % H + H) % H, sj = ((j - W / 2) % W + W) % W;
        kA[(size_t)i * W + j] = psf[(size_t)si * W + sj];
      }
  } else {
    // astropy convolve_fft(normalize_kernel=True): kernel/sum, centre at k//2
    // (convolve.py:664-672, 770-787); AT uses psf.conj().T (sgp.py:157)
    double s = 0;
    for (int i = 0; i < kh * kw; ++i) s += psf[i];
    for (int u = 0; u < kh; ++u)
      for (int v = 0; v < kw; ++v) {
        const double val = psf[(size_t)u * kw + v] / s;
        const int a = ((u - kh / 2) % g.P + g.P) % g.P, b = ((v - kw / 2) % g.Q + g.Q) % g.Q;
        kA[(size_t)a * g.Q + b] += val;
        // transposed kernel T[v][u] (shape kw x kh), centre (kw//2, kh//2)
        const int at = ((v - kw / 2) % g.P + g.P) % g.P, bt = ((u - kh / 2) % g.Q + g.Q) % g.Q;
        kAT[(size_t)at * g.Q + bt] += val;
      }
  }
  double* kc = nullptr;
  cd* spec = nullptr;
  const size_t tfn = (size_t)g.Qh * g.P;
  int rc = BSGP_OK;
  if (hipMalloc(&p->tf, 2 * tfn * sizeof(cd)) != hipSuccess ||
      hipMalloc(&kc, 2 * PQ * sizeof(double)) != hipSuccess ||
      hipMalloc(&spec, (size_t)g.P * g.Qh * sizeof(cd)) != hipSuccess) {
    rc = fail(BSGP_ERR_HIP, "plan allocation failed");
  }
  if (rc == BSGP_OK) {
    g.tfA = p->tf;
    g.tfAT = p->tf + tfn;
    const double scale = 1.0 / ((double)g.P * (double)g.Q);
    if (hipMemcpy(kc, kA.data(), PQ * sizeof(double), hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(kc + PQ, kAT.data(), PQ * sizeof(double), hipMemcpyHostToDevice) != hipSuccess)
      rc = fail(BSGP_ERR_HIP, "psf upload failed");
    if (rc == BSGP_OK) {
      if (launch_build_tf(g, kc, spec, p->tf, scale, 0, p->lds_bytes, 0) != hipSuccess)
        rc = fail(BSGP_ERR_HIP, "build_tf(A) launch failed");
      else if (hipDeviceSynchronize() != hipSuccess)
        rc = fail(BSGP_ERR_HIP, "build_tf(A) failed");
    }
    if (rc == BSGP_OK) {
      // circular: TF_AT = conj(TF_A) (sgp.py:110); linear: FFT of the transposed kernel
      const bool circ = conv_mode == BSGP_CONV_CIRCULAR;
      if (launch_build_tf(g, circ ? kc : kc + PQ, spec, p->tf + tfn, scale, circ ? 1 : 0,
                          p->lds_bytes, 0) != hipSuccess)
        rc = fail(BSGP_ERR_HIP, "build_tf(AT) launch failed");
      else if (hipDeviceSynchronize() != hipSuccess)
        rc = fail(BSGP_ERR_HIP, "build_tf(AT) failed");
    }
  }
  if (kc) (void)hipFree(kc);
  if (spec) (void)hipFree(spec);
  if (rc != BSGP_OK) {
    std::string m = g_err;
    bsgp_plan_destroy(p);
    return fail(rc, m);
  }
  const size_t N = (size_t)H * W;
  p->storage = storage;
  // slot: gn and bkg in float64 (vec_stride each), the seven iteration vectors
  // in the storage type, then the half spectrum (complex float64)
  p->vec_stride = round_up(N, 32) + BSGP_VEC_PAD;
  const size_t vbytes = storage == BSGP_STORAGE_F32 ? sizeof(float) : sizeof(double);
  p->spec_off = 2 * p->vec_stride + 7 * p->vec_stride * vbytes / sizeof(double);
  p->slot_stride = p->spec_off + round_up((size_t)g.sld * g.Qh * 2, 32);
  {
    const std::vector<int> prog = pairwise_program((long)N, &p->pw);
    if (hipMalloc(&p->pwprog, prog.size() * sizeof(int)) != hipSuccess ||
        hipMemcpy(p->pwprog, prog.data(), prog.size() * sizeof(int), hipMemcpyHostToDevice) !=
            hipSuccess) {
      bsgp_plan_destroy(p);
      return fail(BSGP_ERR_HIP, "pairwise program upload failed");
    }
    p->pw.prog = p->pwprog;
  }
  if (hipMalloc(&p->active, 256) != hipSuccess ||
      hipHostMalloc(&p->active_h, 256, hipHostMallocDefault) != hipSuccess ||
      hipHostMalloc(&p->done_h, 256, hipHostMallocMapped) != hipSuccess ||
      hipHostGetDevicePointer((void**)&p->done_d, p->done_h, 0) != hipSuccess) {
    bsgp_plan_destroy(p);
    return fail(BSGP_ERR_HIP, "counter allocation failed");
  }
  // a reused pinned block may still hold an old plan's seq; seqs
  // also come from one process-wide counter, so a stale word never matches
  *p->done_h = 0;
  *out = p;
  return BSGP_OK;
}

int bsgp_plan_destroy(bsgp_plan p) {
  if (!p) return BSGP_OK;
  DeviceGuard dev_guard_(p->device);
  if (p->tw) (void)hipFree(p->tw);
  if (p->tf) (void)hipFree(p->tf);
  if (p->ws) (void)hipFree(p->ws);
  for (int i = 1; i < p->nsub; ++i) {
    if (p->sub[i]) (void)hipStreamDestroy(p->sub[i]);
    if (p->ev_join[i]) (void)hipEventDestroy(p->ev_join[i]);
  }
  if (p->ev_fork) (void)hipEventDestroy(p->ev_fork);
  if (p->st) (void)hipFree(p->st);
  if (p->active) (void)hipFree(p->active);
  if (p->active_h) (void)hipHostFree(p->active_h);
  if (p->done_h) (void)hipHostFree(p->done_h);
  for (hipEvent_t e : p->ev_it)
    if (e) (void)hipEventDestroy(e);
  if (p->opws) (void)hipFree(p->opws);
  if (p->tpart) (void)hipFree(p->tpart);
  if (p->tctr) (void)hipFree(p->tctr);
  if (p->plist) (void)hipFree(p->plist);
  if (p->pwprog) (void)hipFree(p->pwprog);
  if (p->pq) (void)hipFree(p->pq);
  delete p;
  return BSGP_OK;
}

int bsgp_plan_set_psfs(bsgp_plan p, const double* psfs, int32_t n, void* stream) {
  if (!p || !psfs || n < 1) return fail(BSGP_ERR_ARG, "bad arguments");
  Geo& g = p->g;
  const bool circ = p->conv_mode == BSGP_CONV_CIRCULAR;
  // the device placement stores (no accumulation): the kernel must not wrap on the grid
  if (!circ && (p->kh > g.P || p->kw > g.Q || p->kw > g.P || p->kh > g.Q))
    return fail(BSGP_ERR_ARG, "per-image PSFs need a kernel no larger than the FFT grid");
  DEVICE_SCOPE(p->device);
  hipStream_t s = (hipStream_t)stream;
  const size_t PQ = (size_t)g.P * g.Q, tfn = (size_t)g.Qh * g.P, specn = (size_t)g.P * g.Qh;
  // chunks bound the placement/spectrum workspace (~256 MiB)
  const size_t per = 2 * PQ * sizeof(double) + specn * sizeof(cd);
  const int chunk = (int)std::max<size_t>(1, std::min<size_t>((size_t)n, (256u << 20) / per));
  cd* tf = nullptr;
  double* kc = nullptr;
  cd* spec = nullptr;
  double* sums = nullptr;
  int rc = BSGP_OK;
  if (hipMalloc(&tf, (size_t)n * 2 * tfn * sizeof(cd)) != hipSuccess ||
      hipMalloc(&kc, (size_t)chunk * 2 * PQ * sizeof(double)) != hipSuccess ||
      hipMalloc(&spec, (size_t)chunk * specn * sizeof(cd)) != hipSuccess ||
      hipMalloc(&sums, (size_t)n * sizeof(double)) != hipSuccess)
    rc = fail(BSGP_ERR_HIP, "per-image PSF allocation failed");
  const double scale = 1.0 / ((double)g.P * (double)g.Q);
  Geo gb = g;
  gb.tf_stride = 0;
  for (int c0 = 0; rc == BSGP_OK && c0 < n; c0 += chunk) {
    const int m = std::min(chunk, n - c0);
    cd* t = tf + (size_t)c0 * 2 * tfn;
    if (hipMemsetAsync(kc, 0, (size_t)m * 2 * PQ * sizeof(double), s) != hipSuccess ||
        launch_place_psfs(gb, m, psfs + (size_t)c0 * p->kh * p->kw, p->kh, p->kw, circ ? 1 : 0,
                          kc, sums + c0, s) != hipSuccess ||
        launch_build_tfs(gb, m, kc, 2 * PQ, spec, specn, t, 2 * tfn, scale, 0, p->lds_bytes,
                         s) != hipSuccess ||
        // circular: TF_AT = conj(TF_A) (sgp.py:110); linear: FFT of the transposed kernel
        launch_build_tfs(gb, m, circ ? kc : kc + PQ, 2 * PQ, spec, specn, t + tfn, 2 * tfn,
                         scale, circ ? 1 : 0, p->lds_bytes, s) != hipSuccess)
      rc = fail(BSGP_ERR_HIP, "per-image TF launch failed");
  }
  std::vector<double> hs(n);
  if (rc == BSGP_OK && (hipMemcpyAsync(hs.data(), sums, (size_t)n * sizeof(double),
                                       hipMemcpyDeviceToHost, s) != hipSuccess ||
                        hipStreamSynchronize(s) != hipSuccess))
    rc = fail(BSGP_ERR_HIP, "per-image TF build failed");
  for (int i = 0; rc == BSGP_OK && i < n; ++i)
    if (!(std::fabs(hs[i] - 1.0) <= 1e4 * 2.220446049250313e-16)) {  // sgp.py:97-102
      char b[160];
      snprintf(b, sizeof b, "PSF %d is not normalized! sum(psf) - 1. = %.17g", i, hs[i] - 1.0);
      rc = fail(BSGP_ERR_PSF, b);
    }
  if (kc) (void)hipFree(kc);
  if (spec) (void)hipFree(spec);
  if (sums) (void)hipFree(sums);
  if (rc != BSGP_OK) {
    if (tf) (void)hipFree(tf);
    return rc;
  }
  if (p->tf) (void)hipFree(p->tf);
  p->tf = tf;
  p->n_tf = n;
  g.tfA = tf;
  g.tfAT = tf + tfn;
  g.tf_stride = n > 1 ? 2 * tfn : 0;
  return BSGP_OK;
}

int bsgp_plan_info(bsgp_plan p, int32_t* P, int32_t* Q, int64_t* slot_bytes,
                   int32_t* fft_waves) {
  if (!p) return fail(BSGP_ERR_ARG, "plan is NULL");
  if (P) *P = p->g.P;
  if (Q) *Q = p->g.Q;
  if (slot_bytes) *slot_bytes = (int64_t)(p->slot_stride * sizeof(double));
  if (fft_waves) *fft_waves = p->g.nfw;
  return BSGP_OK;
}

static int check_params(const bsgp_params* q) {
  if (!q) return fail(BSGP_ERR_ARG, "params is NULL");
  if (q->variant != BSGP_VARIANT_KL && q->variant != BSGP_VARIANT_BETA)
    return fail(BSGP_ERR_ARG, "bad variant");
  if (q->MAXIT < 1) return fail(BSGP_ERR_ARG, "MAXIT must be >= 1");
  if (q->M_alpha < 1 || q->M_alpha > 32) return fail(BSGP_ERR_ARG, "M_alpha must be in [1, 32]");
  if (q->M < 1 || q->M > 32) return fail(BSGP_ERR_ARG, "M must be in [1, 32]");
  if (q->ls_spec < 1 || q->ls_spec > 8) return fail(BSGP_ERR_ARG, "ls_spec must be in [1, 8]");
  if (q->init_recon < 0 || q->init_recon > 3) return fail(BSGP_ERR_ARG, "bad init_recon");
  if (q->proj_type != 0 && q->proj_type != 1) return fail(BSGP_ERR_ARG, "bad proj_type");
  if (q->scale_data < 0 || q->scale_data > 2) return fail(BSGP_ERR_ARG, "bad scale_data");
  if (q->flux_f32 && !(q->gn_f32 && q->scale_data != 2))
    return fail(BSGP_ERR_ARG, "flux_f32 needs gn_f32 with scale_data 0 or 1");
  return BSGP_OK;
}

// Profiled solves: events around every kernel class of every iteration.
struct SolveProf {
  std::vector<hipEvent_t> ev;  // [MAXIT][6] + setup pair
  double* kernel_ms;
  int64_t* launches;
};

static int solve_impl(bsgp_plan p, int32_t B, const bsgp_params* prm, const bsgp_inputs* in,
                      const bsgp_outputs* out, void* stream, SolveProf* prof);

int bsgp_solve_device(bsgp_plan p, int32_t B, const bsgp_params* prm, const bsgp_inputs* in,
                      const bsgp_outputs* out, void* stream) {
  return solve_impl(p, B, prm, in, out, stream, nullptr);
}

int bsgp_solve_profiled(bsgp_plan p, int32_t B, const bsgp_params* prm, const bsgp_inputs* in,
                        const bsgp_outputs* out, void* stream, double* kernel_ms,
                        int64_t* launches) {
  if (!kernel_ms || !launches) return fail(BSGP_ERR_ARG, "kernel_ms / launches missing");
  if (!prm) return fail(BSGP_ERR_ARG, "params is NULL");
  if (!p) return fail(BSGP_ERR_ARG, "plan is NULL");
  DEVICE_SCOPE(p->device);
  SolveProf prof;
  prof.kernel_ms = kernel_ms;
  prof.launches = launches;
  const size_t nev = 6 * (size_t)(prm->MAXIT > 0 ? prm->MAXIT : 0) + 2;
  prof.ev.resize(nev, nullptr);
  int rc = BSGP_OK;
  for (size_t i = 0; i < nev && rc == BSGP_OK; ++i)
    if (hipEventCreate(&prof.ev[i]) != hipSuccess) rc = fail(BSGP_ERR_HIP, "event create failed");
  if (rc == BSGP_OK) {
    bsgp_params q = *prm;
    q.streams = 1;  // one stream: kernel spans do not overlap
    rc = solve_impl(p, B, &q, in, out, stream, &prof);
  }
  for (hipEvent_t e : prof.ev)
    if (e) (void)hipEventDestroy(e);
  return rc;
}

static int solve_impl(bsgp_plan p, int32_t B, const bsgp_params* prm, const bsgp_inputs* in,
                      const bsgp_outputs* out, void* stream, SolveProf* prof) {
  if (!p) return fail(BSGP_ERR_ARG, "plan is NULL");
  int rc = check_params(prm);
  if (rc) return rc;
  if (B < 1) return fail(BSGP_ERR_ARG, "B must be >= 1");
  if (!in || !in->gn || !in->bkg) return fail(BSGP_ERR_ARG, "inputs gn/bkg missing");
  if ((prm->init_recon == 1 || prm->scale_data == 2) && !in->x0)
    return fail(BSGP_ERR_ARG, "init_recon=1 and scale_data=2 need x0");
  if (!out || !out->x || !out->iters || !out->discr) return fail(BSGP_ERR_ARG, "outputs missing");
  if (out->err && !in->obj) return fail(BSGP_ERR_ARG, "err needs the ground truth obj");
  if (p->n_tf > 1 && B != p->n_tf)
    return fail(BSGP_ERR_ARG, "the plan holds one PSF per image: B must equal its PSF count");
  DEVICE_SCOPE(p->device);
  rc = ensure_ws(p, (size_t)B);
  if (rc) return rc;
  const int T = choose_team(p, B, prm->team);
  rc = ensure_team(p, (size_t)B, T);
  if (rc) return rc;
  SolveArgs a;
  a.g = p->g;
  a.prm = *prm;
  a.in = *in;
  a.out = *out;
  a.B = B;
  a.img0 = 0;
  a.nimg = B;
  a.st = p->st;
  a.active = p->active;
  a.ws = p->ws;
  a.slot_stride = p->slot_stride;
  a.vec_stride = p->vec_stride;
  a.lds_fft_bytes = p->lds_fft_bytes;
  a.T = T;
  // k_col has no team reduction, so a team image may spread its columns over
  // more workgroups than the team has (C4: 1025 columns, 256-member team)
  a.Tc = T;
  if (T > 1) {
    // (one-group cooperative columns pair column 0 with the Nyquist column)
    const int ncol = (p->g.coop && p->g.nfc == 1 && BSGP_COL_PAIR_NYQ && p->g.Q % 2 == 0)
                         ? p->g.Qh - 1
                         : p->g.Qh;
    const int nc = (ncol + p->g.nfc - 1) / p->g.nfc;
    const int want = 4 * p->ncu / B;
    a.Tc = std::max(T, std::min(nc, want));
  }
  // column passes fused into the row kernels: one-workgroup images always;
  // teams of per-wave plans as BSGP_FUSE_COL_TEAM says (the team's own waves
  // run the columns after a team barrier, instead of a k_col launch)
  a.fuse_col = T == 1 ? BSGP_FUSE_COL : (p->g.coop ? 0 : BSGP_FUSE_COL_TEAM);
  a.tpart = T > 1 ? p->tpart : nullptr;
  a.tctr = p->tctr;
  a.tfail = reinterpret_cast<int*>(p->tctr + (size_t)B * kTeamWords);
  a.plist = nullptr;
  a.plist_stride = 0;
  a.lcap = 0;
  a.list_lds = 0;
  a.pw = p->pw;
  a.storage = p->storage;
  a.spec_off = p->spec_off;
  a.spin_limit = (unsigned)env_knob("BSGP_SPIN_LIMIT", 1ll << 26, 0, 0xffffffffll);
  a.ls_cap = (prm->beta > 0.0 && prm->beta < 1.0)
                 ? (int)std::ceil(std::log(1e-12) / std::log(prm->beta)) + 2
                 : 4096;
  if (prm->proj_cache && prm->proj_type == 1) {
    a.lcap = proj_list_cap(p->g, T);
    const size_t half = round_up((size_t)a.lcap * T * plan_block(p->g), 32);
    a.plist_stride = 2 * half;
    rc = ensure_plist(p, (size_t)B * a.plist_stride);
    if (rc) return rc;
    a.plist = p->plist;
    if (BSGP_LIST_LDS && T > 1) {
      const size_t fit = p->lds_fft_bytes / ((size_t)plan_block(p->g) * 2 * sizeof(double));
      a.list_lds = (int)std::min<size_t>((size_t)a.lcap, fit);
    }
  }
  hipStream_t s = (hipStream_t)stream;
  const int K = (prm->adapt_beta && prm->variant == BSGP_VARIANT_BETA)
                    ? 1
                    : (prm->ls_spec <= 1 ? 1 : prm->ls_spec <= 2 ? 2 : prm->ls_spec <= 4 ? 4 : 8);
  // Sub-batches on their own streams (fork/join with the caller's stream):
  // while one sub-batch runs the compute-bound line search the other can
  // stream its memory-bound phases.
  int S = prm->streams < 1 ? 1 : prm->streams;
  if (S > bsgp_plan_s::kMaxStreams) S = bsgp_plan_s::kMaxStreams;
  if (S > B) S = B;
  // per-iteration error / iterate snapshots (errflag, save): one small kernel
  // after setup and after every iteration, off the hot kernels
  const bool track = out->err != nullptr || out->x_iter != nullptr;
  // persistent solver (one launch for every iteration, k_persist): one-workgroup
  // images, with per-wave transforms or (cooperative plans: the application's
  // 375^2 / 450^2 subdivisions) the 512-thread build's thread-group transforms
  // (bsgp_persist_c512.hip); it overlaps the phases of different images itself,
  // so it runs the whole batch as one sub-batch
  const bool persist = prm->persistent && T == 1 && (!p->g.coop || BSGP_COOP512) && !track;
  if (persist) S = 1;
  // fixed-length persistent solves run every image's setup as the first task
  // of its chain inside k_persist: the setups of the last images overlap the
  // first iterations of the others, with no k_setup launch and no boundary
  // (BSGP_FOLD_SETUP=0: k_setup first, for A/B)
  const bool ring = prm->stop_criterion >= 2 && prm->stop_criterion <= 4;
  a.fold_setup = (persist && !ring && env_knob("BSGP_FOLD_SETUP", 1, 0, 1)) ? 1 : 0;
  // sub-batch 0 runs on the caller's stream itself, sub-batches 1..S-1 on the
  // plan's streams: S streams in all, so S = 4 fits the 4 hardware queues HIP
  // opens per process (GPU_MAX_HW_QUEUES)
  if (S > 1 && p->nsub < S) {
    if (!p->ev_fork) HIP_TRY(hipEventCreateWithFlags(&p->ev_fork, hipEventDisableTiming));
    for (int i = (p->nsub > 1 ? p->nsub : 1); i < S; ++i) {
      HIP_TRY(hipStreamCreateWithFlags(&p->sub[i], hipStreamNonBlocking));
      HIP_TRY(hipEventCreateWithFlags(&p->ev_join[i], hipEventDisableTiming));
    }
    p->nsub = S;
  }
  // device counter of images not yet stopped: B, counted down by every image
  // the setup or k_bb stops (count_stopped); the last one writes this solve's
  // seq to the host-mapped word
  HIP_TRY(hipMemsetD32Async((hipDeviceptr_t)p->active, B, 1, s));
  a.seq = g_solve_seq.fetch_add(1, std::memory_order_relaxed) + 1;
  p->seq = a.seq;
  a.done_host = p->done_d;
  // team barrier counters and the timeout word restart at 0 every solve
  HIP_TRY(hipMemsetAsync(p->tctr, 0, p->tctr_bytes, s));
  // flag barriers: every partial slot starts empty
  if (T > 1 && (T <= BSGP_TEAM_FLAGS || (BSGP_TEAM_HIER && T >= 8)))
    HIP_TRY(hipMemsetD32Async((hipDeviceptr_t)p->tpart, kPartEmptyWord,
                              B * kPartBufs * (size_t)(T + 8) * kMaxRed * 2, s));
  hipStream_t ss[bsgp_plan_s::kMaxStreams];
  SolveArgs sa[bsgp_plan_s::kMaxStreams];
  if (S > 1) HIP_TRY(hipEventRecord(p->ev_fork, s));
  for (int j = 0; j < S; ++j) {
    ss[j] = j > 0 ? p->sub[j] : s;
    if (j > 0) HIP_TRY(hipStreamWaitEvent(ss[j], p->ev_fork, 0));
    sa[j] = a;
    sa[j].img0 = (int)((int64_t)B * j / S);
    sa[j].nimg = (int)((int64_t)B * (j + 1) / S) - sa[j].img0;
    if (prof) HIP_TRY(hipEventRecord(prof->ev[0], ss[j]));
    if (!a.fold_setup) HIP_TRY(launch_setup(sa[j], p->lds_bytes, ss[j]));
    if (prof) HIP_TRY(hipEventRecord(prof->ev[1], ss[j]));
    if (track) HIP_TRY(launch_track(sa[j], 0, ss[j]));
  }
  if (persist) {
    const size_t need = (size_t)2 * B + 4;  // head, tail, pad, ready ring[B] (64-bit entries)
    if (need > p->pq_n) {
      if (p->pq) HIP_TRY(hipFree(p->pq));
      p->pq = nullptr;
      p->pq_n = 0;
      HIP_TRY(hipMalloc(&p->pq, need * sizeof(unsigned)));
      p->pq_n = need;
    }
    HIP_TRY(hipMemsetAsync(p->pq, 0, need * sizeof(unsigned), s));
    int per_cu = 0;
    HIP_TRY(persist_resident_per_cu(sa[0], K, p->lds_bytes, &per_cu));
    if (per_cu < 1) return fail(BSGP_ERR_HIP, "persistent solver does not fit a CU");
    // every workgroup resident at once (a dequeued task's predecessor is always
    // running or done); no more workgroups than images
    const int grid = (int)std::min<long>(B, (long)p->ncu * per_cu);
    if (prof) HIP_TRY(hipEventRecord(prof->ev[2], s));
    HIP_TRY(launch_persist(sa[0], K, p->lds_bytes, s, p->pq, p->pq + 1, grid));
    if (prof) {
      HIP_TRY(hipEventRecord(prof->ev[3], s));
      HIP_TRY(hipStreamSynchronize(s));
      for (int k = 0; k < 6; ++k) {
        prof->kernel_ms[k] = 0.0;
        prof->launches[k] = 0;
      }
      float ms = 0.f;
      HIP_TRY(hipEventElapsedTime(&ms, prof->ev[0], prof->ev[1]));
      // (a folded setup runs inside k_persist: no k_setup launch)
      prof->kernel_ms[0] = a.fold_setup ? 0.0 : ms;
      prof->launches[0] = a.fold_setup ? 0 : 1;
      HIP_TRY(hipEventElapsedTime(&ms, prof->ev[2], prof->ev[3]));
      prof->kernel_ms[5] = ms;
      prof->launches[5] = 1;
    }
    return BSGP_OK;
  }
  // Fixed-length runs (stop_criterion 0/1) are launched back to back with no
  // host synchronisation.  Data-dependent stop rules are polled with
  // lookahead: the host keeps at most kLook iterations queued ahead of the
  // device (it waits for the event after iteration it - kLook, never for the
  // stream to drain) and stops enqueueing once the host-mapped word carries
  // this solve's seq, i.e. every image has stopped; the iterations queued
  // past the last stop find every image stopped and return at once.  (Round 4
  // drained the stream and copied the counter after EVERY iteration for
  // B <= 4: one host round trip per iteration on the latency-bound
  // single-image solves.)
  const bool data_stop = prm->stop_criterion >= 2 && prm->stop_criterion <= 4;
  constexpr int kLook = 2;
  if (data_stop)
    for (int i = 0; i < bsgp_plan_s::kPollRing; ++i)
      if (!p->ev_it[i]) HIP_TRY(hipEventCreateWithFlags(&p->ev_it[i], hipEventDisableTiming));
  int it_run = 0;
  for (int it = 1; it <= prm->MAXIT; ++it) {
    it_run = it;
    for (int j = 0; j < S; ++j) {
      HIP_TRY(launch_iteration(sa[j], K, p->lds_bytes, ss[j],
                               prof ? &prof->ev[2 + 6 * (size_t)(it - 1)] : nullptr));
      if (track) HIP_TRY(launch_track(sa[j], it, ss[j]));
    }
    if (data_stop && it < prm->MAXIT && !BSGP_POLL_LOOKAHEAD) {  // (A/B: round 4's polling)
      for (int j = 0; j < S; ++j) HIP_TRY(hipStreamSynchronize(ss[j]));
      if (__atomic_load_n(p->done_h, __ATOMIC_ACQUIRE) == a.seq) break;
    } else if (data_stop && it < prm->MAXIT) {
      HIP_TRY(hipEventRecord(p->ev_it[it % bsgp_plan_s::kPollRing], ss[0]));
      if (it > kLook) {
        HIP_TRY(hipEventSynchronize(p->ev_it[(it - kLook) % bsgp_plan_s::kPollRing]));
        if (__atomic_load_n(p->done_h, __ATOMIC_ACQUIRE) == a.seq) break;
      }
    }
  }
  if (S > 1) {
    for (int j = 1; j < S; ++j) {
      HIP_TRY(hipEventRecord(p->ev_join[j], ss[j]));
      HIP_TRY(hipStreamWaitEvent(s, p->ev_join[j], 0));
    }
  }
  if (prof) {
    // kernel classes: 0 setup, 1 dir, 2 col (A and AT launches), 3 ls, 4 bb
    HIP_TRY(hipStreamSynchronize(s));
    for (int k = 0; k < 6; ++k) {
      prof->kernel_ms[k] = 0.0;
      prof->launches[k] = 0;
    }
    float ms = 0.f;
    HIP_TRY(hipEventElapsedTime(&ms, prof->ev[0], prof->ev[1]));
    prof->kernel_ms[0] = ms;
    prof->launches[0] = 1;
    const int cls[5] = {1, 2, 3, 2, 4};
    const bool launched[5] = {true, !(sa[0].fuse_col & 5), true, !(sa[0].fuse_col & 2), true};
    for (int it = 0; it < it_run; ++it) {
      hipEvent_t* e = &prof->ev[2 + 6 * (size_t)it];
      for (int k = 0; k < 5; ++k) {
        HIP_TRY(hipEventElapsedTime(&ms, e[k], e[k + 1]));
        prof->kernel_ms[cls[k]] += ms;
        if (launched[k]) prof->launches[cls[k]] += 1;
      }
    }
  }
  return BSGP_OK;
}

int bsgp_solve_host(bsgp_plan p, int32_t B, const bsgp_params* prm, const bsgp_inputs* in,
                    const bsgp_outputs* out) {
  if (!p) return fail(BSGP_ERR_ARG, "plan is NULL");
  int rc = check_params(prm);
  if (rc) return rc;
  if (B < 1 || !in || !in->gn || !in->bkg || !out || !out->x || !out->iters || !out->discr)
    return fail(BSGP_ERR_ARG, "bad arguments");
  DEVICE_SCOPE(p->device);
  const size_t N = (size_t)p->g.H * p->g.W, M1 = (size_t)prm->MAXIT + 1;
  std::vector<void*> bufs;
  auto dalloc = [&](size_t bytes) -> void* {
    void* d = nullptr;
    if (hipMalloc(&d, bytes ? bytes : 8) != hipSuccess) return nullptr;
    bufs.push_back(d);
    return d;
  };
  auto cleanup = [&]() {
    for (void* b : bufs) (void)hipFree(b);
  };
  bsgp_inputs di{};
  bsgp_outputs dout{};
  const size_t nb = prm->bkg_is_map ? B * N : (size_t)B;
  di.gn = (const double*)dalloc(B * N * 8);
  di.bkg = (const double*)dalloc(nb * 8);
  if (in->flux) di.flux = (const double*)dalloc(B * 8);
  if (in->x0) di.x0 = (const double*)dalloc(B * N * 8);
  if (in->beta0) di.beta0 = (const double*)dalloc(B * 8);
  if (in->obj) di.obj = (const double*)dalloc(B * N * 8);
  dout.x = (double*)dalloc(B * N * 8);
  dout.iters = (int32_t*)dalloc(B * 4);
  dout.discr = (double*)dalloc(B * M1 * 8);
  if (out->times) dout.times = (double*)dalloc(B * M1 * 8);
  if (out->crit) dout.crit = (double*)dalloc(B * M1 * 8);
  if (out->flags) dout.flags = (int32_t*)dalloc(B * M1 * 4);
  if (out->beta_final) dout.beta_final = (double*)dalloc(B * 8);
  if (out->counters) dout.counters = (int64_t*)dalloc(B * 8 * 8);
  if (out->err) dout.err = (double*)dalloc(B * M1 * 8);
  if (out->x_iter) dout.x_iter = (double*)dalloc(B * (M1 - 1) * N * 8);
  for (void* b : bufs)
    if (!b) {
      cleanup();
      return fail(BSGP_ERR_HIP, "device allocation failed");
    }
  auto h2d = [&](const void* d, const void* h, size_t bytes) {
    return hipMemcpy(const_cast<void*>(d), h, bytes, hipMemcpyHostToDevice) == hipSuccess;
  };
  bool ok = h2d(di.gn, in->gn, B * N * 8) && h2d(di.bkg, in->bkg, nb * 8) &&
            (!in->flux || h2d(di.flux, in->flux, B * 8)) &&
            (!in->x0 || h2d(di.x0, in->x0, B * N * 8)) &&
            (!in->beta0 || h2d(di.beta0, in->beta0, B * 8)) &&
            (!in->obj || h2d(di.obj, in->obj, B * N * 8));
  if (!ok) {
    cleanup();
    return fail(BSGP_ERR_HIP, "host to device copy failed");
  }
  rc = bsgp_solve_device(p, B, prm, &di, &dout, nullptr);
  if (rc) {
    std::string m = g_err;
    cleanup();
    return fail(rc, m);
  }
  auto d2h = [&](void* h, const void* d, size_t bytes) {
    return !h || hipMemcpy(h, d, bytes, hipMemcpyDeviceToHost) == hipSuccess;
  };
  ok = hipDeviceSynchronize() == hipSuccess && d2h(out->x, dout.x, B * N * 8) &&
       d2h(out->iters, dout.iters, B * 4) && d2h(out->discr, dout.discr, B * M1 * 8) &&
       (!out->times || d2h(out->times, dout.times, B * M1 * 8)) &&
       (!out->crit || d2h(out->crit, dout.crit, B * M1 * 8)) &&
       (!out->flags || d2h(out->flags, dout.flags, B * M1 * 4)) &&
       (!out->beta_final || d2h(out->beta_final, dout.beta_final, B * 8)) &&
       (!out->counters || d2h(out->counters, dout.counters, B * 64)) &&
       (!out->err || d2h(out->err, dout.err, B * M1 * 8)) &&
       (!out->x_iter || d2h(out->x_iter, dout.x_iter, B * (M1 - 1) * N * 8));
  cleanup();
  if (!ok) return fail(BSGP_ERR_HIP, "solve or device to host copy failed");
  return BSGP_OK;
}

int bsgp_apply_operator(bsgp_plan p, int32_t B, int32_t transpose, const double* x, double* out,
                        void* stream) {
  if (!p || !x || !out || B < 1) return fail(BSGP_ERR_ARG, "bad arguments");
  if (p->n_tf > 1 && B != p->n_tf)
    return fail(BSGP_ERR_ARG, "the plan holds one PSF per image: B must equal its PSF count");
  DEVICE_SCOPE(p->device);
  const int slots = p->ncu * p->wg_per_cu;
  // few images: spread each over many workgroups (rows, columns, rows), one
  // spectrum per image; many images: one persistent workgroup per image
  const bool split = (size_t)B * 4 <= (size_t)slots;
  const int grid = split ? B : (B < slots ? B : slots);
  const size_t stride = round_up((size_t)p->g.sld * p->g.Qh, 16);
  if ((size_t)grid > p->opws_slots) {
    if (p->opws) HIP_TRY(hipFree(p->opws));
    p->opws = nullptr;
    p->opws_slots = 0;
    HIP_TRY(hipMalloc(&p->opws, (size_t)grid * stride * sizeof(cd)));
    p->opws_slots = grid;
  }
  if (split)
    HIP_TRY(launch_apply_op_split(p->g, B, transpose, x, out, p->opws, stride, slots / B,
                                  p->lds_bytes, (hipStream_t)stream));
  else
    HIP_TRY(launch_apply_op(p->g, B, transpose, x, out, p->opws, stride, grid, p->lds_bytes,
                            (hipStream_t)stream));
  return BSGP_OK;
}

int bsgp_project_df(int64_t n, double b, const double* c, const double* dia, double scaling,
                    int32_t has_sat, double ccd_sat_level, double lambda0, double dlambda0,
                    double tol_lam, int32_t biter, int32_t siter, int32_t max_projs, double* x,
                    double* info, void* stream) {
  if (n < 1 || n > 0x7fffffff || !c || !dia || !x || !info)
    return fail(BSGP_ERR_ARG, "bad arguments");
  ProjClip clip{has_sat != 0, ccd_sat_level / scaling - 2.220446049250313e-16};
  HIP_TRY(launch_project_df((int)n, b, c, dia, clip, lambda0, dlambda0, tol_lam, biter, siter,
                            max_projs, x, info, (hipStream_t)stream));
  return BSGP_OK;
}

int bsgp_extract_tiles(const double* img, int32_t H, int32_t W, const int32_t* boxes, int32_t n,
                       int32_t th, int32_t tw, double* out, void* stream) {
  if (!img || !boxes || !out || H < 1 || W < 1 || n < 1 || th < 1 || tw < 1 || th > H || tw > W)
    return fail(BSGP_ERR_ARG, "bad arguments");
  if ((int64_t)n * th > 0x7fffffff) return fail(BSGP_ERR_ARG, "too many tile rows");
  HIP_TRY(launch_extract_tiles(img, W, boxes, n, th, tw, out, (hipStream_t)stream));
  return BSGP_OK;
}

int bsgp_coadd_tiles(const double* tiles, int32_t n, int32_t th, int32_t tw, const int32_t* boxes,
                     int32_t H, int32_t W, double* mean, double* footprint, void* stream) {
  if (!tiles || !boxes || !mean || H < 1 || W < 1 || n < 1 || n > 8192 || th < 1 || tw < 1)
    return fail(BSGP_ERR_ARG, "bad arguments");
  HIP_TRY(launch_coadd_tiles(tiles, n, th, tw, boxes, H, W, mean, footprint, (hipStream_t)stream));
  return BSGP_OK;
}

int bsgp_fits_to_f64(const void* raw, int64_t n, int32_t bitpix, double bscale, double bzero,
                     double* out, void* stream) {
  if (!raw || !out || n < 0) return fail(BSGP_ERR_ARG, "bad arguments");
  if (bitpix != 8 && bitpix != 16 && bitpix != 32 && bitpix != 64 && bitpix != -32 &&
      bitpix != -64)
    return fail(BSGP_ERR_ARG, "BITPIX must be 8, 16, 32, 64, -32 or -64");
  if (n == 0) return BSGP_OK;
  HIP_TRY(launch_fits_to_f64(raw, n, bitpix, bscale, bzero, out, (hipStream_t)stream));
  return BSGP_OK;
}

int bsgp_psf_stamps(const bsgp_psf_model* m, const double* xy, int32_t n, int32_t spatial,
                    int32_t normalize, double* out, void* stream) {
  if (!m || !out || n < 0 || (spatial && !xy) || !m->coeffs)
    return fail(BSGP_ERR_ARG, "bad arguments");
  if (m->hw < 0 || m->hw > 255 || m->ngauss < 1 || m->ldeg < 0 || m->sdeg < 0)
    return fail(BSGP_ERR_ARG, "bad PSF model degrees or half width");
  PsfModel M{};
  M.ncomp = m->ngauss * (m->ldeg + 1) * (m->ldeg + 2) / 2;
  const int nterm = (m->sdeg + 1) * (m->sdeg + 2) / 2;
  const int need = spatial ? M.ncomp * nterm : M.ncomp;
  if (M.ncomp > kPsfMaxLocal || need > kPsfMaxCoef)
    return fail(BSGP_ERR_ARG, "PSF model has too many coefficients");
  if (m->ncoef < need) return fail(BSGP_ERR_ARG, "too few PSF coefficients for the degrees");
  if (n == 0) return BSGP_OK;
  M.cosv = m->cos;
  M.sinv = m->sin;
  M.ax = m->ax;
  M.ay = m->ay;
  M.sig2 = m->sigma_inc * m->sigma_inc;
  M.x_orig = m->x_orig;
  M.y_orig = m->y_orig;
  M.ngauss = m->ngauss;
  M.ldeg = m->ldeg;
  M.sdeg = m->sdeg;
  M.hw = m->hw;
  M.ncoef = need;
  for (int i = 0; i < need; ++i) M.coef[i] = m->coeffs[i];
  HIP_TRY(launch_psf_stamps(M, xy, n, spatial ? 1 : 0, normalize ? 1 : 0, out,
                            (hipStream_t)stream));
  return BSGP_OK;
}

int bsgp_beta_div(int64_t n, const double* y, const double* x, double beta, double* out,
                  void* stream) {
  if (n < 1 || n > 0x7fffffff || !y || !x || !out) return fail(BSGP_ERR_ARG, "bad arguments");
  HIP_TRY(launch_beta_div((int)n, y, x, beta, out, (hipStream_t)stream));
  return BSGP_OK;
}

int bsgp_beta_div_deriv(int64_t n, const double* y, const double* x, double beta, double* out,
                        void* stream) {
  if (n < 1 || !y || !x || !out) return fail(BSGP_ERR_ARG, "bad arguments");
  HIP_TRY(launch_beta_div_deriv(n, y, x, beta, out, (hipStream_t)stream));
  return BSGP_OK;
}

int bsgp_beta_div_grad_parts(int64_t n, const double* den, const double* gn, double beta,
                             double* pow1, double* w, void* stream) {
  if (n < 1 || !den || !gn || !pow1 || !w) return fail(BSGP_ERR_ARG, "bad arguments");
  HIP_TRY(launch_grad_parts(n, den, gn, beta, pow1, w, (hipStream_t)stream));
  return BSGP_OK;
}

}  // extern "C"
