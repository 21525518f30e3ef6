// bsgp_kernels.hpp — the batched beta-SGP phase kernels for gfx950, templated
// on the FFT mode (COOP) and the iterate storage V (double / float), with
// their launchers.  Included by bsgp_solver.hip (float64 storage + the
// standalone kernels) and bsgp_solver_f32.hip (float32 storage): two
// translation units so the two builds compile in parallel.
//
// Reference hot path: restoration/sgp.py:41-438 (sgp, KL) and :506-895
// (sgp_betaDiv), restoration/flux_conserve_proj.py:7-144 (projectDF).
//
// One workgroup = one image in every phase kernel: setup, then per SGP
// iteration k_dir (projection + direction + rows of d), k_col (columns with
// A's transfer function), k_ls (line search + accept + rows of w), k_col (AT),
// k_bb (gradient, x update, Barzilai-Borwein, stop rules).  All scalar
// control runs on the device; per-image state lives in ImgState.
#pragma once

#include <hip/hip_runtime.h>

#include <type_traits>
#include <vector>

#include "bsgp_device.hpp"
#include "bsgp_internal.hpp"

namespace bsgp {

// The phase kernels are sized for 4 waves per SIMD (<= 128 VGPRs): four
// 256-thread workgroups = four images per CU, so a 1024-image batch is
// resident in one round on 256 CUs.
#ifndef BSGP_OCC4
#define BSGP_OCC4 __attribute__((amdgpu_waves_per_eu(4, 8)))
#endif

// Operand batching of the inverse row passes (tuning knobs, see row_inv2)
#ifndef BSGP_LS1_PRE
#define BSGP_LS1_PRE false
#endif
#ifndef BSGP_LS1_JCH
#define BSGP_LS1_JCH 1
#endif
#ifndef BSGP_DIR_ATTR
#define BSGP_DIR_ATTR
#endif
#ifndef BSGP_COL_ATTR
#define BSGP_COL_ATTR
#endif
// k_ls at 3 waves/SIMD (<= 168 VGPRs; a few spills) with single-column operand
// batches and plain radix stages in its row passes: +3 % end to end on C3
// against 2 waves at 216 VGPRs (measured A/B).  Cooperative builds keep 1; adaptive beta
// (the per-trial float32 K and beta derivative) takes 2: 141 spills at 3.
#ifndef BSGP_LS_ATTR
#define BSGP_LS_ATTR __attribute__((amdgpu_waves_per_eu(COOP ? 1 : ((K <= 2 && !ADAPT) ? 3 : 2))))
#endif
// line search: pass 1 also sums the second trial (lam = beta) directly.  On in
// the per-wave float64 builds (bsgp_persist.hip and bsgp_solver.hip's phase
// kernels, which must stay bitwise equal to it; A/B same box: C3 +0.5 %,
// 1.41 -> 1.21 passes per iteration, C5 -0.1 %); never in the cooperative
// kernels, whose k_ls spills with it (C4 -3.7 %).
#ifndef BSGP_LS1_K2
#define BSGP_LS1_K2 0
#endif
// closed-form line-search trials evaluated kLsLanes at a time, one per lane
// (ls_phase); 0 = one trial per step (the scalar loop, A/B)
#ifndef BSGP_LS_SERIES_LANES
#define BSGP_LS_SERIES_LANES 1
#endif
constexpr int kLsLanes = 32;
#ifndef BSGP_SERIES_BOUND
#define BSGP_SERIES_BOUND 1  // closed-form trials past lam*max|u| <= 0.01 under the tail bound
#endif
#ifndef BSGP_ACC_SERIES
#define BSGP_ACC_SERIES 0  // den^(b-1) by the series at series-step accepts: same speed on C3 (A/B), off
#endif
#ifndef BSGP_LSACC_JCH
#define BSGP_LSACC_JCH 1
#endif
#ifndef BSGP_LSACC_PF
#define BSGP_LSACC_PF true
#endif
// two operand batches in flight in the single-column row passes (row_inv2 /
// row_fwd2 PIPE): k_ls pass 1 and accept, k_bb
#ifndef BSGP_LS1_PIPE
#define BSGP_LS1_PIPE false
#endif
#ifndef BSGP_LSACC_PIPE
#define BSGP_LSACC_PIPE false
#endif
#ifndef BSGP_BB_PIPE
#define BSGP_BB_PIPE false
#endif
#ifndef BSGP_PROJ_U
#define BSGP_PROJ_U 4
#endif
#ifndef BSGP_DIR_JCH
#define BSGP_DIR_JCH 4
#endif
#ifndef BSGP_DIR_PF
#define BSGP_DIR_PF true
#endif
// composite radix-6/9 FFT stages per row pass (the column pass always uses them):
// fewer LDS round trips vs ~20 more live VGPRs
#ifndef BSGP_DIR_COMP
#define BSGP_DIR_COMP true
#endif
#ifndef BSGP_LS_COMP
#define BSGP_LS_COMP false
#endif
#ifndef BSGP_BB_COMP
#define BSGP_BB_COMP false
#endif
#ifndef BSGP_BB_PRE
#define BSGP_BB_PRE false
#endif
#ifndef BSGP_BB_JCH
#define BSGP_BB_JCH 1  // one column per operand batch: 117 VGPRs, 4 waves/SIMD (k_bb -17 %, A/B)
#endif

// (phase profile macros PH_T / PH_ADD: bsgp_device.hpp)
// ------------------------------------------------------------------ helpers
__device__ __forceinline__ double clipX(double x, double lo, double hi) {
  // X[X < lo] = lo; X[X > hi] = hi  (sgp.py:355-357)
  double X = (x < lo) ? lo : x;
  return (X > hi) ? hi : X;
}

__device__ __forceinline__ double realtime_s() {
  return (double)__builtin_amdgcn_s_memrealtime() * 1e-8;  // 100 MHz constant clock
}

// Streaming pass over pixel pairs [0, npair): every thread issues the loads of
// U pairs before computing any of them (memory-level parallelism for one
// workgroup streaming a whole image).  `ld(p)` loads, `cp(p, v)` computes.
template <int U, class LD, class CP>
__device__ __forceinline__ void stream_range(int p0, int p1, LD&& ld, CP&& cp) {
  using T = decltype(ld(0));
  for (int b = p0 + threadIdx.x; b < p1; b += kBlock * U) {
    T v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = ld(min(b + u * kBlock, p1 - 1));  // clamped, branch-free
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int p = b + u * kBlock;
      if (p < p1) cp(p, v[u]);
    }
  }
}
// T == 1: the whole image; T > 1: this member's row chunks (Part::cp pairs
// each), so a pass reads only pixels this member itself produced.
template <int U, class LD, class CP>
__device__ __forceinline__ void stream2(const Part& D, int npair, LD&& ld, CP&& cp) {
  if (D.T == 1) {
    stream_range<U>(0, npair, ld, cp);
    return;
  }
  for (int p0 = D.m * D.cp; p0 < npair; p0 += D.T * D.cp)
    stream_range<U>(p0, p0 + D.cp < npair ? p0 + D.cp : npair, ld, cp);
}

__device__ __forceinline__ double2 ld2(const double* a, int p) {
  return reinterpret_cast<const double2*>(a)[p];
}
// float32 storage (BSGP_STORAGE_F32): a pair of stored floats, widened
__device__ __forceinline__ double2 ld2(const float* a, int p) {
  const float2 f = reinterpret_cast<const float2*>(a)[p];
  return double2{(double)f.x, (double)f.y};
}

// Branch-free optional operands.  A load under a runtime condition compiles to
// a branch whose join waits for it (s_waitcnt vmcnt(0) before the phi copy),
// which serialises the loads of an operand batch.  Instead every lane loads:
// its own pixel when the wave-uniform flag is on, element 0 of the same slot
// vector (one cache line for the whole wave) when it is off; the value is
// selected after the load.  Every slot vector exists in every plan.
template <class T>
__device__ __forceinline__ double opt_ld(bool on, const T* a, int i, double off) {
  const double v = (double)a[on ? i : 0];
  return on ? v : off;
}
__device__ __forceinline__ double2 opt_ld2(bool on, const double* a, int p, double off) {
  const double2 v = ld2(a, on ? p : 0);
  return on ? v : double2{off, off};
}
// The observed-image operand in one 8-byte load for both layouts: compact
// (ImgState::g32, the raw float32 gnf[i] in the low word) or float64 gns[i].
// The compact array is the first half of the gns slot vector, so the word
// after gnf[i] is in bounds.
__device__ __forceinline__ double g_raw(bool g32, const double* gns, int i) {
  const unsigned int* w = reinterpret_cast<const unsigned int*>(gns) + (g32 ? i : 2 * i);
  unsigned long long u;
  __builtin_memcpy(&u, __builtin_assume_aligned(w, 4), 8);
  return __longlong_as_double((long long)u);
}
// Pixel pair p: compact = floats gnf[2p], gnf[2p+1] in the first 8 bytes
// (16 bytes are read either way; the wave's lines are the same).
__device__ __forceinline__ double2 g_raw2(bool g32, const double* gns, int p) {
  const double* a = g32 ? gns + p : gns + 2 * p;  // gnf + 2p == (double*)gns + p
  double2 v;
  __builtin_memcpy(&v, __builtin_assume_aligned(a, 8), 16);
  return v;
}

// Per-image slot vectors (x and g double-buffered; `par` picks the current
// iterate).  Slot = image: state persists across the phase kernels.  The
// observed image and the background map are float64 (gn may be kept compact,
// ImgState::g32); the seven iteration vectors are stored as V: double, or
// float for BSGP_STORAGE_F32 (every sum and scalar stays float64).
template <class V>
struct Bufs {
  double *gns, *bks;
  V *xa, *xb, *ga, *gb, *xtf, *dtf;
  V* pw;  // den^(beta-1) at the current x_tf (beta objective): reused by the
          // gradient (k_bb) and the next line search's series moments
  cd* spec;
};

template <class V>
__device__ __forceinline__ Bufs<V> slot_bufs(const SolveArgs& A, int img, int par) {
  Bufs<V> b;
  double* ws = A.ws + (size_t)img * A.slot_stride;
  const size_t v = A.vec_stride;
  b.gns = ws;
  b.bks = ws + v;
  V* vb = reinterpret_cast<V*>(ws + 2 * v);
  V* x0 = vb;
  V* x1 = vb + v;
  V* g0 = vb + 2 * v;
  V* g1 = vb + 3 * v;
  b.xa = par ? x1 : x0;
  b.xb = par ? x0 : x1;
  b.ga = par ? g1 : g0;
  b.gb = par ? g0 : g1;
  b.xtf = vb + 4 * v;
  b.dtf = vb + 5 * v;
  b.pw = vb + 6 * v;
  b.spec = reinterpret_cast<cd*>(ws + A.spec_off);
  return b;
}

// The search direction of sgp.py:311-318 for one pixel: y = x - alpha*X*g,
// projected (pflag 1: x(lambda_p) of projectDF(flux, y*D, D); pflag 0: y>=0).
struct Dir {
  bool Xones, proj;
  double alpha, lo, hi, lam_p;
  ProjClip clip;
  __device__ __forceinline__ void cd_of(double x, double g, double& c, double& dia) const {
    const double X = Xones ? 1.0 : clipX(x, lo, hi);
    const double D = 1 / X;
    const double y = x - alpha * (X * g);
    c = y * D;
    dia = D;
  }
  // y = x - alpha*X*g and X of one pixel (sgp.py:311-313)
  __device__ __forceinline__ void yx(double x, double g, double& y, double& X) const {
    X = Xones ? 1.0 : clipX(x, lo, hi);
    y = x - alpha * (X * g);
  }
  // x_i(lambda) of projectDF(flux, y*D, D) in multiplier form: (c + lam)/dia
  // = y + lam*X up to rounding, clipped to [0, sat] (flux_conserve_proj.py:22-25).
  // The sums of the multiplier search use this form; the projected pixels
  // themselves (d below) use the reference's division.
  __device__ __forceinline__ double pv(double y, double X, double lam) const {
    double v = fma(lam, X, y);
    v = (0.0 > v) ? 0.0 : v;
    if (clip.has_sat) v = (clip.satv < v) ? clip.satv : v;
    return v;
  }
  __device__ __forceinline__ double d(double x, double g) const {
    double y;
    if (proj) {
      double c, dia;
      cd_of(x, g, c, dia);
      y = clip(c, dia, lam_p);
    } else {
      const double X = Xones ? 1.0 : clipX(x, lo, hi);
      y = x - alpha * (X * g);
      if (y < 0) y = 0;
    }
    return y - x;
  }
};

__device__ __forceinline__ Dir make_dir(const SolveArgs& A, const ImgState& st) {
  Dir D;
  D.Xones = st.Xones != 0;
  D.proj = A.prm.proj_type == 1;
  D.alpha = st.alpha;
  D.lo = st.lo;
  D.hi = st.hi;
  D.lam_p = st.lam_p;
  D.clip = ProjClip{A.prm.has_sat != 0, A.prm.ccd_sat_level / st.sc - 2.220446049250313e-16};
  // float32 image, proj_type 0: the first scaling matrix is x.copy() of the
  // float32 start, clipped (compared and assigned) at float32 bounds
  // (sgp.py:279-285 / 723-729); from iteration 2 on x is float64
  if (A.prm.gn_f32 && A.prm.proj_type == 0 && st.iter == 1) {
    D.lo = (double)(float)st.lo;
    D.hi = (double)(float)st.hi;
  }
  return D;
}

__device__ __forceinline__ Objective make_obj(const SolveArgs& A, double beta) {
  Objective o;
  o.variant = A.prm.variant;
  o.f32g = A.prm.gn_f32 != 0;
  o.set_beta(beta);
  return o;
}

// Team of the workgroup: members blockIdx.x % T of image img0 + blockIdx.x / T.
__device__ __forceinline__ Team make_team(const SolveArgs& A, int img, const ImgState& st) {
  Team t;
  t.T = A.T;
  t.m = A.T == 1 ? 0 : (int)(blockIdx.x % (unsigned)A.T);
  t.part = A.tpart ? A.tpart + (size_t)img * kPartBufs * (A.T + 8) * kMaxRed : nullptr;
  t.flags = A.T <= 1 ? 0 : A.T <= BSGP_TEAM_FLAGS ? 1 : (BSGP_TEAM_HIER && A.T >= 8) ? 2 : 0;
  t.ctr = A.tctr ? A.tctr + (size_t)img * kTeamWords : nullptr;
  t.base = (unsigned int)st.bar_base;
  t.nb = 0;
  t.fail = A.tfail;
  // barrier groups: blockIdx % 8 (the XCD under round-robin dispatch)
  t.grp = (int)(blockIdx.x & 7u);
  const unsigned first = blockIdx.x - (unsigned)t.m;  // the team's first workgroup
  const int r = (int)(((unsigned)t.grp - (first & 7u)) & 7u);
  t.ng = t.T / 8 + (r < (t.T & 7) ? 1 : 0);
  t.G = t.T < 8 ? t.T : 8;
  return t;
}
__device__ __forceinline__ int team_img(const SolveArgs& A) {
  return A.img0 + (A.T == 1 ? (int)blockIdx.x : (int)(blockIdx.x / (unsigned)A.T));
}
// Member 0 records how many team barriers the image has completed, for the
// next kernel; all members read bar_base before their first arrival, member
// 0 writes it after its last one, so no member can see the new value early.
__device__ __forceinline__ void team_end(ImgState& st, const Team& t) {
  if (t.T > 1 && t.m == 0 && threadIdx.x == 0 && t.nb > 0)
    st.bar_base = (int)(t.base + (unsigned int)t.nb);
}
__device__ __forceinline__ bool leader(const Team& t) { return t.m == 0 && threadIdx.x == 0; }

#define BSGP_LDS_VIEWS(A)                                                           \
  extern __shared__ __attribute__((aligned(16))) char smem[];                      \
  cd* lds = reinterpret_cast<cd*>(smem + (A).g.tw2);                               \
  double* red = reinterpret_cast<double*>(smem + (A).g.tw2 + (A).lds_fft_bytes)

// numpy's float32 np.sum of term(i) for i < N, in numpy's exact order (the
// plan's PwProg, bsgp_api.hip pairwise_program): the leaves by the team's
// threads (each a numpy leaf: 8 strided float32 accumulators), the inner nodes
// level by level with a team barrier between levels, then the chunk fold
// res = res + root from 0.  `vals` is float scratch in HBM (leaves + nodes).
template <class TERM>
__device__ __forceinline__ float np_f32_sum(const PwProg& pw, TERM&& term, float* vals, const Part& D, Team& tm) {
  const int* lv = pw.prog;
  const int* nd = lv + 2 * pw.nleaf;
  const int* off = nd + 2 * pw.nnode;
  const int* roots = off + pw.nlev + 1;
  // A leaf's 8 accumulators on 8 neighbouring lanes: lane j of the leaf's lane
  // group sums terms j, j+8, ... in order, the group folds them as numpy does,
  // ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)), by xor-shuffles (a+b == b+a bit for
  // bit), and its lane 0 adds the n % 8 tail in order.  One lane per leaf ran
  // 8x longer chains (a 961-pixel stamp: 8 leaves of up to 128 float32 powers
  // on 8 lanes of the workgroup, at every trial of adaptive beta).
  const int q = D.gt0 + (int)threadIdx.x;
  const int j = q & 7;
  const int lstride = D.gts >> 3;
  const int nrounds = (pw.nleaf + lstride - 1) / lstride;  // the same in every lane
  for (int it = 0; it < nrounds; ++it) {
    const int l = (q >> 3) + it * lstride;
    const bool act = l < pw.nleaf;
    const int s0 = act ? lv[2 * l] : 0, n = act ? lv[2 * l + 1] : 0;
    float r = 0.0f;
    if (n >= 8) {
      const int m8 = n - (n % 8);
      r = term(s0 + j);
      for (int i = 8 + j; i < m8; i += 8) r += term(s0 + i);
    }
    float s = r + __shfl_xor(r, 1);
    s = s + __shfl_xor(s, 2);
    s = s + __shfl_xor(s, 4);
    if (act && j == 0) {
      float res;
      int i;
      if (n < 8) {
        res = 0.0f;
        i = 0;
      } else {
        res = s;
        i = n - (n % 8);
      }
      for (; i < n; ++i) res += term(s0 + i);
      vals[l] = res;
    }
  }
  team_sync(tm);
  for (int h = 0; h < pw.nlev; ++h) {
    for (int k = off[h] + D.gt0 + (int)threadIdx.x; k < off[h + 1]; k += D.gts)
      vals[pw.nleaf + k] = vals[nd[2 * k]] + vals[nd[2 * k + 1]];
    team_sync(tm);
  }
  float res = 0.0f;
  for (int c = 0; c < pw.nchunk; ++c) res = res + vals[roots[c]];
  return res;
}

// Per-image counters of a finished solve (include/bsgp.h bsgp_outputs.counters),
// written by the image's leader when it stops.
__device__ __forceinline__ void write_counters(const SolveArgs& A, const ImgState& st, int img,
                                               int T) {
  if (!A.out.counters) return;
  int64_t* c = A.out.counters + (size_t)img * 8;
  c[0] = st.E_p;
  c[1] = st.E_ls;
  c[2] = st.ls_passes;
  c[3] = st.status |
         ((A.tfail && __hip_atomic_load(A.tfail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) ? 4
                                                                                              : 0);
  c[4] = st.ls_series;
  c[5] = T;
  c[6] = st.proj_passes;
  c[7] = st.proj_list;
}

// An image stopped: count it down; the one that takes the count to 0 tells
// the host (a system-scope vector store to host-mapped memory, read after an
// event the host waits on), so the host need not drain the stream to learn
// that every image has stopped.
__device__ __forceinline__ void count_stopped(const SolveArgs& A) {
  if (atomicSub(A.active, 1) == 1 && A.done_host)
    __hip_atomic_store(A.done_host, A.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// ------------------------------------------------------------ kernel: setup
// sgp.py:163-298 (= 617-742): scaling, null pixels, flux, x0, initial
// projection, x_tf = A(x), f, g and the scaling-matrix bounds.
// Waves per SIMD the setup kernel is compiled for (per-wave plans; 0: the
// compiler's choice).  Setup runs once per solve, one workgroup per image:
// at four workgroups per CU C3's 1024 images are one round instead of two.
#ifndef BSGP_SETUP_WAVES
#define BSGP_SETUP_WAVES 0
#endif
#if BSGP_SETUP_WAVES
#define BSGP_SETUP_ATTR __attribute__((amdgpu_waves_per_eu(COOP ? 1 : BSGP_SETUP_WAVES)))
#else
#define BSGP_SETUP_ATTR
#endif
// One image's setup (k_setup below, or the persistent solver's first task of
// the image, SolveArgs::fold_setup); the caller has loaded the twiddles into LDS.
template <bool COOP, class V>
__device__ __forceinline__ void setup_phase(const SolveArgs& A, int img) {
  BSGP_LDS_VIEWS(A);
  const Geo& G = A.g;
  const bsgp_params& P = A.prm;
  const int N = G.H * G.W;
  const int tid = threadIdx.x;
  const bool bmap = P.bkg_is_map != 0;
  const bool odd = (N & 1) != 0;
  Bufs<V> B = slot_bufs<V>(A, img, 0);
  ImgState& st = A.st[img];
  // counters are zeroed per solve: the setup kernel starts the count at 0
  Team tm = make_team(A, img, st);
  tm.base = 0;
  const Part D = make_part(tm, G.nfw, G.W);
  const double* gn_in = A.in.gn + (size_t)img * N;
  const double* bk_in = bmap ? A.in.bkg + (size_t)img * N : nullptr;
  const double bk_scalar_raw = bmap ? 0.0 : A.in.bkg[img];
  const double t0 = realtime_s();

  // raw statistics (sgp.py:174-177, 190, 193-194)
  double v2[3] = {0.0, 0.0, 0.0};  // sum(gn - bkg), sum(gn), #values not exact in f32
  double mx = -INFINITY;
  for (int i = D.gt0 + tid; i < N; i += D.gts) {
    const double g = gn_in[i];
    const double bkr = bmap ? bk_in[i] : bk_scalar_raw;
    v2[0] += g - bkr;
    v2[1] += g;
    mx = (g > mx || g != g) ? g : mx;
    if (!(isfinite(g) && (double)(float)g == g)) v2[2] += 1.0;  // params.gn_compact
  }
  team_sum_max<3>(v2, mx, red, tm);  // one team barrier
  const bool ok32 = v2[2] == 0.0;     // every raw value finite and exact in f32
  // float32 image, prelude on the device (include/bsgp.h, ABI 3): numpy 1.x
  // keeps gn / scaling and x / scaling in float32 (sgp.py:648-652)
  const bool pre32 = P.gn_f32 && P.scale_data != 2;
  const double sc = P.scale_data == 2 ? P.prescaled_scaling : (P.scale_data ? mx : 1.0);
  const float sc32 = (float)sc;  // exact: max of float32 values
  const double fl_raw = A.in.flux ? A.in.flux[img] : v2[0];
  // np.sum(gn-bkg)/gn.size*ones (sgp.py:175); a float32 image keeps the float32 array
  const double x3 = pre32 ? (double)(float)(fl_raw / (double)N) : (fl_raw / (double)N) * 1.0;
  double tol4 = P.scale_data == 2 ? P.prescaled_tol4 : 1 + 1 / (v2[1] / (double)N);
  if (pre32 && P.stop_criterion == 4) {
    // 1 + 1/np.mean(gn) of the raw float32 image (sgp.py:644): numpy's float32
    // pairwise sum, the mean rounded to float32, the rest in float64
    const float s32 = np_f32_sum(
        A.pw, [&](int i) { return (float)gn_in[i]; }, reinterpret_cast<float*>(B.dtf), D, tm);
    tol4 = 1 + 1 / (double)(float)((double)s32 / (double)N);
  }
  const bool divide = P.scale_data == 1;
  const double bks_scalar = P.scale_data == 2 ? bk_scalar_raw : (divide ? bk_scalar_raw / sc
                                                                        : bk_scalar_raw);
  // gn (and an init_recon 2 start) / scaling: float64, or float32 for a float32 image
  auto scale_px = [&](double g) {
    if (pre32) return divide ? (double)((float)g / sc32) : g;
    return divide ? g / sc : g;
  };
  // scale + null-pixel minimum (sgp.py:193-204)
  double vmin = INFINITY;
  for (int i = D.gt0 + tid; i < N; i += D.gts) {
    const double g = scale_px(gn_in[i]);
    B.gns[i] = g;
    if (g > 0 && g < vmin) vmin = g;
    if (bmap) B.bks[i] = divide ? bk_in[i] / sc : bk_in[i];
  }
  vmin = team_min(vmin, red, tm);
  const double eps = 2.220446049250313e-16;
  // the fill is stored into the float32 array for a float32 image (sgp.py:659)
  const double fill = pre32 ? (double)(float)(vmin * eps * eps) : vmin * eps * eps;
  double v1[1] = {0.0};
  for (int i = D.gt0 + tid; i < N; i += D.gts) {
    double g = B.gns[i];
    if (g <= 0) {
      g = fill;
      B.gns[i] = g;
    }
    v1[0] += g - (bmap ? B.bks[i] : bks_scalar);
    // initial x (sgp.py:166-177, 197), then the pflag==0 clamp (:248-249)
    double x;
    if (A.in.x0) {
      x = A.in.x0[(size_t)img * N + i];  // float64 (randn): x / scaling stays float64
      if (divide) x = x / sc;
    } else if (P.init_recon == 0) {
      x = 0.0;
    } else if (P.init_recon == 2) {
      x = scale_px(gn_in[i]);  // gn.copy() / scaling, before the null-pixel fix
    } else {
      x = scale_px(x3);
    }
    if (P.proj_type == 0 && x < 0) x = 0;
    B.xa[i] = x;
  }
  if (odd && leader(tm)) {  // benign pad element of the pair-vectorised streams
    B.gns[N] = 1.0;
    if (bmap) B.bks[N] = 0.0;
    B.xa[N] = B.xb[N] = B.ga[N] = B.gb[N] = B.xtf[N] = B.dtf[N] = 0.0;
  }
  team_sum<1>(v1, red, tm);
  // sgp.py:208-211 (scale_data 2: the caller scaled the flux in its own dtype)
  // (a numpy float32 flux over the float32 scaling divides in float32)
  const double flux =
      A.in.flux ? (P.scale_data == 2 ? A.in.flux[img]
                   : (pre32 && P.flux_f32 && divide) ? (double)((float)A.in.flux[img] / sc32)
                                                     : A.in.flux[img] / sc)
                : v1[0];
  const ProjClip clip{P.has_sat != 0, P.ccd_sat_level / sc - eps};

  // initial projection with dia = 1 (sgp.py:250-253); every thread clips the
  // pixels it wrote, so only the rows pass below needs the team barrier
  if (P.proj_type == 1) {
    auto psum = [&](double lam) {
      double s1[1] = {0.0};
      for (int i = D.gt0 + tid; i < N; i += D.gts) s1[0] += clip(B.xa[i], 1.0, lam);
      team_sum<1>(s1, red, tm);
      return s1[0];
    };
    ProjOut po = project_df_fn(psum, flux, 0.0, 1.0, 1e-11, 0, 0, P.max_projs);
    for (int i = D.gt0 + tid; i < N; i += D.gts) B.xa[i] = clip(B.xa[i], 1.0, po.lam);
  }
  team_sync(tm);  // x0 / gns / bks complete before the row passes
  // x_tf = A(x), f and g (sgp.py:260-265 / 702-709)
  const double beta0 = A.in.beta0 ? A.in.beta0[img] : P.betaParam;
  Objective obj = make_obj(A, beta0);
  // float32 image: the lambda-independent sum np.sum(s*gn**beta) is a float32
  // array reduced by numpy in float32 (sgp.py:458); its order is the plan's
  // pairwise program.  The dtf vector is free scratch until the first k_ls.
  const bool konst_f32 = P.gn_f32 && P.variant == BSGP_VARIANT_BETA && obj.mode == 3;
  double konst32 = 0.0;
  if (konst_f32) {
    const float sf = (float)obj.scal;
    const float bf = (float)obj.beta;  // x**beta: the exponent is cast to float32
    konst32 = (double)np_f32_sum(
        A.pw, [&](int i) { return sf * libm_powf((float)B.gns[i], bf); },
        reinterpret_cast<float*>(B.dtf), D, tm);
  }
  double fsum[3] = {0.0, 0.0, 0.0};  // K, T0, T1
  row_fwd<COOP>(G, D, G.H, G.W, G.sld, B.spec, lds, [&](int r, int j) { return B.xa[r * G.W + j]; });
  team_sync(tm);
  col_conv<COOP>(G, D, B.spec, tf_of(G, img, 0), lds);
  team_sync(tm);
  const bool beta_obj = P.variant == BSGP_VARIANT_BETA;
  row_inv_fwd<COOP>(G, D, B.spec, lds, [&](int r, int j, double v) {
    const int i = r * G.W + j;
    B.xtf[i] = v;
    const double den = v + (bmap ? B.bks[i] : bks_scalar);
    const double g = B.gns[i];
    fsum[0] += obj.konst(g);
    obj.terms(v, den, g, &fsum[1]);
    if (!beta_obj) return g / den;  // KL: w = gn/den (sgp.py:262)
    const double p = fpow(den, obj.beta - 1);
    B.pw[i] = p;
    return g * (p / den);  // gn*den^(b-2) (sgp.py:499)
  });
  team_sum<3>(fsum, red, tm);
  team_sync(tm);  // publishes xtf / spec / pw
  if (konst_f32) fsum[0] = konst32;
  const double fv = obj.combine(fsum[0], fsum[1], fsum[2], flux, (double)N);
  col_conv<COOP>(G, D, B.spec, tf_of(G, img, 1), lds);
  team_sync(tm);
  row_inv<COOP>(G, D, B.spec, lds, [&](int r, int j, double at) {
    const int i = r * G.W + j;
    B.ga[i] = (beta_obj ? B.pw[i] : 1.0) - at;  // sgp.py:263 / 499
  });
  team_sync(tm);  // every row of spec read before it is overwritten
  // scaling-matrix bounds from AT(gn) (sgp.py:268-273)
  row_fwd<COOP>(G, D, G.H, G.W, G.sld, B.spec, lds, [&](int r, int j) { return B.gns[r * G.W + j]; });
  team_sync(tm);
  col_conv<COOP>(G, D, B.spec, tf_of(G, img, 1), lds);
  team_sync(tm);
  double ymin = INFINITY, ymax = -INFINITY;
  row_inv<COOP>(G, D, B.spec, lds, [&](int r, int j, double at) {
    const int i = r * G.W + j;
    const double bkv = bmap ? B.bks[i] : bks_scalar;
    const double y = (flux / (flux + bkv)) * at;
    if (y > 0 && y < ymin) ymin = y;
    ymax = (y > ymax || y != y) ? y : ymax;
  });
  {
    // max(y) and min(y[y > 0]) = -max(-y) in one team barrier
    double none[1] = {0.0};
    double m2[2] = {ymax, -ymin};
    team_reduce<0, 2>(none, m2, red, tm);
    ymax = m2[0];
    ymin = -m2[1];
  }
  double lo = ymin, hi = ymax;
  if (hi / lo < 50) {
    lo = lo / 10;
    hi = hi * 10;
  }
  // Compact observed image: the raw f32-exact values replace gn_s in the first
  // half of its slot vector (every f64 read of gn_s is done: team_sync above).
  // Readers recompute gn_s = raw / sc (or raw), and the null-pixel fill for
  // raw <= 0, with the operations used above: the same bits as f64 storage.
  // A float32 image's scaled values are float32 themselves: kept as they are
  // (mode 1), with the fill for values <= 0 on read.
  const int g32 = (P.gn_compact && ok32) ? ((divide && !pre32) ? (sc > 0 ? 2 : 0) : 1) : 0;
  if (g32) {
    float* gf = reinterpret_cast<float*>(B.gns);
    for (int i = D.gt0 + tid; i < N; i += D.gts)
      gf[i] = (float)(g32 == 2 ? gn_in[i] : scale_px(gn_in[i]));  // mode 2 divides on read
    if (odd && leader(tm)) gf[N] = 1.0f;  // pad element of the pair-vectorised streams
  }
  const double Dcoeff = 2 / (double)N * sc;
  double tol = P.tol_convergence;
  if (P.stop_criterion == 4) tol = tol4;
  if (P.verbose && P.stop_criterion == 2) tol = tol * tol;
  if (leader(tm)) {
    const int M1 = P.MAXIT + 1;
    A.out.discr[(size_t)img * M1] = Dcoeff * fv;
    if (A.out.times) A.out.times[(size_t)img * M1] = 0.0;
    if (A.out.crit) A.out.crit[(size_t)img * M1] = 0.0;
    if (A.out.flags) A.out.flags[(size_t)img * M1] = 0;
    for (int k = 0; k < P.M_alpha; ++k) st.Valpha[k] = P.alpha_max;
    for (int k = 0; k < P.M; ++k) st.Fold[k] = -1e30;
    st.par = 0;
    st.Xones = P.init_recon == 0;  // X = ones until the first BB update (sgp.py:279-280)
    st.stop = 0;
    st.iter = 1;
    st.epoch = 0;
    st.bar_base = tm.nb;
    st.E_p = st.E_ls = st.ls_passes = st.status = st.ls_series = 0;
    st.proj_passes = st.proj_list = 0;
    st.lam_p = 0.0;  // no previous multiplier: the first projection splits no bracket
    st.lam_ratio = 0.0;
    st.kappa = 0.0;
    st.sc = sc;
    st.flux = flux;
    st.bks_scalar = bks_scalar;
    st.lo = lo;
    st.hi = hi;
    st.Dcoeff = Dcoeff;
    st.tol = tol;
    st.t0 = t0;
    st.fv = fv;
    st.alpha = P.alpha;
    st.tau = P.tau;
    st.lr = P.lr;
    st.init_lr = P.lr;
    st.beta = beta0;
    st.konst = fsum[0];
    st.g32 = g32;
    st.gfill = fill;
    if (!(ymin < INFINITY)) {
      // no positive entry in y = flux/(flux+bkg)*AT(gn): the reference's
      // np.min(y[y > 0]) raises before the first iteration (sgp.py:269-270,
      // 711-712); the image stops here with status bit 8
      st.status = 8;
      st.stop = 1;
      A.out.iters[img] = 0;
      if (A.out.beta_final) A.out.beta_final[img] = st.beta;
      write_counters(A, st, img, tm.T);
      count_stopped(A);
    }
  }
}

template <bool COOP, class V>
__global__ void __launch_bounds__(kBlock) BSGP_SETUP_ATTR k_setup(SolveArgs A) {
  load_tw_lds(A.g);
  setup_phase<COOP, V>(A, team_img(A));
}

// --------------------------------------- projection with pixel lists
// projectDF(flux, y*D, D) (flux_conserve_proj.py:7-144) for the direction of
// sgp.py:311-318: the reference's multiplier sequence, step for step
// (project_df_fn).  What changes is how sum_i x_i(lambda) is evaluated:
//  * the first evaluation (lambda_ = 0) is a full pass over (x, g) that also
//    sums x(lambda_ - dlambda_) and x(lambda_ + dlambda_), the second
//    evaluation of either bracketing branch (:32 / :57), and the slope at
//    lambda_ (for a Newton bound on the root);
//  * a full pass can split the pixels for a bracket [qL, qU]: pixels at 0 or
//    at saturation for every lambda in it add a constant, pixels strictly
//    inside add y + lambda*X (two running sums), and only the pixels that
//    change state inside the bracket go to this thread's list (y, X);
//  * an evaluation whose lambda lies in the split bracket reads only the list
//    (typically 2-5% of the pixels, written and read back by the same thread).
// Split brackets: the previous iteration's multiplier +/- 30% on the first
// pass; on the first miss, the hull of the missing lambda and the Newton
// bound (for the convex sum the secant and Newton iterates fall on either
// side of the root); on later misses, the tightest bracket of signs seen.
// A miss is just a full pass, so the choice of bracket never changes results.
#ifndef BSGP_PROJ_GUESS_W
#define BSGP_PROJ_GUESS_W 0.3
#endif
constexpr double kProjGuessW = BSGP_PROJ_GUESS_W;
// Round 6: the first pass's bracket from the search's own history.  The root
// moves with the step length alpha of y = x - alpha X g (without clipping,
// sum x = flux makes lambda = alpha sum(X g) / sum X): C3's stagnating
// iterations alternate alpha ~3.2 / ~34 (Barzilai-Borwein), and the root
// with it, which is what made the +/-30 % guess around the previous root
// miss.  The prediction is alpha * (previous root / previous alpha), +/- W1;
// the bracket also covers the search's first secant point, kappa times the
// root (kappa from the previous search: ~1.9 on C3), +/- W2, which lies
// outside any bracket around the root.  Offline replay of the reference's
// multiplier sequences (oracle) through these rules: full passes + list
// reads per projection 1.97 -> 1.33 pass-equivalents on C3's images 0-1,
// 2.39 -> 1.80 on C4.  A miss is still just a full pass: results unchanged.
#ifndef BSGP_PROJ_ALPHA
#define BSGP_PROJ_ALPHA 1
#endif
#ifndef BSGP_PROJ_W1
#define BSGP_PROJ_W1 0.1
#endif
#ifndef BSGP_PROJ_W2
#define BSGP_PROJ_W2 0.2
#endif
// Teams with few pixels per thread (C2: 8) split the first pass for
// [lambda_ - dlambda_, lambda_ + dlambda_] instead: the reference's bracketing
// phase stops there whenever r(0) and r(-/+1) differ in sign (every iteration
// of the C2 workload, oracle trace), and its secant phase never leaves its
// bracket, so no evaluation misses; the wider list costs a few entries per
// thread where each evaluation is one team reduction either way.  (The root
// moves 2-25x between iterations there, so the +/-30 % guess missed on most.)
#ifndef BSGP_PROJ_WIDE_PX
#define BSGP_PROJ_WIDE_PX 16
#endif

// Teams keep the first SolveArgs::list_lds entries of every thread's list in
// the transform buffers' LDS, which the row pass after the projection is the
// next to use (C2 and the application's subdivisions: the whole list, so an
// evaluation reads no global memory; C4: 16 of up to 32 entries), the rest
// in global memory (LL: compiled in; the persistent one-workgroup solver
// keeps global lists).
template <class V, bool LL>
__device__ __forceinline__ ProjOut cached_projection(const SolveArgs& A, int img, const Part& Pt, Team& tm,
                                     const Dir& D, const Bufs<V>& B, double* red, cd* lds,
                                     double lam_prev, double flux, int npair, bool odd, int N,
                                     int64_t& passes, int64_t& list_reads, double lam_ratio,
                                     double kappa, double& first_lam) {
  const V* xa = B.xa;
  const V* ga = B.ga;
  const int LS = tm.T * kBlock;
  const int gt = tm.m * kBlock + (int)threadIdx.x;
  double* ly = A.plist + (size_t)img * A.plist_stride;
  double* lX = ly + A.plist_stride / 2;
  const int lcap = A.lcap;
  const int nl = LL ? A.list_lds : 0;  // entries per thread in LDS
  double* const qy = reinterpret_cast<double*>(lds);
  double* const qX = qy + (size_t)nl * kBlock;
  const int tl = (int)threadIdx.x;
  const bool hs = D.clip.has_sat;
  const double satv = D.clip.satv;
  // identical in every thread of the team
  bool have = false;
  double cL = 0.0, cU = 0.0, SA = 0.0, SB = 0.0, nsat = 0.0, nstr = 0.0;
  double Lk = -INFINITY, Uk = INFINITY;  // largest lambda with r < 0, smallest with r > 0
  double xl0 = NAN, xs0 = 0.0, xl1 = NAN, xs1 = 0.0, lamN = NAN;
  bool first_miss = true;
  int calls = 0;
  int cnt = 0;  // this thread's list entries

  auto note = [&](double lam, double S) {
    const double r = S - flux;
    if (r < 0 && lam > Lk) Lk = lam;
    if (r > 0 && lam < Uk) Uk = lam;
  };
  // One full pass: sums at lams[0..NL), optional split for [qL, qU]; returns
  // the slope sum_{0 < x_i(lams[0]) < sat} X_i.
  auto pass = [&](auto nlc, const double* lams, double* S, bool split, double qL,
                  double qU) -> double {
    constexpr int NL = decltype(nlc)::value;
    constexpr int NT = NL + 6;  // sums | SA, SB, n_sat, n_list, n_overflow | slope
    PH_T(tp0);
    double t[NT];
#pragma unroll
    for (int k = 0; k < NT; ++k) t[k] = 0.0;
    double lm[NL];
#pragma unroll
    for (int k = 0; k < NL; ++k) lm[k] = lams[k];
    if (split) cnt = 0;
    auto px = [&](double x, double g) __attribute__((always_inline)) {
      double y, X;
      D.yx(x, g, y, X);
#pragma unroll
      for (int k = 0; k < NL; ++k) {
        const double v = D.pv(y, X, lm[k]);
        t[k] += v;
        if (k == 0 && v > 0.0 && (!hs || v < satv)) t[NL + 5] += X;
      }
      if (split) {
        const double vL = D.pv(y, X, qL), vU = D.pv(y, X, qU);
        if (vU == 0.0) {
          // 0 for every lambda <= qU
        } else if (hs && vL == satv) {
          t[NL + 2] += 1.0;  // saturated for every lambda >= qL
        } else if (vL > 0.0 && (!hs || vU < satv)) {
          t[NL] += y;  // unclipped over the whole bracket
          t[NL + 1] += X;
        } else if (cnt < lcap) {
          if (cnt < nl) {
            qy[cnt * kBlock + tl] = y;
            qX[cnt * kBlock + tl] = X;
          } else {
            ly[(size_t)cnt * LS + gt] = y;
            lX[(size_t)cnt * LS + gt] = X;
          }
          ++cnt;
          t[NL + 3] += 1.0;
        } else {
          t[NL + 4] += 1.0;
        }
      }
    };
    stream2<BSGP_PROJ_U>(
        Pt, npair,
        [&](int p) {
          struct Ld {
            double2 x, g;
          } v;
          v.x = ld2(xa, p);
          v.g = ld2(ga, p);
          return v;
        },
        [&](int p, const auto& v) {
          px(v.x.x, v.g.x);
          if (!odd || 2 * p + 1 < N) px(v.x.y, v.g.y);
        });
    // the list is read back by the thread that wrote it: drain its stores
    if (split) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    team_sum<NT>(t, red, tm);
#pragma unroll
    for (int k = 0; k < NL; ++k) S[k] = t[k];
    if (split) {
      have = t[NL + 4] == 0.0;
      cL = qL;
      cU = qU;
      SA = t[NL];
      SB = t[NL + 1];
      nsat = t[NL + 2];
      nstr = t[NL + 3];
    }
    ++passes;
    PH_ADD(NL == 3 ? 10 : 12, tp0);
    return t[NL + 5];
  };
  // sum over the split bracket's list
  auto leval = [&](double lam) {
    PH_T(tl0);
    double t[1] = {0.0};
    int k = 0;
    if (nl > 0) {
      const int kl = cnt < nl ? cnt : nl;
      for (; k < kl; ++k) t[0] += D.pv(qy[k * kBlock + tl], qX[k * kBlock + tl], lam);
    }
    for (; k + 4 <= cnt; k += 4) {
      double yv[4], Xv[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        yv[u] = ly[(size_t)(k + u) * LS + gt];
        Xv[u] = lX[(size_t)(k + u) * LS + gt];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) t[0] += D.pv(yv[u], Xv[u], lam);
    }
    for (; k < cnt; ++k) t[0] += D.pv(ly[(size_t)k * LS + gt], lX[(size_t)k * LS + gt], lam);
    team_sum<1>(t, red, tm);
    PH_ADD(11, tl0);
    const double lin = SA + lam * SB;
    return (hs ? lin + nsat * satv : lin) + t[0];
  };
  auto sumf = [&](double lam) {
    double S;
    if (calls == 0) {
      const double lams[3] = {lam, lam - 1.0, lam + 1.0};  // lambda_ -/+ dlambda_ (dlambda_ = 1)
      double Sv[3];
      const bool wide = tm.T > 1 && (long)N <= (long)BSGP_PROJ_WIDE_PX * LS;
      bool guess = wide || (isfinite(lam_prev) && lam_prev != 0.0);
      const double w = kProjGuessW * fabs(lam_prev);
      double gL = wide ? lams[1] : lam_prev - w, gU = wide ? lams[2] : lam_prev + w;
      const double lh = D.alpha * lam_ratio;
      if (BSGP_PROJ_ALPHA && !wide && isfinite(lh) && lh != 0.0) {
        gL = lh - BSGP_PROJ_W1 * fabs(lh);
        gU = lh + BSGP_PROJ_W1 * fabs(lh);
        const double pk = kappa * lh;
        if (isfinite(pk) && pk != 0.0) {
          gL = fmin(gL, pk - BSGP_PROJ_W2 * fabs(pk));
          gU = fmax(gU, pk + BSGP_PROJ_W2 * fabs(pk));
        }
        guess = true;
      }
      const double slope = pass(std::integral_constant<int, 3>{}, lams, Sv, guess, gL, gU);
      S = Sv[0];
      xl0 = lams[1];
      xs0 = Sv[1];
      xl1 = lams[2];
      xs1 = Sv[2];
      note(lams[1], Sv[1]);
      note(lams[2], Sv[2]);
      lamN = slope > 0.0 ? lam - (S - flux) / slope : NAN;
    } else if (lam == xl0) {
      S = xs0;
    } else if (lam == xl1) {
      S = xs1;
    } else {
      // the first multiplier off the first pass (the first secant or bracket
      // step), recorded for the next search's bracket
      if (!isfinite(first_lam)) first_lam = lam;
      if (have && lam >= cL && lam <= cU) {
        S = leval(lam);
        list_reads += (int64_t)nstr;
      } else {
        bool split = false;
        double qL = 0.0, qU = 0.0;
        if (first_miss && isfinite(lamN)) {
          qL = fmin(lam, lamN);
          qU = fmax(lam, lamN);
          split = true;
        } else if (isfinite(Lk) && isfinite(Uk)) {
          qL = fmin(Lk, Uk);
          qU = fmax(Lk, Uk);
          split = true;
        }
        first_miss = false;
        const double lams[1] = {lam};
        double Sv[1];
        (void)pass(std::integral_constant<int, 1>{}, lams, Sv, split, qL, qU);
        S = Sv[0];
      }
    }
    ++calls;
    note(lam, S);
    return S;
  };
  return project_df_fn(sumf, flux, 0.0, 1.0, 1e-11, 0, 0, A.prm.max_projs);
}

// ------------------------------------------ kernel: direction + rows of d
// sgp.py:306-325: memory shifts, y = x - alpha*X*g, projectDF(flux, y*D, D)
// with every x(lambda) evaluation one streaming pass over (x, g), d = y - x,
// d.g, and the row transforms of d.
// One image's phase (the kernel below, or the persistent solver's task): the
// caller has checked st.stop and loaded the twiddles into LDS.
template <bool COOP, class V, bool LL = true>
__device__ __forceinline__ void dir_phase(const SolveArgs& A, int img) {
  BSGP_LDS_VIEWS(A);
  ImgState& st = A.st[img];
  PH_T(tk0);
  Team tm = make_team(A, img, st);
  const Geo& G = A.g;
  const Part Pt = make_part(tm, G.nfw, G.W);
  const bsgp_params& P = A.prm;
  const int N = G.H * G.W;
  const int npair = (N + 1) / 2;
  const bool odd = (N & 1) != 0;
  Bufs<V> B = slot_bufs<V>(A, img, st.par);
  Dir D = make_dir(A, st);
  const double flux = st.flux;
  int evals = 0;
  int64_t ppass = 0, plist_reads = 0;
  double lam_ratio = 0.0, kappa = 0.0;
  if (P.proj_type == 1 && A.plist != nullptr) {
    double first_lam = NAN;  // the search's first multiplier off the first pass
    ProjOut po = cached_projection<V, LL>(A, img, Pt, tm, D, B, red, lds, st.lam_p, flux, npair,
                                          odd, N, ppass, plist_reads, st.lam_ratio, st.kappa,
                                          first_lam);
    D.lam_p = po.lam;
    evals = po.evals;
    lam_ratio = D.alpha != 0.0 ? po.lam / D.alpha : 0.0;
    kappa = (isfinite(first_lam) && po.lam != 0.0) ? first_lam / po.lam : 0.0;
  } else if (P.proj_type == 1) {
    const V* xa = B.xa;
    const V* ga = B.ga;
    auto psum = [&](double lam) {
      double s[1] = {0.0};
      stream2<4>(
          Pt, npair,
          [&](int p) {
            struct Ld {
              double2 x, g;
            } v;
            v.x = ld2(xa, p);
            v.g = ld2(ga, p);
            return v;
          },
          [&](int p, const auto& v) {
            double c, d;
            D.cd_of(v.x.x, v.g.x, c, d);
            s[0] += D.clip(c, d, lam);
            if (!odd || 2 * p + 1 < N) {
              D.cd_of(v.x.y, v.g.y, c, d);
              s[0] += D.clip(c, d, lam);
            }
          });
      team_sum<1>(s, red, tm);
      return s[0];
    };
    ProjOut po = project_df_fn(psum, flux, 0.0, 1.0, 1e-11, 0, 0, P.max_projs);
    D.lam_p = po.lam;
    evals = po.evals;
    ppass = po.evals;
  }
  PH_ADD(0, tk0);
  PH_T(tk1);
  double gd[1] = {0.0};
  row_fwd2<BSGP_DIR_JCH, BSGP_DIR_PF, BSGP_DIR_COMP, COOP, false, 22>(
      G, Pt, G.H, G.W, G.sld, B.spec, lds,
      [&](int r, int j) {
        const int i = r * G.W + j;
        return double2{B.xa[i], B.ga[i]};
      },
      [&](int, int, const double2& v) {
        const double d = D.d(v.x, v.y);
        gd[0] += d * v.y;
        return d;
      });
  team_sum<1>(gd, red, tm);
  PH_ADD(1, tk1);
  if ((BSGP_FUSE_COL_CODE & 1) && (A.fuse_col & 1)) {  // A's column pass follows here
    PH_T(tc0);
    team_sync(tm);
    col_conv<COOP>(G, Pt, B.spec, tf_of(G, img, 0), lds);
    PH_ADD(3, tc0);
  }
  PH_ADD(2, tk0);
  team_end(st, tm);
  if (leader(tm)) {  // sgp.py:306-308 (memory shifts) + direction scalars
    for (int k = 0; k < P.M_alpha - 1; ++k) st.Valpha[k] = st.Valpha[k + 1];
    for (int k = 0; k < P.M - 1; ++k) st.Fold[k] = st.Fold[k + 1];
    st.Fold[P.M - 1] = st.fv;
    st.epoch += 1;
    st.lam_p = D.lam_p;
    st.lam_ratio = isfinite(lam_ratio) ? lam_ratio : 0.0;
    st.kappa = isfinite(kappa) ? kappa : 0.0;
    st.E_p += evals;
    st.proj_passes += ppass;
    st.proj_list += plist_reads;
    st.gd = gd[0];
  }
}

template <bool COOP, class V>
__global__ void __launch_bounds__(kBlock) BSGP_DIR_ATTR k_dir(SolveArgs A) {
  const int img = team_img(A);
  if (A.st[img].stop) return;
  load_tw_lds(A.g);
  dir_phase<COOP, V>(A, img);
}

// ----------------------------------------------------------- kernel: columns
template <bool COOP>
__global__ void __launch_bounds__(kBlock) BSGP_COL_ATTR k_col(SolveArgs A, int transpose) {
  BSGP_LDS_VIEWS(A);
  // A.Tc workgroups per image (>= the team size T): columns only, no barrier
  const int img = A.img0 + (A.Tc == 1 ? (int)blockIdx.x : (int)(blockIdx.x / (unsigned)A.Tc));
  const ImgState& st = A.st[img];
  if (st.stop) return;
  PH_T(tc0);
  Team tm{};
  tm.T = A.Tc;
  tm.m = A.Tc == 1 ? 0 : (int)(blockIdx.x % (unsigned)A.Tc);
  const Bufs<double> B = slot_bufs<double>(A, img, 0);  // spec only (same offset for V)
  load_tw_lds(A.g);
  col_conv<COOP>(A.g, make_part(tm, A.g.nfc, A.g.W), B.spec, tf_of(A.g, img, transpose), lds);
  PH_ADD(3, tc0);
}

// ------------------------------- kernel: line search + accept + rows of w
// sgp.py:326-349 / 774-801: K trial lambdas per pass over (x_tf, d_tf, gn);
// the first pass is fused into the inverse row transforms that produce d_tf.
// Then x_tf += lam*d_tf and the row transforms of AT's input w.
template <int K, int MODE, bool ADAPT, bool COOP, class V, bool SB = false>
__device__ __forceinline__ void ls_phase(const SolveArgs& A, int img) {
  // first pass (fused into the inverse rows of A(d)): one trial lambda = 1,
  // which is where most non-stagnating iterations accept; later passes
  // stream K trial lambdas each.
  BSGP_LDS_VIEWS(A);
  ImgState& st = A.st[img];
  PH_T(tk0);
  Team tm = make_team(A, img, st);
  const Geo& G = A.g;
  const Part Pt = make_part(tm, G.nfw, G.W);
  const bsgp_params& P = A.prm;
  const int N = G.H * G.W;
  const int npair = (N + 1) / 2;
  const bool odd = (N & 1) != 0;
  // SB: a scalar background known at compile time (the persistent solver's
  // build for the timed workload): no per-pixel background operand at all,
  // not even the branch-free stand-in load of opt_ld
  const bool bmap = SB ? false : P.bkg_is_map != 0;
  const double lr_st = st.lr;
  constexpr bool adapt = ADAPT;  // adaptive beta (sgp.py:798-800): K == 1, runtime mode
  Bufs<V> B = slot_bufs<V>(A, img, st.par);
  if ((BSGP_FUSE_COL_CODE & 4) && (A.fuse_col & 4)) {  // A's column pass of k_dir's rows
    PH_T(tc0);
    col_conv<COOP>(G, Pt, B.spec, tf_of(G, img, 0), lds);
    team_sync(tm);
    PH_ADD(3, tc0);
  }
  const double bks_scalar = st.bks_scalar;
  const double flux = st.flux;
  const double gd = st.gd;
  // compact gn (ImgState::g32): loaders fetch the raw f32, users decode it
  const int g32 = st.g32;
  const double gsc = st.sc, grc = 1.0 / st.sc, gfill = st.gfill;
  // (the raw f32 travels in the low word of the f64 operand register, so both
  // storage modes use the same registers)
  auto gdec1 = [&](float v) __attribute__((always_inline)) {
    const double g = v;
    return g > 0 ? (g32 == 2 ? div_rn(g, gsc, grc) : g) : gfill;
  };
  auto gdec = [&](double r) __attribute__((always_inline)) {
    return g32 ? gdec1(__int_as_float(__double2loint(r))) : r;
  };
  double fr = st.Fold[0];
  for (int k = 1; k < P.M; ++k) fr = py_max2(fr, st.Fold[k]);
  const int ls_cap = A.ls_cap;  // trial cap (bsgp_api.hip): never reached for 0 < beta < 1
  Objective obj = make_obj(A, st.beta);
  double lam = 1.0;
  double f_acc = 0.0;
  int nls = 0, passes = 0, status = 0, series_evals = 0;
  bool accepted = false;
  bool acc_series = false;  // the accepted trial came from the series (lam * max|u| <= rho)
  constexpr int NT = 2 * K + 2;  // [2k],[2k+1]: lambda_k sums; [2K]: const; [2K+1]: dDiv/dbeta
  // The lambda-independent sum (sum s*gn^b, or sum gn at beta = 1) is carried
  // in the state; with adaptive beta it changes with beta and is recomputed.
  double konst = st.konst;
  // Adaptive beta on a float32 image (params.gn_f32): the reference re-sums
  // s*gn**beta at every trial's beta as float32 terms in numpy's float32
  // order (sgp.py:458, 782), and the float32 terms of betaDivDeriv round to
  // float32 (beta_deriv_px_f32).  pw is free scratch until the accept
  // rewrites it (no series moments with adaptive beta).
  const bool k32 = ADAPT && P.gn_f32 != 0;
  // One-workgroup images keep each trial's float32 powers x**beta from the
  // beta derivative's pass (xbc, the upper half of pw: the np_f32_sum values
  // take its first nleaf + nnode floats) for that trial's K, read back after
  // the pass's block barrier: one float64 pow per pixel and trial less, the
  // same bits.  Teams recompute them (no data barrier between the pass and K).
  // Only float64 storage has room for it: a float32 pw holds vec_stride floats
  // and the half spectrum follows right after it.
  float* const xbc =
      (k32 && tm.T == 1 && sizeof(V) == 8) ? reinterpret_cast<float*>(B.pw) + N : nullptr;
  auto konst32 = [&](double b) -> double {
    const float sf = (float)(1 / (b * (b - 1)));
    const float bf = (float)b;  // x**beta: the exponent is cast to float32
    return (double)np_f32_sum(
        A.pw,
        [&](int i) {
          if (xbc) return sf * xbc[i];
          const double g = g32 ? gdec1(reinterpret_cast<const float*>(B.gns)[i]) : B.gns[i];
          return sf * libm_powf((float)g, bf);
        },
        reinterpret_cast<float*>(B.pw), Pt, tm);
  };
  auto bderiv = [&](double den, double g, double b, int i) __attribute__((always_inline)) {
    return k32 ? beta_deriv_px_f32(den, g, b, xbc ? xbc + i : nullptr) : beta_deriv_px(den, g, b);
  };
  // Small-step series (general beta, fixed beta): with den_i(lam) =
  // a_i (1 + lam u_i), a_i = x_tf_i + bkg_i, u_i = d_tf_i / a_i,
  //   sum den^b        = sum_m binom(b, m)   lam^m P_m,  P_m = sum a^b u^m
  //   sum gn den^(b-1) = sum_m binom(b-1, m) lam^m Q_m,  Q_m = sum gn a^(b-1) u^m
  // so every trial with lam * max|u| <= kSeriesRho is evaluated without a pass
  // over the image (truncation < 1e-17 relative at MS = 6: (0.01)^7 * binom).
  constexpr int MS = 6;
  constexpr double kSeriesRho = 0.01;
  // Beyond lam * max|u| <= kSeriesRho the series is still exact to rounding
  // when the terms past m = MS are small: with |binom(b, m+1) / binom(b, m)|
  // <= 1 for m >= MS + 1 (0 <= b <= MS + 2; also for b - 1) and
  // sum w |u|^(MS+1) <= max|u| * P_MS
  // (P_MS = sum w u^MS >= 0), the tail of each series is at most
  //   |binom(b, MS+1)| lam^(MS+1) max|u| P_MS / (1 - lam max|u|),
  // and trials whose tails stay below 2^-60 of the leading moment are taken
  // in closed form too.  The bound is driven by the few pixels with large u:
  // on C3's stagnating iterations (max|u| ~ 0.04 from ~80 pixels, the rest
  // <= 0.004) it covers every trial after the first, where lam * max|u| <=
  // kSeriesRho left lam = 0.4 to a direct pass (0.46 passes per iteration).
  constexpr double kSeriesTail = 8.673617379884035e-19;  // 2^-60
  const bool tail_bound = BSGP_SERIES_BOUND && obj.beta >= 0.0 && obj.beta <= MS + 2;
  const bool series = (MODE == 3 || MODE == 4) && !adapt && P.ls_series != 0;
  // the moments and binomial coefficients are the same in every thread: they
  // live in LDS after the first pass (ser[0..3][MS+1] = P, Q, binom(b, m),
  // binom(b-1, m)), not in VGPRs across the trial passes
  double* ser = red + kWaves * kMaxRed + kMaxRed + 8;
  double rho = INFINITY;
  // Pass 1 also sums the second trial (lam = beta) directly when the series is
  // on: where max|u| keeps that trial out of the closed form (the iterations
  // whose first trial fails at a large step), it is taken from these sums
  // instead of a direct pass over the image.  Both sums come from the same
  // per-pixel arithmetic as a direct pass's (x0 + lam d_tf), summed in the
  // pass's own order.
  const bool k2 = BSGP_LS1_K2 && !COOP && series;
  const double lam2 = lam * P.beta;
  double f2 = NAN;     // the second trial's objective from pass 1
  bool have2 = false;  // f2 holds the next trial's objective
  // ---- pass 1, fused into the inverse rows that produce d_tf: lam = 1 direct
  {
    constexpr int O2 = 4 + 2 * (MS + 1);
    constexpr int N1 = O2 + ((BSGP_LS1_K2 && !COOP) ? 2 : 0);  // lam=1 sums, const, dDiv/dbeta, P_m, Q_m, lam=beta sums
    double t1[N1];
#pragma unroll
    for (int k = 0; k < N1; ++k) t1[k] = 0.0;
    double umax = 0.0;
    struct LsIn {
      double x0, g, p0, bkv;
    };
    row_inv2<BSGP_LS1_PRE, BSGP_LS1_JCH, BSGP_LS_COMP, COOP, BSGP_LS1_PIPE, 13>(
        G, Pt, B.spec, lds,
        [&](int r, int j) {
          const int i = r * G.W + j;
          LsIn q;
          q.x0 = B.xtf[i];
          q.g = g_raw(g32, B.gns, i);
          q.p0 = opt_ld(series, B.pw, i, 0.0);
          q.bkv = opt_ld(bmap, B.bks, i, bks_scalar);
          return q;
        },
        [&](int r, int j, double v, const LsIn& q) {
      const int i = r * G.W + j;
      B.dtf[i] = v;
      const double g = gdec(q.g);
      const double x0 = q.x0;
      const double bkv = q.bkv;
      const double xt = x0 + lam * v;
      obj.template terms_m<MODE>(xt, xt + bkv, g, &t1[0]);
      if constexpr (adapt) {
        if (!k32) t1[2] += obj.konst(g);
        t1[3] += bderiv(xt + bkv, g, obj.beta, i);
      }
      if (series) {
        const double a = x0 + bkv;
        const double u = v / a;
        const double p0 = q.p0;  // = fpow(a, beta-1), stored at the last accept
        // MODE 4: the float32-rounded (s*b)*gn factor; combined without c2 below
        const double A0 = a * p0, B0 = (MODE == 4 ? (double)(obj.c2f * (float)g) : g) * p0;
        double um = 1.0;
#pragma unroll
        for (int m = 0; m <= MS; ++m) {
          t1[4 + m] += A0 * um;
          t1[4 + MS + 1 + m] += B0 * um;
          um *= u;
        }
        const double au = fabs(u);
        umax = (au > umax || au != au || !(a > 0)) ? (a > 0 ? au : INFINITY) : umax;
        if constexpr (BSGP_LS1_K2 && !COOP) {
          if (k2) {
            const double x2 = x0 + lam2 * v;
            obj.template terms_m<MODE>(x2, x2 + bkv, g, &t1[O2]);
          }
        }
      }
    });
    // sums and max|u| in one team barrier (the same bits as team_sum + team_max)
    if (series) {
      team_sum_max<N1>(t1, umax, red, tm, 25);  // (phase profile slots 25, 26)
      rho = umax;
    } else {
      team_sum<N1>(t1, red, tm);
    }
    PH_ADD(4, tk0);
    if (series && threadIdx.x == 0) {
      for (int m = 0; m <= MS; ++m) {
        ser[m] = t1[4 + m];
        ser[MS + 1 + m] = t1[4 + MS + 1 + m];
      }
    }
    if (adapt) konst = k32 ? konst32(obj.beta) : t1[2];
    ++passes;
    ++nls;
    const double f1 = obj.combine(konst, t1[0], t1[1], flux, (double)N);
    if (f1 <= fr + P.gamma * lam * gd || lam < 1e-12) {
      f_acc = f1;
      accepted = true;
    } else {
      lam = lam * P.beta;
      if (adapt) {  // sgp.py:798-800: beta -= lr * mean(dDiv/dbeta)
        const double bgrad = (obj.beta == 0.0 || obj.beta == 1.0) ? 0.0 : t1[3] / N;
        obj.set_beta(obj.beta - lr_st * bgrad);
      }
      if constexpr (BSGP_LS1_K2 && !COOP) {
        if (k2) {
          f2 = obj.combine(konst, t1[O2], t1[O2 + 1], flux, (double)N);
          have2 = true;
        }
      }
    }
  }
  // binomial coefficients of the series (and, for the tail bound, the
  // scaled leading terms |binom(., MS+1)| P_MS / P_0 of both series)
  if (series && threadIdx.x == 0) {
    double c0 = 1.0, c1 = 1.0;
    ser[2 * (MS + 1)] = 1.0;
    ser[3 * (MS + 1)] = 1.0;
    for (int m = 1; m <= MS; ++m) {
      c0 = c0 * (obj.beta - (m - 1)) / m;
      c1 = c1 * (obj.beta - 1 - (m - 1)) / m;
      ser[2 * (MS + 1) + m] = c0;
      ser[3 * (MS + 1) + m] = c1;
    }
    const double c7p = fabs(c0 * (obj.beta - MS) / (MS + 1));
    const double c7q = fabs(c1 * (obj.beta - 1 - MS) / (MS + 1));
    const double tp = c7p * ser[MS] / ser[0], tq = c7q * ser[2 * MS + 1] / ser[MS + 1];
    // (a NaN or non-positive leading moment: no closed form past kSeriesRho)
    ser[4 * (MS + 1)] = (ser[0] > 0 && ser[MS + 1] > 0 && tp == tp && tq == tq)
                            ? (tp > tq ? tp : tq)
                            : INFINITY;
  }
  __syncthreads();
  const double tail_c = (series && tail_bound) ? ser[4 * (MS + 1)] : INFINITY;
  auto series_ok = [&](double l) __attribute__((always_inline)) {
    const double lu = l * rho;
    if (lu <= kSeriesRho) return true;
    if (!(lu <= 0.5)) return false;
    double l7 = l;
#pragma unroll
    for (int m = 1; m <= MS; ++m) l7 *= l;
    return l7 * rho * tail_c / (1.0 - lu) <= kSeriesTail;
  };
  PH_T(tk1);
  while (!accepted) {
    if (have2 && !series_ok(lam)) {
      // the second trial, summed by pass 1 (f2 is NaN only if its sums are:
      // then it fails the test, as a direct pass's NaN would)
      have2 = false;
      ++nls;
      if (f2 <= fr + P.gamma * lam * gd || lam < 1e-12) {
        f_acc = f2;
        accepted = true;
        break;
      }
      lam = lam * P.beta;
      if (nls > ls_cap) {
        status = 1;
        break;
      }
      continue;
    }
    have2 = false;
    if (BSGP_LS_SERIES_LANES && series && series_ok(lam)) {
      // Closed-form trials, kLsLanes at once: lane j of every wave evaluates
      // the j-th next trial, lam * beta^j (the same sequential products the
      // one-trial-at-a-time loop below forms, so the same bits), with the same
      // arithmetic as that loop.  The first lane whose trial ends the search
      // decides: it accepts, it is past the closed form's range (a direct pass
      // from there on), or it fails at the trial cap.  Every wave computes the
      // same decision (scalar control stays identical in every thread).
      constexpr int L = kLsLanes;
      const int ln = (int)(threadIdx.x & 63u);
      const int lj = ln < L ? ln : L - 1;
      double lt = lam;
      for (int i = 0; i < lj; ++i) lt = lt * P.beta;
      double s0 = 0.0, s1 = 0.0, lm = 1.0;
      for (int m = 0; m <= MS; ++m) {
        s0 += ser[2 * (MS + 1) + m] * lm * ser[m];
        s1 += ser[3 * (MS + 1) + m] * lm * ser[MS + 1 + m];
        lm *= lt;
      }
      const double fk =
          obj.combine(konst, obj.c1 * s0, (MODE == 4 ? 1.0 : obj.c2) * s1, flux, (double)N);
      const bool ok = series_ok(lt);
      const bool acc = fk <= fr + P.gamma * lt * gd || lt < 1e-12;
      const bool cap = nls + lj + 1 > ls_cap;
      const unsigned long long ends = __ballot(ln < L && (!ok || acc || cap));
      const int j = ends ? __ffsll((long long)ends) - 1 : L - 1;
      const double lt_j = __shfl(lt, j, 64);
      const double fk_j = __shfl(fk, j, 64);
      const bool ok_j = __shfl((int)ok, j, 64) != 0;
      const bool acc_j = __shfl((int)acc, j, 64) != 0;
      if (!ok_j) {  // trial j needs a direct pass (its predecessors failed)
        nls += j;
        series_evals += j;
        lam = lt_j;
        continue;
      }
      nls += j + 1;
      series_evals += j + 1;
      if (acc_j) {
        f_acc = fk_j;
        lam = lt_j;
        accepted = true;
        acc_series = true;
        break;
      }
      lam = lt_j * P.beta;
      if (nls > ls_cap) {
        status = 1;
        break;
      }
      continue;
    }
    if (series && series_ok(lam)) {
      // closed-form trial: no pass over the image
      double s0 = 0.0, s1 = 0.0, lm = 1.0;
      for (int m = 0; m <= MS; ++m) {
        s0 += ser[2 * (MS + 1) + m] * lm * ser[m];
        s1 += ser[3 * (MS + 1) + m] * lm * ser[MS + 1 + m];
        lm *= lam;
      }
      const double fk =
          obj.combine(konst, obj.c1 * s0, (MODE == 4 ? 1.0 : obj.c2) * s1, flux, (double)N);
      ++nls;
      ++series_evals;
      if (fk <= fr + P.gamma * lam * gd || lam < 1e-12) {
        f_acc = fk;
        accepted = true;
        acc_series = true;
        break;
      }
      lam = lam * P.beta;
      if (nls > ls_cap) {
        status = 1;
        break;
      }
      continue;
    }
    // ---- direct pass: K trial lambdas streamed over (x_tf, d_tf, gn)
    double lamk[K];
    lamk[0] = lam;
#pragma unroll
    for (int k = 1; k < K; ++k) lamk[k] = lamk[k - 1] * P.beta;
    double t[NT];
#pragma unroll
    for (int k = 0; k < NT; ++k) t[k] = 0.0;
    auto eval_px = [&](double x0, double dt, double g, double bkv, int i) __attribute__((always_inline)) {
      if constexpr (adapt) {
        if (!k32) t[2 * K] += obj.konst(g);
      }
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const double xt = x0 + lamk[k] * dt;
        const double den = xt + bkv;
        obj.template terms_m<MODE>(xt, den, g, &t[2 * k]);
      }
      if constexpr (K == 1 && adapt)
        t[2 * K + 1] += bderiv(x0 + lamk[0] * dt + bkv, g, obj.beta, i);
    };
    const V* xtf = B.xtf;
    const V* dtf = B.dtf;
    const double* gns = B.gns;
    const double* bks = B.bks;
    stream2<2>(
        Pt, npair,
        [&](int p) {
          struct Ld {
            double2 x, d, g, b;
          } v;
          v.x = ld2(xtf, p);
          v.d = ld2(dtf, p);
          v.g = g_raw2(g32, gns, p);  // compact: the pair's two f32 in the first f64
          v.b = opt_ld2(bmap, bks, p, bks_scalar);
          return v;
        },
        [&](int p, const auto& v) {
          double g0 = v.g.x, g1 = v.g.y;
          if (g32) {
            const long long w = __double_as_longlong(v.g.x);
            g0 = gdec1(__int_as_float((int)(w & 0xffffffffLL)));
            g1 = gdec1(__int_as_float((int)(w >> 32)));
          }
          eval_px(v.x.x, v.d.x, g0, v.b.x, 2 * p);
          if (!odd || 2 * p + 1 < N) eval_px(v.x.y, v.d.y, g1, v.b.y, 2 * p + 1);
        });
    team_sum<NT>(t, red, tm);
    if (adapt) konst = k32 ? konst32(obj.beta) : t[2 * K];
    ++passes;
#pragma unroll
    for (int k = 0; k < K; ++k) {
      if (!accepted) {
        const double fk = obj.combine(konst, t[2 * k], t[2 * k + 1], flux, (double)N);
        ++nls;
        if (fk <= fr + P.gamma * lamk[k] * gd || lamk[k] < 1e-12) {
          accepted = true;
          f_acc = fk;
          lam = lamk[k];
        }
      }
    }
    if (accepted) break;
    lam = lamk[K - 1] * P.beta;
    if (adapt) {  // sgp.py:798-800: beta -= lr * mean(dDiv/dbeta)   (K == 1 here)
      const double bgrad = (obj.beta == 0.0 || obj.beta == 1.0) ? 0.0 : t[2 * K + 1] / N;
      obj.set_beta(obj.beta - lr_st * bgrad);
    }
    if (nls > ls_cap) {  // only for beta outside (0, 1): the reference never terminates
      status = 1;
      break;
    }
  }
  PH_ADD(5, tk1);
  PH_T(tk2);
  // accept: x_tf += lam*d_tf; w = gn/den or gn*den^(b-2) (sgp.py:337-345, 790)
  const double lam_acc = lam;
  // A series step moved every den_i by a factor (1 + t_i), |t_i| = lam|u_i| <=
  // kSeriesRho: den^(b-1) follows from the stored one as pw * (1 + t)^(b-1), the
  // binomial series to t^MS (truncation < 1e-16 relative), ~25 VALU ops
  // instead of a log and an exp per pixel.
  const bool pw_series = BSGP_ACC_SERIES && acc_series && MODE >= 3;
  const double bm1 = obj.beta - 1;
  struct AcIn {
    double x, d, g, bkv, p0;
  };
  row_fwd2<BSGP_LSACC_JCH, BSGP_LSACC_PF, BSGP_LS_COMP, COOP, BSGP_LSACC_PIPE, 16>(
      G, Pt, G.H, G.W, G.sld, B.spec, lds,
      [&](int r, int j) {
        const int i = r * G.W + j;
        AcIn q;
        q.x = B.xtf[i];
        q.d = B.dtf[i];
        q.g = g_raw(g32, B.gns, i);
        q.bkv = opt_ld(bmap, B.bks, i, bks_scalar);
        q.p0 = opt_ld(pw_series, B.pw, i, 0.0);
        return q;
      },
      [&](int r, int j, const AcIn& q) {
        const int i = r * G.W + j;
        const double xt = q.x + lam_acc * q.d;
        B.xtf[i] = xt;
        const double den = xt + q.bkv;
        const double g = gdec(q.g);
        if (P.variant != BSGP_VARIANT_BETA) return g / den;  // KL: w = gn/den
        double p;
        if (pw_series) {
          const double t = lam_acc * (q.d / (q.x + q.bkv));
          // (1+t)^(b-1) = 1 + e1 t (1 + e2 t (1 + ... (1 + e6 t))), e_m = (b-m)/m
          double h = 1.0;
#pragma unroll
          for (int m = MS; m >= 1; --m) h = fma(fma(obj.beta, 1.0 / m, -1.0) * t, h, 1.0);
          p = q.p0 * h;
        } else {
          p = fpow(den, bm1);
        }
        B.pw[i] = p;
        return g * (p / den);
      });
  PH_ADD(6, tk2);
  if ((BSGP_FUSE_COL_CODE & 2) && (A.fuse_col & 2)) {  // AT's column pass follows here
    PH_T(tc0);
    team_sync(tm);
    col_conv<COOP>(G, Pt, B.spec, tf_of(G, img, 1), lds);
    PH_ADD(3, tc0);
  }
  PH_ADD(7, tk0);
  team_end(st, tm);
  if (leader(tm)) {
    // bit 0: the fv >= fr warning (sgp.py:803-804); bits 8..23: this
    // iteration's line-search trials (the reference's betaDiv calls at :782)
    if (A.out.flags)
      A.out.flags[(size_t)img * (P.MAXIT + 1) + st.iter] =
          ((f_acc >= fr) ? 1 : 0) | ((nls < 0xffff ? nls : 0xffff) << 8);
    st.fv = f_acc;
    st.beta = obj.beta;
    st.konst = konst;
    st.lam = lam_acc;
    st.E_ls += nls;
    st.ls_passes += passes;
    st.ls_series += series_evals;
    st.status |= status;
  }
}

template <int K, int MODE, bool ADAPT, bool COOP, class V>
__global__ void __launch_bounds__(kBlock) BSGP_LS_ATTR k_ls(SolveArgs A) {
  const int img = team_img(A);
  if (A.st[img].stop) return;
  load_tw_lds(A.g);
  ls_phase<K, MODE, ADAPT, COOP, V>(A, img);
}


// ------------------------------ kernel: gradient, x update, BB, stop rules
// sgp.py:337-414 (= 785-879): g_new = g1(den) - AT(w), x += lam*d, the
// Barzilai-Borwein step lengths with the tau alternation, the stop rules,
// and the outputs once the image stops (sgp.py:424-438).
template <bool COOP, class V>
__device__ __forceinline__ void bb_phase(const SolveArgs& A, int img) {
  BSGP_LDS_VIEWS(A);
  ImgState& st = A.st[img];
  PH_T(tk0);
  Team tm = make_team(A, img, st);
  const Geo& G = A.g;
  const Part Pt = make_part(tm, G.nfw, G.W);
  const bsgp_params& P = A.prm;
  const int N = G.H * G.W;
  const int tid = threadIdx.x;
  const bool beta_obj = P.variant == BSGP_VARIANT_BETA;
  Bufs<V> B = slot_bufs<V>(A, img, st.par);
  Dir D = make_dir(A, st);
  const double lam = st.lam;
  const double lo = st.lo, hi = st.hi;
  // every state value the members use is read before the first team barrier:
  // member 0 rewrites the state after the last one
  const double alpha = st.alpha;
  double vmin_ring = INFINITY;  // min(Valpha[0 .. M_alpha-2])
  for (int k = 0; k < P.M_alpha - 1; ++k) vmin_ring = k ? py_min2(vmin_ring, st.Valpha[k]) : st.Valpha[0];
  const int iter = st.iter;
  const double tau0 = st.tau, init_lr = st.init_lr, lr0 = st.lr;
  const int epoch = st.epoch;
  const double fv = st.fv, Dcoeff = st.Dcoeff, tol = st.tol, fold_last = st.Fold[P.M - 1];
  const double sc = st.sc;
  double bb[6] = {0, 0, 0, 0, 0, 0};  // bk, ck, sk2.sk2, yk2.yk2, sk.sk, x.x
  struct BbIn {
    double p, x, g;
  };
  row_inv2<BSGP_BB_PRE, BSGP_BB_JCH, BSGP_BB_COMP, COOP, BSGP_BB_PIPE, 19>(
      G, Pt, B.spec, lds,
      [&](int r, int j) {
        const int i = r * G.W + j;
        BbIn q;
        q.p = opt_ld(beta_obj, B.pw, i, 1.0);
        q.x = B.xa[i];
        q.g = B.ga[i];
        return q;
      },
      [&](int r, int j, double at, const BbIn& q) {
    const int i = r * G.W + j;
    const double gnew = q.p - at;  // sgp.py:342 / 790
    const double x = q.x, g = q.g;
    const double d = D.d(x, g);
    const double sk = lam * d;
    const double xn = x + lam * d;
    const double yk = gnew - g;
    const double X = clipX(xn, lo, hi);
    const double Dd = 1 / X;
    const double sk2 = sk * Dd;
    const double yk2 = yk * X;
    bb[0] += sk2 * yk;
    bb[1] += yk2 * sk;
    bb[2] += sk2 * sk2;
    bb[3] += yk2 * yk2;
    bb[4] += sk * sk;
    bb[5] += xn * xn;
    B.xb[i] = xn;
    B.gb[i] = gnew;
  });
  team_sum<6>(bb, red, tm);
  PH_ADD(8, tk0);
  // Barzilai-Borwein (sgp.py:366-386)
  double alpha1, alpha2;
  if (bb[0] <= 0) {
    alpha1 = py_min2(10 * alpha, P.alpha_max);
  } else {
    alpha1 = py_min2(P.alpha_max, py_max2(P.alpha_min, bb[2] / bb[0]));
  }
  if (bb[1] <= 0) {
    alpha2 = py_min2(10 * alpha, P.alpha_max);
  } else {
    alpha2 = py_min2(P.alpha_max, py_max2(P.alpha_min, bb[1] / bb[3]));
  }
  const double vmin = P.M_alpha > 1 ? py_min2(vmin_ring, alpha2) : alpha2;  // python min(Valpha)
  double tau = tau0, anew;
  if (iter <= 20) {
    anew = vmin;
  } else if (alpha2 / alpha1 < tau) {
    anew = vmin;
    tau = tau * 0.9;
  } else {
    anew = alpha1;
    tau = tau * 1.1;
  }
  const double lr = (P.variant == BSGP_VARIANT_BETA && P.schedule_lr)
                        ? init_lr * exp(-P.lr_exp_param * epoch)
                        : lr0;
  // stop rules (sgp.py:390-414)
  const int it2 = iter + 1;
  bool loop = true;
  double crit = 0.0;
  const double dk = Dcoeff * fv;
  if (P.stop_criterion == 2) {
    crit = bb[4] / bb[5];
    loop = crit > tol;
  } else if (P.stop_criterion == 3) {
    crit = (fold_last - fv) / fv;
    loop = crit > tol && crit >= 0;
  } else if (P.stop_criterion == 4) {
    crit = dk;
    loop = dk > tol;
  }
  if (it2 > P.MAXIT) loop = false;
  if (!loop) {
    // outputs: x reverts to prev_x = xa (sgp.py:424-438, 892-895)
    double* xo = A.out.x + (size_t)img * N;
    for (int i = Pt.gt0 + tid; i < N; i += Pt.gts) xo[i] = B.xa[i] * sc;
  }
  team_end(st, tm);
  if (leader(tm)) {
    const size_t M1 = (size_t)P.MAXIT + 1;
    A.out.discr[img * M1 + it2 - 1] = dk;
    if (A.out.times) A.out.times[img * M1 + it2 - 1] = realtime_s() - st.t0;
    if (A.out.crit) A.out.crit[img * M1 + it2 - 1] = crit;
    st.Valpha[P.M_alpha - 1] = alpha2;
    st.alpha = anew;
    st.tau = tau;
    st.lr = lr;
    st.iter = it2;
    if (loop) {
      st.par ^= 1;
      st.Xones = 0;
    } else {
      st.stop = 1;
      A.out.iters[img] = it2 - 1;
      if (A.out.beta_final) A.out.beta_final[img] = st.beta;
      write_counters(A, st, img, tm.T);
      count_stopped(A);
    }
  }
}

template <bool COOP, class V>
__global__ void __launch_bounds__(kBlock) k_bb(SolveArgs A) {
  const int img = team_img(A);
  if (A.st[img].stop) return;
  load_tw_lds(A.g);
  bb_phase<COOP, V>(A, img);
}

// ------------------------------------------- persistent task-queue solver
// One-workgroup images with per-wave transforms (T == 1, the batched configs
// C3/C5 and the star stamps): ONE launch runs every iteration of every image
// of a sub-batch.  A task is one iteration of one image.  Images wait in a
// ready ring: a workgroup takes the entry at the ring's head, runs one
// iteration of that image and, unless the image stopped, appends it at the
// tail.  So every resident workgroup has work until the last iterations, no
// launch ends in a partly-occupied round (1024 images on 768 slots are 1.33
// rounds per launch in the phase-kernel solve), a CU holds workgroups in
// different phases of their tasks at once (memory-bound row passes beside
// LDS-bound transforms), and a stopped image costs nothing more (the star
// stamps stop after ~20 of MAXIT 500 iterations at different times: with one
// task per (iteration, image) slot, the slots of stopped images were still
// dequeued and skipped one by one, 15 % of the stamp solve).  A task runs the
// phases of one iteration (dir_phase, A's column pass, ls_phase with AT's
// column pass, bb_phase), the same device code the phase kernels run, so the
// results are bit-identical to theirs.  Solves with a data-dependent stop
// rule (2-4) take the ring; fixed-length solves take the slot order below.
//
// Ring (queue[0] = head, queue[1] = tail, then ring[nimg] of 64-bit entries
// (h << 32 | image) for position h; k_ring_init fills positions 0..nimg-1):
// an image is in the ring at most once, so the entries written and not yet
// read are distinct images, at most nimg, and position h + nimg is never
// written before position h has been read.  Hand-off (MI355X_MICROARCH.md,
// inter-workgroup visibility, valid producer/consumer forms): the producer's
// waves drain their stores, a workgroup barrier, lane 0 releases at agent
// scope, takes a tail position with an atomic add and stores the entry with a
// relaxed agent-scope (sc1) 64-bit store; the consumer's lane 0 polls its
// position with sc1 loads until the entry carries that position, acquires at
// agent scope, and a workgroup barrier lets the other waves load.  A consumer
// whose position is never written (every image stopped) sees the running
// count at 0 and leaves; the poll is bounded anyway (timeout -> status bit 4,
// every workgroup leaves).
static __global__ void k_ring_init(unsigned* queue, int nimg, int img0) {
  unsigned long long* ring = reinterpret_cast<unsigned long long*>(queue + 4);
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i == 0) {
    queue[0] = 0;
    queue[1] = (unsigned)nimg;
  }
  if (i < nimg) ring[i] = ((unsigned long long)i << 32) | (unsigned)(img0 + i);
}

#ifndef BSGP_PERSIST_ATTR
// (per-wave plans: 3 waves/SIMD, the phase kernels' own; cooperative plans'
// 512-thread workgroups: 2 waves/SIMD per workgroup, BSGP_PERSIST_COOP_WAVES)
#ifndef BSGP_PERSIST_COOP_WAVES
#define BSGP_PERSIST_COOP_WAVES 2
#endif
#ifndef BSGP_PERSIST_WAVES
#define BSGP_PERSIST_WAVES 3
#endif
#define BSGP_PERSIST_ATTR \
  __attribute__((amdgpu_waves_per_eu(COOP ? BSGP_PERSIST_COOP_WAVES : BSGP_PERSIST_WAVES)))
#endif

__device__ __forceinline__ unsigned long long ld_sc1_u64(const unsigned long long* p) {
  return __hip_atomic_load((gu64*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// The phases of a task are separate (noinline) functions, so each keeps the
// register allocation of its own kernel.  Their argument block is the
// kernel's own (the kernarg segment): the kernel passes its address, the
// callee makes it wave-uniform (readfirstlane) and reads it as constant
// memory, i.e. with scalar loads (the kernarg-segment intrinsic itself
// yields 0 outside a kernel).  Inlined into one kernel body the phases
// spilled 57-88 VGPRs inside their loops at the 168 VGPRs of 3 waves/SIMD (the
// scalar state of all phases at once); as calls the only spill code is each
// phase's callee-saved registers at its entry and exit (~210 VGPRs per wave
// per task, ~3 % of a task's bytes, L2-resident).
#ifndef BSGP_PERSIST_SB
#define BSGP_PERSIST_SB 1
#endif
#ifndef BSGP_PERSIST_CALLS
#define BSGP_PERSIST_CALLS 1
#endif
#if BSGP_PERSIST_CALLS
#define BSGP_PERSIST_FN __attribute__((noinline))
#else
#define BSGP_PERSIST_FN __forceinline__
#endif
struct ArgRef {
  unsigned lo, hi;  // address of the kernel's SolveArgs (kernarg segment)
};
__device__ __forceinline__ ArgRef kernarg_ref() {
  const unsigned long long a = (unsigned long long)__builtin_amdgcn_kernarg_segment_ptr();
  return ArgRef{(unsigned)a, (unsigned)(a >> 32)};
}
__device__ __forceinline__ const SolveArgs& args_of(ArgRef r) {
  typedef const __attribute__((address_space(4))) SolveArgs* KP;
  // (readfirstlane returns int: widen through unsigned, no sign extension)
  const unsigned lo = (unsigned)__builtin_amdgcn_readfirstlane((int)r.lo);
  const unsigned hi = (unsigned)__builtin_amdgcn_readfirstlane((int)r.hi);
  const unsigned long long a = ((unsigned long long)hi << 32) | (unsigned long long)lo;
  KP p = (KP)a;
  asm volatile("" : "+s"(p));  // re-read per call: nothing of it is hoisted across phases
  return *(const SolveArgs*)p;
}
template <bool COOP, class V>
__device__ BSGP_PERSIST_FN void persist_setup(ArgRef r, int img) {
  setup_phase<COOP, V>(args_of(r), __builtin_amdgcn_readfirstlane(img));
}
template <bool COOP, class V>
__device__ BSGP_PERSIST_FN void persist_dir(ArgRef r, int img) {
  dir_phase<COOP, V, false>(args_of(r), __builtin_amdgcn_readfirstlane(img));
}
template <bool COOP>
__device__ BSGP_PERSIST_FN void persist_col_a(ArgRef r, int img) {
  const SolveArgs& A = args_of(r);
  img = __builtin_amdgcn_readfirstlane(img);
  BSGP_LDS_VIEWS(A);
  (void)red;
  Team tm{};
  tm.T = 1;
  const Bufs<double> Bd = slot_bufs<double>(A, img, 0);  // spec only (same offset for V)
  PH_T(tc0);
  // (a cooperative plan's column pass on its column groups, as k_col)
  col_conv<COOP>(A.g, make_part(tm, COOP ? A.g.nfc : A.g.nfw, A.g.W), Bd.spec,
                 tf_of(A.g, img, 0), lds);
  PH_ADD(3, tc0);
}
template <int K, int MODE, bool ADAPT, bool COOP, class V, bool SB = false>
__device__ BSGP_PERSIST_FN void persist_ls(ArgRef r, int img) {
  ls_phase<K, MODE, ADAPT, COOP, V, SB>(args_of(r), __builtin_amdgcn_readfirstlane(img));
}
template <bool COOP, class V>
__device__ BSGP_PERSIST_FN void persist_bb(ArgRef r, int img) {
  bb_phase<COOP, V>(args_of(r), __builtin_amdgcn_readfirstlane(img));
}

// Slot order (fixed-length solves, stop rules 0/1): task t = (k - 1) * nimg + i
// runs iteration k of image i, dequeued from one counter; iteration k waits
// for done[i] >= k - 1 (published as below with a 32-bit sc1 store).  Every
// image runs every iteration, so no slot is ever skipped, and the iterations
// of all images advance in lock step (C3: the ring's completion order was
// 5 % slower, A/B).  Data-dependent stop rules (2-4) take the ready ring.
constexpr unsigned kDoneStop = 0x40000000u;
__device__ __forceinline__ unsigned ld_sc1_u32(const unsigned* p) {
  return __hip_atomic_load((gu32*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <bool COOP, int K, int MODE, bool ADAPT, class V, bool SB = false>
__global__ void __launch_bounds__(kBlock) BSGP_PERSIST_ATTR k_persist(SolveArgs A,
                                                                        unsigned* queue,
                                                                        unsigned* done) {
  BSGP_LDS_VIEWS(A);
  (void)red;
  __shared__ int s_img;
  __shared__ unsigned s_k;
  const int tid = threadIdx.x;
  const Geo& G = A.g;
  load_tw_lds(G);
  const unsigned nimg = (unsigned)A.nimg;
  // fold_setup (slot order only): task t = kk * nimg + i is image i's kk-th
  // task, the setup first (kk = 0), then iteration kk; without it iteration
  // kk + 1.  Either way task kk waits for done[i] >= kk and publishes kk + 1.
  const unsigned fs = A.fold_setup ? 1u : 0u;
  const unsigned total = ((unsigned)A.prm.MAXIT + fs) * nimg;
  const bool use_ring = A.prm.stop_criterion >= 2 && A.prm.stop_criterion <= 4;
  unsigned long long* ring = reinterpret_cast<unsigned long long*>(queue + 4);
  for (;;) {
    PH_T(tq);
    if (tid == 0) {
      int img = -1;  // -1: leave, -2: nothing to run for this entry
      unsigned k = 0;
      if (use_ring) {
        const unsigned h = atomicAdd(queue, 1u);
        unsigned long long e = ld_sc1_u64(ring + h % nimg);
        unsigned spins = 0;
        while ((unsigned)(e >> 32) != h) {
          __builtin_amdgcn_s_sleep(2);
          if ((++spins & 63u) == 0) {
            if (__hip_atomic_load((gi32*)A.active, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) <=
                0)
              break;  // every image has stopped: position h is never written
            if (__hip_atomic_load((gi32*)A.tfail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ||
                spins > A.spin_limit) {
              __hip_atomic_store((gi32*)A.tfail, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              break;
            }
          }
          e = ld_sc1_u64(ring + h % nimg);
        }
        if ((unsigned)(e >> 32) == h) {
          img = (int)(unsigned)e;
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          // stopped by the setup (status 8) before its first iteration: it
          // leaves the ring (the setup already counted it down from B in
          // count_stopped, so it is not among the running images)
          if (A.st[img].stop) img = -2;
        }
      } else {
        unsigned t = atomicAdd(queue, 1u);
        if (t < total && __hip_atomic_load((gi32*)A.active, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT) <= 0)
          t = total;  // every image has stopped: nothing left to run
        if (t < total) {
          img = A.img0 + (int)(t % nimg);
          const unsigned need = t / nimg;  // tasks of img that must be done
          k = need + 1;
          unsigned d = ld_sc1_u32(done + img), spins = 0;
          while (d < need) {
            __builtin_amdgcn_s_sleep(2);
            d = ld_sc1_u32(done + img);
            if (((++spins & 1023u) == 0 || spins > A.spin_limit) &&
                (__hip_atomic_load((gi32*)A.tfail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ||
                 spins > A.spin_limit)) {
              __hip_atomic_store((gi32*)A.tfail, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              img = -1;
              break;
            }
          }
          if (img >= 0) {
            if (d & kDoneStop) {
              img = -2;  // stopped: nothing of this image is read or written
            } else {
              __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
              asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
              // (a folded setup publishes its own stop, below)
              if (!fs && need == 0 && A.st[img].stop) {
                // stopped by the setup (status 8): published as stopped
                __hip_atomic_store((gu32*)(done + img), kDoneStop, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
                img = -2;
              }
            }
          }
        }
      }
      s_img = img;
      s_k = k;
    }
    __syncthreads();
    const int img = s_img;
    const unsigned k = s_k;
    __syncthreads();  // s_img is rewritten by lane 0 only after every wave has read it
    PH_ADD(31, tq);  // dequeue + wait for an image
    if (img == -1) break;
    if (img < 0) continue;
    const ArgRef ar = kernarg_ref();
    if (fs && k == 1) {
      persist_setup<COOP, V>(ar, img);  // the image's first task: its setup
    } else {
      persist_dir<COOP, V>(ar, img);
      __syncthreads();  // rows of d and the direction scalars complete
      persist_col_a<COOP>(ar, img);
      persist_ls<K, MODE, ADAPT, COOP, V, SB>(ar, img);
      __syncthreads();  // the accepted step and AT's columns complete
      persist_bb<COOP, V>(ar, img);
    }
    // hand the image on: every wave's stores drained, then lane 0 releases at
    // agent scope and publishes (sc1 store): ring append, or done[img]
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      const bool stopped = A.st[img].stop != 0;  // lane 0 is bb's (setup's) leader: its own write
      if (use_ring) {
        if (!stopped) {
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          const unsigned t = atomicAdd(queue + 1, 1u);
          __hip_atomic_store((gu64*)(ring + t % nimg),
                             ((unsigned long long)t << 32) | (unsigned)img, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
        }
      } else {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_store((gu32*)(done + img), stopped ? (kDoneStop | k) : k, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
}

// After the persistent solver: an image a timed-out hand-off wait abandoned
// (status bit 4, the tfail word) never reached its stop, so nothing wrote its
// outputs.  Its completed iterations are reported as if it had stopped there
// -- x the current iterate, iters, final beta, the counters with bit 4 -- so
// the host sees the timeout (the phase-kernel path runs such images to MAXIT
// and reports the same bit).  One workgroup per image; stopped images return.
template <class V>
__global__ void __launch_bounds__(kBlock) k_persist_finalize(SolveArgs A) {
  const int img = A.img0 + (int)blockIdx.x;
  ImgState& st = A.st[img];
  if (st.stop) return;
  const int N = A.g.H * A.g.W;
  const Bufs<V> B = slot_bufs<V>(A, img, st.par);
  double* xo = A.out.x + (size_t)img * N;
  for (int i = threadIdx.x; i < N; i += kBlock) xo[i] = (double)B.xa[i] * st.sc;
  __syncthreads();
  if (threadIdx.x == 0) {
    st.status |= 4;
    st.stop = 1;
    A.out.iters[img] = st.iter - 1;
    if (A.out.beta_final) A.out.beta_final[img] = st.beta;
    write_counters(A, st, img, 1);
  }
}

// The persistent kernel for a trial width / objective mode (the same choice as
// ls_kernel); nullptr where no persistent build exists (the phase kernels run).
template <class V, bool COOP = false>
inline const void* persist_kernel(int K, int mode, bool adapt, bool scalar_bkg = false) {
  // the timed workload's combination (general beta, trial width 2, scalar
  // backgrounds) has a build without the per-pixel background operand
  if (!COOP && BSGP_PERSIST_SB && scalar_bkg && !adapt && mode == 3 && K >= 2)
    return (const void*)k_persist<COOP, 2, 3, false, V, true>;
  if (adapt) return (const void*)k_persist<COOP, 1, -1, true, V>;
  if (K > 2) K = 2;
  if (mode == -1) return (const void*)k_persist<COOP, 2, -1, false, V>;
  if (mode == 0) return K == 1 ? (const void*)k_persist<COOP, 1, 0, false, V>
                               : (const void*)k_persist<COOP, 2, 0, false, V>;
  if (mode == 4) return K == 1 ? (const void*)k_persist<COOP, 1, 4, false, V>
                               : (const void*)k_persist<COOP, 2, 4, false, V>;
  return K == 1 ? (const void*)k_persist<COOP, 1, 3, false, V>
                : (const void*)k_persist<COOP, 2, 3, false, V>;
}
template <class V, bool COOP = false>
inline void persist_kernels(std::vector<const void*>& f) {
  for (int adapt = 0; adapt < 2; ++adapt)
    for (int mode : {-1, 0, 3, 4})
      for (int K : {1, 2}) f.push_back(persist_kernel<V, COOP>(K, mode, adapt != 0));
  if (!COOP && BSGP_PERSIST_SB) f.push_back(persist_kernel<V, COOP>(2, 3, false, true));
}
template <class V, bool COOP = false>
inline hipError_t launch_persist_t(const SolveArgs& a, int K, size_t lds, hipStream_t s,
                                   unsigned* queue, unsigned* done, int grid) {
  if (a.prm.stop_criterion >= 2 && a.prm.stop_criterion <= 4)
    hipLaunchKernelGGL(k_ring_init, dim3((a.nimg + 255) / 256), dim3(256), 0, s, queue, a.nimg,
                       a.img0);
  const bsgp_params& P = a.prm;
  const bool adapt = P.adapt_beta && P.variant == BSGP_VARIANT_BETA;
  const bool special = a.in.beta0 ? !P.beta0_general : (P.betaParam == 0.0 || P.betaParam == 1.0);
  const int mode = P.variant == BSGP_VARIANT_KL ? 0 : special ? -1 : P.gn_f32 ? 4 : 3;
  SolveArgs aa = a;
  void* args[] = {&aa, &queue, &done};
  hipError_t e = hipLaunchKernel(persist_kernel<V, COOP>(K, mode, adapt, !a.prm.bkg_is_map), dim3(grid),
                                 dim3(kBlock), args, lds, s);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_persist_finalize<V>, dim3(a.nimg), dim3(kBlock), 0, s, a);
  return hipGetLastError();
}

// ---------------------------------------- kernel: per-iteration tracking
// errflag / save (sgp.py:240-257, 394-396, 416-422): launched after setup
// (it = 0) and after iteration it; for every image whose iteration `it` ran it
// writes the relative error of the scaled iterate against obj/scaling and a
// copy of the iterate (after the update, before any revert).  Off the hot
// kernels: only solves that ask for err / x_iter launch it.
template <class V>
__global__ void __launch_bounds__(kBlock) k_track(SolveArgs A, int it) {
  __shared__ double red[(kWaves + 1) * kMaxRed];
  const int img = A.img0 + (int)blockIdx.x;
  const ImgState& st = A.st[img];
  if (it > 0 && st.iter != it + 1) return;  // iteration `it` did not run for this image
  const int N = A.g.H * A.g.W;
  const Bufs<V> B = slot_bufs<V>(A, img, st.par);
  // k_bb flips `par` when the image goes on; a stopping image keeps it
  const V* x = (it == 0 || !st.stop) ? B.xa : B.xb;
  const int tid = threadIdx.x;
  if (A.out.err) {
    const double* o = A.in.obj + (size_t)img * N;
    double s[2] = {0.0, 0.0};
    for (int i = tid; i < N; i += kBlock) {
      const double ov = o[i] / st.sc;  // obj / scaling (sgp.py:243)
      const double e = x[i] - ov;
      s[0] += e * e;
      s[1] += ov * ov;
    }
    block_sum<2>(s, red);
    if (tid == 0) A.out.err[(size_t)img * (A.prm.MAXIT + 1) + it] = sqrt(s[0] / s[1]);
  }
  if (A.out.x_iter && it > 0) {
    double* d = A.out.x_iter + ((size_t)img * A.prm.MAXIT + (it - 1)) * N;
    for (int i = tid; i < N; i += kBlock) d[i] = x[i];
  }
}

// Kernels come in builds per FFT mode (COOP: workgroup-cooperative transforms
// for long rows/columns) and iterate storage V (double, or float for
// BSGP_STORAGE_F32); separate instantiations keep each build's register
// allocation its own.  Trial widths 4 and 8 exist for the float64
// one-wave-per-transform build only.
template <bool COOP, class V>
inline const void* ls_kernel(int K, int mode, bool adapt) {
  constexpr bool WIDE = !COOP && std::is_same<V, double>::value;
  if (adapt) return (const void*)k_ls<1, -1, true, COOP, V>;
  if (!WIDE && K > 2) K = 2;
  if (mode == 4 && K > 2) K = 2;
  if (mode == -1) return (const void*)k_ls<2, -1, false, COOP, V>;
  if (mode == 4) return K == 1 ? (const void*)k_ls<1, 4, false, COOP, V>
                               : (const void*)k_ls<2, 4, false, COOP, V>;
  if constexpr (WIDE) {
    if (mode == 0 && K == 4) return (const void*)k_ls<4, 0, false, false, double>;
    if (mode == 0 && K == 8) return (const void*)k_ls<8, 0, false, false, double>;
    if (mode == 3 && K == 4) return (const void*)k_ls<4, 3, false, false, double>;
    if (mode == 3 && K == 8) return (const void*)k_ls<8, 3, false, false, double>;
  }
  if (mode == 0) return K == 1 ? (const void*)k_ls<1, 0, false, COOP, V>
                               : (const void*)k_ls<2, 0, false, COOP, V>;
  return K == 1 ? (const void*)k_ls<1, 3, false, COOP, V> : (const void*)k_ls<2, 3, false, COOP, V>;
}

// Team kernels (T > 1 workgroups per image spin on each other) need every
// workgroup of the grid resident at once.  choose_team (bsgp_api.hip) sizes
// teams from the occupancy the runtime reports for every team kernel of the
// plan's build (team_resident_per_cu), so the grid fits the idle device; the
// barrier's bounded spin turns a violation (another tenant holding CUs) into
// status bit 4 instead of a hang.  BSGP_COOP_LAUNCH=1 launches them
// cooperatively instead, which the runtime guarantees but which costs ~17 us
// per launch (C2 -29 %, C4 -6 %, measured A/B).
#ifndef BSGP_COOP_LAUNCH
#define BSGP_COOP_LAUNCH 0
#endif
inline hipError_t launch_fn(const void* f, dim3 grid, size_t lds, hipStream_t s, const SolveArgs& a) {
  void* args[] = {const_cast<SolveArgs*>(&a)};
  if (BSGP_COOP_LAUNCH && a.T > 1)
    return hipLaunchCooperativeKernel(f, grid, dim3(kBlock), args, (unsigned)lds, s);
  return hipLaunchKernel(f, grid, dim3(kBlock), args, lds, s);
}
// k_col (no barrier: a team image's columns are independent)
inline hipError_t launch_fn(const void* f, dim3 grid, size_t lds, hipStream_t s, const SolveArgs& a,
                            int i) {
  void* args[] = {const_cast<SolveArgs*>(&a), &i};
  return hipLaunchKernel(f, grid, dim3(kBlock), args, lds, s);
}

template <bool COOP, class V>
inline hipError_t launch_setup_t(const SolveArgs& a, size_t lds, hipStream_t s) {
  return launch_fn((const void*)k_setup<COOP, V>, dim3(a.nimg * a.T), lds, s, a);
}
template <bool COOP, class V>
inline hipError_t launch_iteration_t(const SolveArgs& a, int K, size_t lds, hipStream_t s,
                                     hipEvent_t* ev) {
  const dim3 grid(a.nimg * a.T), gcol(a.nimg * a.Tc);
  hipError_t e = hipSuccess;
  auto chk = [&](hipError_t r) {
    if (e == hipSuccess) e = r;
  };
  // ev (profiled solves): recorded before k_dir and after every kernel class
  // (dir, col of A, ls, col of AT, bb); a class not launched gets an empty span
  if (ev) chk(hipEventRecord(ev[0], s));
  chk(launch_fn((const void*)k_dir<COOP, V>, grid, lds, s, a));
  if (ev) chk(hipEventRecord(ev[1], s));
  // k_col of a cooperative plan needs only its own groups' buffers (no
  // reduction scratch, no LDS twiddles)
#ifndef BSGP_COL_LDS_FULL
#define BSGP_COL_LDS_FULL 0
#endif
  const size_t lds_col =
      (COOP && !BSGP_COL_LDS_FULL) ? (size_t)a.g.nfc * 2 * a.g.lpad * sizeof(cd) + a.g.tw2 : lds;
  if (!(a.fuse_col & 5)) chk(launch_fn((const void*)k_col<COOP>, gcol, lds_col, s, a, 0));
  if (ev) chk(hipEventRecord(ev[2], s));
  // line-search kernel specialised on trial width, objective mode, adaptivity
  const bsgp_params& P = a.prm;
  const bool adapt = P.adapt_beta && P.variant == BSGP_VARIANT_BETA;
  const bool special = a.in.beta0 ? !P.beta0_general : (P.betaParam == 0.0 || P.betaParam == 1.0);
  const int mode = P.variant == BSGP_VARIANT_KL ? 0 : special ? -1 : P.gn_f32 ? 4 : 3;
  chk(launch_fn(ls_kernel<COOP, V>(K, mode, adapt), grid, lds, s, a));
  if (ev) chk(hipEventRecord(ev[3], s));
  if (!(a.fuse_col & 2)) chk(launch_fn((const void*)k_col<COOP>, gcol, lds_col, s, a, 1));
  if (ev) chk(hipEventRecord(ev[4], s));
  chk(launch_fn((const void*)k_bb<COOP, V>, grid, lds, s, a));
  if (ev) chk(hipEventRecord(ev[5], s));
  return e;
}
template <class V>
inline hipError_t launch_track_t(const SolveArgs& a, int it, hipStream_t s) {
  void* args[] = {const_cast<SolveArgs*>(&a), &it};
  return hipLaunchKernel((const void*)k_track<V>, dim3(a.nimg), dim3(kBlock), args, 0, s);
}

template <bool COOP, class V>
inline void solver_kernels(std::vector<const void*>& f) {
  f.push_back((const void*)k_setup<COOP, V>);
  f.push_back((const void*)k_dir<COOP, V>);
  f.push_back((const void*)k_bb<COOP, V>);
  for (int adapt = 0; adapt < 2; ++adapt)
    for (int mode : {-1, 0, 3, 4})
      for (int K : {1, 2, 4, 8}) f.push_back(ls_kernel<COOP, V>(K, mode, adapt != 0));
}
// Workgroups of every team kernel of a build that one CU holds at once (the
// minimum over the kernels, from hipOccupancyMaxActiveBlocksPerMultiprocessor).
inline hipError_t team_resident(const std::vector<const void*>& fns, size_t lds, int* per_cu) {
  int m = 1 << 30;
  for (const void* f : fns) {
    int n = 0;
    hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, f, kBlock, lds);
    if (e != hipSuccess) return e;
    if (n < m) m = n;
  }
  *per_cu = m;
  return hipSuccess;
}
hipError_t team_resident_per_cu(bool coop, int storage, size_t lds, int* per_cu);

// float32-storage builds (bsgp_solver_f32.hip)
hipError_t launch_setup_f32(const SolveArgs& a, size_t lds, hipStream_t s);
hipError_t launch_iteration_f32(const SolveArgs& a, int K, size_t lds, hipStream_t s,
                                hipEvent_t* ev);
hipError_t launch_track_f32(const SolveArgs& a, int it, hipStream_t s);
void solver_kernels_f32(std::vector<const void*>& f, bool coop);

}  // namespace bsgp
