// bsgp_device.hpp — gfx950 device building blocks of the beta-SGP engine:
// workgroup reductions, the three fused FFT-convolution passes, the
// flux-conserving projection and the divergence terms.
//
// Execution model: one workgroup (kBlock threads) owns one
// image in every phase kernel of its solve.  All scalar control (projectDF's secant,
// Armijo, Barzilai-Borwein, stop rules) is computed redundantly by every
// thread from block-reduced sums, so no thread ever waits for a broadcast and
// no host round trip exists inside a solve.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "bsgp_fft.hpp"
#include "bsgp_math.hpp"

namespace bsgp {

#ifndef BSGP_BLOCK
#define BSGP_BLOCK 256
#endif
constexpr int kBlock = BSGP_BLOCK;  // threads per workgroup (one image per workgroup)
constexpr int kWaves = kBlock / 64;
constexpr int kMaxRed = 24;  // doubles reduced at once

// Team barriers and reductions on per-member words (round 5)
// for teams of at most BSGP_TEAM_FLAGS members: a member's arrival is one
// store to its own word and its reduction partials are their own arrival
// flags (slots pre-filled with kPartEmpty, triple-buffered), so a barrier is
// one store plus the readers' polls instead of the hierarchical counters'
// chain of atomics.  Every member polls every member, so larger teams (C4's
// 256) go through eight group leaders (BSGP_TEAM_HIER) or keep the
// XCD-hierarchical counters; 0 disables the flags (A/B).
#ifndef BSGP_TEAM_FLAGS
#define BSGP_TEAM_FLAGS 64
#endif
#ifndef BSGP_TEAM_HIER
#define BSGP_TEAM_HIER 1
#endif
constexpr int kPartBufs = 3;
// A signalling NaN (hi word == lo word, so hipMemsetD32 can fill it):
// arithmetic never produces one, and stored partials are canonicalised.
constexpr unsigned long long kPartEmpty = 0xFFF75EE0FFF75EE0ull;
constexpr unsigned int kPartEmptyWord = 0xFFF75EE0u;
constexpr int kSharedBytes = 512;  // LDS after the wave partials: reduced totals + scalars

// Phase profile (builds with -DBSGP_PHASE_PROF only): thread 0 of every
// workgroup adds the shader cycles it spent in each phase to g_phase[slot]
// (tools/phase_prof.py reads them through bsgp_phase_prof).  Row passes given
// a slot base PHS >= 0 split their time into operand batches (PHS), FFTs
// (PHS + 1) and spectrum stores / staging (PHS + 2), as seen by wave 0.
constexpr int kPhaseSlots = 32;
#ifdef BSGP_PHASE_PROF
static __device__ unsigned long long g_phase[kPhaseSlots];
#define PH_T(v) const unsigned long long v = __builtin_amdgcn_s_memtime()
#define PH_ADD(slot, t0)                                                                 \
  do {                                                                                   \
    if (threadIdx.x == 0) atomicAdd(&g_phase[slot], __builtin_amdgcn_s_memtime() - (t0)); \
  } while (0)
#define PH_SUB(slot, t)                                                                 \
  do {                                                                                  \
    if (PHS >= 0) {                                                                     \
      const unsigned long long t_ = __builtin_amdgcn_s_memtime();                        \
      if (threadIdx.x == 0) atomicAdd(&g_phase[(slot) < 0 ? 0 : (slot)], t_ - (t));       \
      t = t_;                                                                           \
    }                                                                                   \
  } while (0)
#define PH_SUB_T(v) unsigned long long v = __builtin_amdgcn_s_memtime()
#else
#define PH_T(v)
#define PH_ADD(slot, t0)
#define PH_SUB(slot, t)
#define PH_SUB_T(v)
#endif

// Geometry of one conv plan (P x Q FFT grid, H x W image).
struct Geo {
  int H, W;      // image
  int P, Q;      // FFT grid (circular: P=H, Q=W)
  int Qh;        // stored half spectrum width = Q/2 + 1
  int nfw;       // FFT workers per workgroup, each owning 2 LDS buffers: waves, or in coop
                 // mode thread groups of kBlock/nfw threads
  int nfc;       // FFT workers of the column kernel k_col (coop: may be fewer, for more
                 // workgroups per CU; == nfw otherwise)
  int coop;      // 1: thread groups of the workgroup run the transforms (long rows/columns)
  int lpad;      // complex elements per LDS buffer (odd: spreads banks)
  int sld;       // column stride of the stored half spectrum (>= H, even; BSGP_SPEC_PAD)
  int tw2;       // bytes at the start of dynamic LDS holding two-level twiddle tables
                 // (FftPlan::lds_tw2; cooperative 2048-point plans) and the column
                 // transforms' stage tables (twmix), else 0
  int twmix;     // byte offset of the 2048-point column stage tables (TwMixL), or -1
  FftPlan fp;    // length P (columns)
  FftPlan fq;    // length Q (rows)
  const cd* tfA;   // [Qh][P] transfer function of A, scaled by 1/(P*Q)
  const cd* tfAT;  // [Qh][P] transfer function of AT
  size_t tf_stride;  // per-image PSFs: elements from image i's TF pair to i+1's (0: one PSF)
};

// Transfer function image `img` uses (bsgp_plan_set_psfs gives every image its own).
__device__ __forceinline__ const cd* tf_of(const Geo& G, int img, int transpose) {
  return (transpose ? G.tfAT : G.tfA) + (size_t)img * G.tf_stride;
}

// Copy the twiddle tables of the static-length transforms into their LDS slot
// (plan.lds_tw); the caller's next workgroup barrier publishes them.
__device__ __forceinline__ void copy_tw(const FftPlan& f) {
  if (f.lds_tw < 0) return;
  extern __shared__ __attribute__((aligned(16))) char bsgp_dyn_lds[];
  cd* d = reinterpret_cast<cd*>(bsgp_dyn_lds + f.lds_tw);
  for (int i = threadIdx.x; i < f.n; i += kBlock) d[i] = f.tw[i];
}
// The two-level table (bsgp_fft.hpp Tw2) of a plan that placed one: entries
// of the full global table, w^a (a < 64) then w^(64 b) (b < n/64).
__device__ __forceinline__ void copy_tw2(const FftPlan& f) {
  if (f.lds_tw2 < 0) return;
  extern __shared__ __attribute__((aligned(16))) char bsgp_dyn_lds[];
  cd* d = reinterpret_cast<cd*>(bsgp_dyn_lds + f.lds_tw2);
  const int m = 64 + f.n / 64;
  for (int i = threadIdx.x; i < m; i += blockDim.x) d[i] = f.tw[i < 64 ? i : 64 * (i - 64)];
}
__device__ __forceinline__ void load_tw_lds(const Geo& G) {
  if (G.twmix >= 0) {  // the column transforms' stage tables (TwMixL)
    extern __shared__ __attribute__((aligned(16))) char bsgp_dyn_lds[];
    cd* d = reinterpret_cast<cd*>(bsgp_dyn_lds + G.twmix);
    for (int i = threadIdx.x; i < 64 + 512; i += blockDim.x)
      d[i] = G.fp.tw[i < 64 ? 32 * i : 4 * (i - 64)];
  }
  copy_tw(G.fp);
  if (G.fq.lds_tw != G.fp.lds_tw) copy_tw(G.fq);
  copy_tw2(G.fp);
  if (G.fq.lds_tw2 != G.fp.lds_tw2) copy_tw2(G.fq);
  __syncthreads();
}

// --------------------------------------------------------------- syncs
// LDS hand-off between lanes of ONE wavefront: wait for this wave's LDS ops
// and keep the compiler from moving LDS accesses across the point.
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

struct WaveSync {
  __device__ __forceinline__ void operator()() const { wave_sync(); }
};

// --------------------------------------------------------------- reductions
// v of lane (lane ^ O), every lane of the wave active: xor 1 and 2 by DPP
// quad permutes (VALU, no LDS pipe), xor 4 / 8 / 16 by ds_swizzle's bit mode
// (no address VGPR), xor 32 by ds_bpermute (__shfl_xor).  The same pairing as
// __shfl_xor for every O, so the reduction trees below keep their bits.
#ifndef BSGP_WAVE_DPP
#define BSGP_WAVE_DPP 1
#endif
template <int O>
__device__ __forceinline__ double xor_lanes(double v) {
  if constexpr (BSGP_WAVE_DPP && (O == 1 || O == 2)) {
    constexpr int ctrl = O == 1 ? 0xB1 : 0x4E;  // quad_perm [1,0,3,2] / [2,3,0,1]
    const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), ctrl, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), ctrl, 0xF, 0xF, false);
    return __hiloint2double(hi, lo);
  } else if constexpr (BSGP_WAVE_DPP && O < 32) {
    constexpr int pat = (O << 10) | 0x1F;  // bit mode: and 0x1F, or 0, xor O
    const int lo = __builtin_amdgcn_ds_swizzle(__double2loint(v), pat);
    const int hi = __builtin_amdgcn_ds_swizzle(__double2hiint(v), pat);
    return __hiloint2double(hi, lo);
  } else {
    return __shfl_xor(v, O, 64);
  }
}
__device__ __forceinline__ double wave_sum(double v) {
  v += xor_lanes<32>(v);
  v += xor_lanes<16>(v);
  v += xor_lanes<8>(v);
  v += xor_lanes<4>(v);
  v += xor_lanes<2>(v);
  v += xor_lanes<1>(v);
  return v;
}
template <bool MAX>
__device__ __forceinline__ double wave_ext_step(double v, double u) {
  // NaN propagates like np.max / np.min
  return MAX ? ((u > v || u != u) ? u : v) : ((u < v || u != u) ? u : v);
}
template <bool MAX>
__device__ __forceinline__ double wave_ext(double v) {
  v = wave_ext_step<MAX>(v, xor_lanes<32>(v));
  v = wave_ext_step<MAX>(v, xor_lanes<16>(v));
  v = wave_ext_step<MAX>(v, xor_lanes<8>(v));
  v = wave_ext_step<MAX>(v, xor_lanes<4>(v));
  v = wave_ext_step<MAX>(v, xor_lanes<2>(v));
  v = wave_ext_step<MAX>(v, xor_lanes<1>(v));
  return v;
}
__device__ __forceinline__ double wave_max(double v) { return wave_ext<true>(v); }
__device__ __forceinline__ double wave_min(double v) { return wave_ext<false>(v); }

// Sum NV per-thread values over the workgroup; every thread gets the totals.
// Wave partials go to LDS, thread i < NV adds the kWaves partials of value i
// in a fixed order, and every thread reads the NV totals: deterministic and
// identical in every thread, with only NV LDS reads per thread.
template <int NV>
__device__ __forceinline__ void block_sum(double (&v)[NV], double* red) {
  static_assert(NV <= kMaxRed, "too many values");
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    double s = wave_sum(v[i]);
    if (lane == 0) red[w * kMaxRed + i] = s;
  }
  __syncthreads();
  if (threadIdx.x < NV) {
    const int i = threadIdx.x;
    double s = red[i];
#pragma unroll
    for (int k = 1; k < kWaves; ++k) s += red[k * kMaxRed + i];
    red[kWaves * kMaxRed + i] = s;
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < NV; ++i) v[i] = red[kWaves * kMaxRed + i];
  __syncthreads();
}

__device__ __forceinline__ double block_max(double v, double* red) {
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  v = wave_max(v);
  if (lane == 0) red[w * kMaxRed] = v;
  __syncthreads();
  double s = red[0];
  for (int k = 1; k < kWaves; ++k) {
    double u = red[k * kMaxRed];
    s = (u > s || u != u) ? u : s;
  }
  __syncthreads();
  return s;
}

__device__ __forceinline__ double block_min(double v, double* red) {
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  v = wave_min(v);
  if (lane == 0) red[w * kMaxRed] = v;
  __syncthreads();
  double s = red[0];
  for (int k = 1; k < kWaves; ++k) {
    double u = red[k * kMaxRed];
    s = (u < s || u != u) ? u : s;
  }
  __syncthreads();
  return s;
}

// --------------------------------------------------------------- teams
// A team = T workgroups cooperating on one image (T = 1: one workgroup, no
// global traffic).  Rows (and columns) are strided over the team's waves;
// every reduction is a team reduction: block totals -> per-member partials in
// global memory -> team barrier -> fixed-order sum of the T partials, so all
// members hold bit-identical scalars and run the same control flow.
//
// Two barrier flavours share one arrival counter per image:
//  * team_sync: bulk data hand-off between members (setup only): every
//    storing wave drains, agent-scope release before the arrival, agent-scope
//    acquire after it (cdna_hip_programming.md §6 Guideline 16 recipe);
//  * the reduction barrier inside team_sum / team_max / team_min: only the
//    partials cross workgroups, written and read with sc1 (agent-scope
//    relaxed atomic) accesses, so neither fence is needed.  In the iteration
//    kernels each member streams only the rows it transforms itself, so the
//    partials are the only inter-workgroup data.
typedef __attribute__((address_space(1))) unsigned long long gu64;
typedef __attribute__((address_space(1))) unsigned int gu32;
typedef __attribute__((address_space(1))) int gi32;

// Barrier words of one image (kTeamWords unsigned ints, every word on a
// 128-B line of its own): per group g < 8 an arrival counter and a
// generation word, and one top counter of completed groups.
constexpr int kTeamLine = 32;
constexpr int kTeamWords = 17 * kTeamLine;
// Largest team: flag barriers use words ctr[m] (m < T) and, through the
// group leaders, ctr[T + q] (q < 8); a leader polls its group with one row
// per lane of wave 0 (members q + 8 * lane).  choose_team clamps T to this.
constexpr int kMaxTeam = 512;
static_assert(kMaxTeam + 8 <= kTeamWords, "team barrier words overflow the image's block");
static_assert(kMaxTeam <= 8 * 64, "a group leader polls at most 64 members");

struct Team {
  int m, T;            // member index, team size
  double* part;        // [3][T + 8][kMaxRed] partial slots of this image (+ group sums)
  int flags;           // 1: flag barriers (T <= BSGP_TEAM_FLAGS), 2: via group leaders, 0: counters
  unsigned int* ctr;   // the image's kTeamWords barrier words (monotonic across kernels)
  unsigned int base;   // barriers the team completed before this kernel (same in all members)
  int nb;              // team barriers passed in this kernel
  int* fail;           // set when a barrier spin times out (solve status bit 4)
  int grp, ng, G;      // this member's group (blockIdx % 8), members in it, groups in the team
};

// Work partition of a team.  Waves: row pairs / columns strided by gws from
// gw0.  Pixel streams: T == 1 streams every pair; T > 1 streams only the
// chunks of 2*nfw rows (cp pixel pairs) whose row FFTs this member runs, i.e.
// chunks m, m+T, ...
struct Part {
  int gw0, gws;  // first global FFT-worker index of this workgroup, global worker stride
  int gt0, gts;  // first global thread index, global thread stride (strided loops)
  int m, T, cp;  // member, team size, pixel pairs per row chunk
  int nf;        // FFT workers per workgroup (waves; thread groups in coop mode)
};

__device__ __forceinline__ Part make_part(const Team& t, int nfw, int W) {
  Part d;
  d.gw0 = t.m * nfw;
  d.gws = t.T * nfw;
  d.gt0 = t.m * kBlock;
  d.gts = t.T * kBlock;
  d.m = t.m;
  d.T = t.T;
  d.cp = nfw * W;
  d.nf = nfw;
  return d;
}

__device__ __forceinline__ Part solo_part(int nfw) {
  Part d;
  d.gw0 = 0;
  d.gws = nfw;
  d.gt0 = 0;
  d.gts = kBlock;
  d.m = 0;
  d.T = 1;
  d.cp = 0;
  d.nf = nfw;
  return d;
}

// Lane 0: arrive, then wait for all T members.  XCD-hierarchical
// (MI355X_MICROARCH.md, barrier-xcd): members are grouped by blockIdx % 8 --
// with the runtime's round-robin dispatch, the members on one XCD -- and each
// arrives on its group's counter; the last arriver of a group (told by the
// value its add returns) adds to the team's top counter, waits for all G
// groups there and publishes the barrier's generation to its group, whose
// other members poll only that word.  One top counter sees G <= 8 adds
// instead of T, and no line is polled by more than a group.  The grouping
// is only a speed choice: any placement gives the same barrier.  Bounded
// spins with s_sleep; once any barrier of the solve timed out, later ones
// return at once and the solve ends with status bit 4 instead of hanging.
__device__ __forceinline__ bool team_spin(Team& t, unsigned& spins) {
  __builtin_amdgcn_s_sleep(1);
  ++spins;
  if ((spins & 1023u) == 0 &&
      __hip_atomic_load((gi32*)t.fail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0)
    return false;
  if (spins > (1u << 24)) {
    __hip_atomic_store((gi32*)t.fail, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return false;
  }
  return true;
}
__device__ __forceinline__ void team_arrive_wait(Team& t) {
  const unsigned int n1 = t.base + (unsigned int)t.nb + 1;  // barriers done after this one
  gu32* gc = (gu32*)(t.ctr + t.grp * kTeamLine);
  gu32* gen = (gu32*)(t.ctr + (8 + t.grp) * kTeamLine);
  gu32* top = (gu32*)(t.ctr + 16 * kTeamLine);
  const unsigned int old = __hip_atomic_fetch_add(gc, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  unsigned int spins = 0;
  if (old + 1 == n1 * (unsigned int)t.ng) {  // the group's last arrival
    __hip_atomic_fetch_add(top, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned int target = n1 * (unsigned int)t.G;
    while ((int)(__hip_atomic_load(top, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - target) < 0)
      if (!team_spin(t, spins)) return;
    __hip_atomic_store(gen, n1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  } else {
    while ((int)(__hip_atomic_load(gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - n1) < 0)
      if (!team_spin(t, spins)) return;
  }
}

__device__ __forceinline__ void st_sc1(double* p, double v) {
  __hip_atomic_store((gu64*)p, (unsigned long long)__double_as_longlong(v), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ld_sc1(const double* p) {
  return __longlong_as_double(
      (long long)__hip_atomic_load((gu64*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}

__device__ __forceinline__ bool part_empty(double v) {
  return (unsigned long long)__double_as_longlong(v) == kPartEmpty;
}

// Flag barriers.  Every barrier of a solve (data or reduction) has a global
// number g = base + nb, the same in every member.  Data barrier g: member m
// stores g + 1 to its arrival word ctr[m] after a release and polls every
// member's word.  Reduction g: member m stores its partials to slot g % 3
// (which holds kPartEmpty) and polls every member's partials of that slot
// until none is empty.  After barrier g a member refills its own slot
// (g + 2) % 3, which held barrier g - 1's partials: every member has read
// those, since every member has arrived at g.  The refill completes before
// the member's next arrival (both are wave 0's, behind an s_waitcnt), so no
// member can see a stale partial in a slot it polls.
//
// Large teams (flags == 2) go through eight group leaders: group q holds the
// members m with m % 8 == q and member q leads it.  A leader polls its
// group's partials (arrival words), folds them and stores the group's sums
// (word) in row T + q (word T + q); every member polls the eight group rows
// (words).  Two hops of one store and one poll each instead of T members
// polling T partials.  The group rows are refilled like the members' rows.
__device__ __forceinline__ double* team_slot(const Team& t, unsigned int ahead) {
  return t.part + (size_t)((t.base + (unsigned int)t.nb + ahead) % 3u) * (t.T + 8) * kMaxRed;
}
__device__ __forceinline__ void team_refill(const Team& t) {
  if (threadIdx.x < kMaxRed) {
    double* r = team_slot(t, 2);
    __hip_atomic_store((gu64*)(r + (size_t)t.m * kMaxRed + threadIdx.x), kPartEmpty,
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (t.flags == 2 && t.m < 8)
      __hip_atomic_store((gu64*)(r + (size_t)(t.T + t.m) * kMaxRed + threadIdx.x), kPartEmpty,
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}
// wave 0: until the arrival words w0, w0 + ws, ... (n of them) are >= n1
__device__ __forceinline__ void team_wait_words(Team& t, int w0, int ws, int n, unsigned int n1) {
  unsigned int spins = 0;
  for (;;) {
    bool ok = true;
    for (int k = (int)threadIdx.x; k < n; k += 64)
      ok &= (int)(__hip_atomic_load((gu32*)(t.ctr + w0 + k * ws), __ATOMIC_RELAXED,
                                    __HIP_MEMORY_SCOPE_AGENT) - n1) >= 0;
    if (__all(ok)) return;
    if (!team_spin(t, spins)) return;
  }
}

// Data barrier: everything any member stored before it is visible to every
// member after it.
__device__ __forceinline__ void team_sync(Team& t) {
  if (t.T == 1) {
    __syncthreads();
    return;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (t.flags) {
    if (threadIdx.x < 64) {
      const unsigned int n1 = t.base + (unsigned int)t.nb + 1;
      if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_store((gu32*)(t.ctr + t.m), n1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      if (t.flags == 2) {
        if (t.m < 8) {  // leader: the group's words, then the group's word
          team_wait_words(t, t.m, 8, (t.T - t.m + 7) >> 3, n1);
          if (threadIdx.x == 0)
            __hip_atomic_store((gu32*)(t.ctr + t.T + t.m), n1, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        }
        team_wait_words(t, t.T, 1, 8, n1);
      } else {
        team_wait_words(t, 0, 1, t.T, n1);
      }
      if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      team_refill(t);
    }
  } else if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    team_arrive_wait(t);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  t.nb += 1;
}

// Reduction barrier (counters): thread 0 has stored this member's partials
// with sc1 stores; drain them, arrive, wait.  The partials are then read
// with sc1 loads (no acquire needed: nothing else crosses workgroups here).
// With flag barriers the partials are the arrival: nothing to do here.
__device__ __forceinline__ void team_red_barrier(Team& t) {
  if (t.flags) return;
  if (threadIdx.x == 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    team_arrive_wait(t);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // compiler ordering only
  }
  __syncthreads();
}
// After the totals are read: with flag barriers refill the slot two
// barriers ahead; count the barrier.
__device__ __forceinline__ void team_red_done(Team& t) {
  if (t.flags && threadIdx.x < 64) team_refill(t);
  t.nb += 1;
}
// This barrier's partial slots.
__device__ __forceinline__ double* red_slot(const Team& t) {
  return t.flags ? team_slot(t, 0) : t.part + (size_t)(t.nb & 1) * (t.T + 8) * kMaxRed;
}
// Wave 0's poll over the partials: with flag barriers the loads repeat until
// no partial is empty; otherwise one pass.
__device__ __forceinline__ bool red_poll_done(Team& t, bool ok, unsigned int& spins) {
  if (!t.flags || __all(ok)) return true;
  return !team_spin(t, spins);
}
// Wide flag reductions (more than BSGP_RED_POLL_MAX loads per lane: NV + NM
// values of ceil(T / 64) members): poll one value per member, the last one
// stored, before loading all of them, so a poll round is one load per member.
#ifndef BSGP_RED_POLL_MAX
#define BSGP_RED_POLL_MAX 24
#endif
__device__ __forceinline__ void red_wait_last(Team& t, const double* slot, int last) {
  if (!t.flags || (last + 1) * ((t.T + 63) >> 6) <= BSGP_RED_POLL_MAX) return;
  unsigned int spins = 0;
  for (;;) {
    bool ok = true;
    for (int mm = (int)threadIdx.x; mm < t.T; mm += 64)
      ok &= !part_empty(ld_sc1(slot + (size_t)mm * kMaxRed + last));
    if (red_poll_done(t, ok, spins)) return;
  }
}

// A member's block totals of NV sums and NM maxima, stored straight to its
// partial slot `dst` (T > 1): wave partials to LDS, one barrier, then lane i <
// NV + NM of wave 0 folds value i over the waves in block_sum's / block_max's
// order (the same bits) and stores it.  The totals are not broadcast inside
// the member (only the team totals are), which saves block_sum's and
// block_max's other barriers; the stores are wave 0's, so the reduction
// barrier's drain in thread 0 covers them.
template <int NV, int NM>
__device__ __forceinline__ void member_partials(const double* v, const double* mx, double* red,
                                                double* dst) {
  static_assert(NV + NM <= kMaxRed && NV + NM <= 64, "too many values");
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const double s = wave_sum(v[i]);
    if (lane == 0) red[w * kMaxRed + i] = s;
  }
#pragma unroll
  for (int k = 0; k < NM; ++k) {
    const double s = wave_max(mx[k]);
    if (lane == 0) red[w * kMaxRed + NV + k] = s;
  }
  __syncthreads();
  if (threadIdx.x < NV + NM) {
    const int i = threadIdx.x;
    double s = red[i];
    if (i < NV) {
      for (int k = 1; k < kWaves; ++k) s += red[k * kMaxRed + i];
    } else {
      for (int k = 1; k < kWaves; ++k) {
        const double u = red[k * kMaxRed + i];
        s = (u > s || u != u) ? u : s;
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's refills first (flags)
    if (s != s) s = __longlong_as_double(0x7ff8000000000000ll);  // never kPartEmpty
    st_sc1(dst + i, s);
  }
}

// Wave 0 of a member: poll row `row` of `rows` (when `on`) until none of its
// NV sums and NM maxima is empty; lanes without a row hold 0 / -inf.
template <int NV, int NM>
__device__ __forceinline__ void poll_row(Team& t, const double* rows, int row, bool on,
                                         double* s, double* m) {
  unsigned int spins = 0;
  for (;;) {
    bool ok = true;
#pragma unroll
    for (int i = 0; i < NV; ++i) s[i] = 0.0;
#pragma unroll
    for (int k = 0; k < NM; ++k) m[k] = -INFINITY;
    if (on) {
      const double* q = rows + (size_t)row * kMaxRed;
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        s[i] = ld_sc1(q + i);
        ok &= !part_empty(s[i]);
      }
#pragma unroll
      for (int k = 0; k < NM; ++k) {
        m[k] = ld_sc1(q + NV + k);
        ok &= !part_empty(m[k]);
      }
    }
    if (red_poll_done(t, ok, spins)) return;
  }
}

// NV sums and NM maxima of a large team through its eight group leaders
// (flags == 2; see team_slot): the member's partials to its row, the leader
// folds its group (lane k: member q + 8k) into row T + q, every member folds
// the eight group rows (lane q).  A fixed order, the same in every member.
template <int NV, int NM>
__device__ __forceinline__ void team_reduce_hier(double* v, double* mx, double* red, Team& t) {
  constexpr int NT = NV + NM;
  static_assert(NT >= 1 && NT <= kMaxRed, "too many values");
  double* slot = team_slot(t, 0);
  member_partials<NV, NM>(v, mx, red, slot + (size_t)t.m * kMaxRed);
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    double s[NV + 1], m[NM + 1];
    if (t.m < 8) {
      const int q = t.m;
      poll_row<NV, NM>(t, slot, q + 8 * lane, lane < ((t.T - q + 7) >> 3), s, m);
      double out = 0.0;
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        const double r = __shfl(wave_sum(s[i]), 0, 64);
        if (lane == i) out = r;
      }
#pragma unroll
      for (int k = 0; k < NM; ++k) {
        const double r = __shfl(wave_max(m[k]), 0, 64);
        if (lane == NV + k) out = r;
      }
      if (lane < NT) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's refills first
        if (out != out) out = __longlong_as_double(0x7ff8000000000000ll);  // never kPartEmpty
        st_sc1(slot + (size_t)(t.T + q) * kMaxRed + lane, out);
      }
    }
    poll_row<NV, NM>(t, slot, t.T + lane, lane < 8, s, m);
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const double r = wave_sum(s[i]);
      if (lane == 0) red[kWaves * kMaxRed + i] = r;
    }
#pragma unroll
    for (int k = 0; k < NM; ++k) {
      const double r = wave_max(m[k]);
      if (lane == 0) red[kWaves * kMaxRed + NV + k] = r;
    }
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < NV; ++i) v[i] = red[kWaves * kMaxRed + i];
#pragma unroll
  for (int k = 0; k < NM; ++k) mx[k] = red[kWaves * kMaxRed + NV + k];
  __syncthreads();
  team_red_done(t);
}

// Team sum of NV values: every thread of every member gets the totals.
template <int NV>
__device__ __forceinline__ void team_sum(double (&v)[NV], double* red, Team& t) {
  if (t.T == 1) {
    block_sum<NV>(v, red);
    return;
  }
  if (t.flags == 2) {
    team_reduce_hier<NV, 0>(v, nullptr, red, t);
    return;
  }
  double* slot = red_slot(t);
  const double none[1] = {0.0};
  member_partials<NV, 0>(v, none, red, slot + (size_t)t.m * kMaxRed);
  team_red_barrier(t);
  // wave 0: lane l loads the partials of members l, l+64, ... (all loads in
  // flight at once), then a fixed shuffle tree: same order in every member
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    double s[NV];
    unsigned int spins = 0;
    red_wait_last(t, slot, NV - 1);
    for (;;) {
      bool ok = true;
#pragma unroll
      for (int i = 0; i < NV; ++i) s[i] = 0.0;
      for (int mm = lane; mm < t.T; mm += 64) {
        const double* q = slot + (size_t)mm * kMaxRed;
#pragma unroll
        for (int i = 0; i < NV; ++i) {
          const double u = ld_sc1(q + i);
          ok &= !part_empty(u);
          s[i] += u;
        }
      }
      if (red_poll_done(t, ok, spins)) break;
    }
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const double r = wave_sum(s[i]);
      if (lane == 0) red[kWaves * kMaxRed + i] = r;
    }
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < NV; ++i) v[i] = red[kWaves * kMaxRed + i];
  __syncthreads();
  team_red_done(t);
}

// NV sums and NM maxima in ONE team barrier (NaN propagates through the
// maxima like np.max); the same values as separate team_sum / team_max calls.
// Used where a kernel needs several reductions at the same point: the line
// search's first pass (sums + max|u|), setup's statistics, the scaling-matrix
// bounds (max y and -min y).
template <int NV, int NM>
__device__ __forceinline__ void team_reduce(double (&v)[NV > 0 ? NV : 1], double (&mx)[NM], double* red,
                                            Team& t, int ph = -1) {
  static_assert(NV + NM <= kMaxRed, "too many values");
  if (t.T == 1) {  // sums first, then maxima: the order of team_sum + team_max
    if constexpr (NV > 0) block_sum<NV>(v, red);
#pragma unroll
    for (int k = 0; k < NM; ++k) mx[k] = block_max(mx[k], red);
    return;
  }
  if (t.flags == 2) {
    team_reduce_hier<NV, NM>(v, mx, red, t);
    return;
  }
  double* slot = red_slot(t);
  PH_T(tr0);
  member_partials<NV, NM>(v, mx, red, slot + (size_t)t.m * kMaxRed);
  team_red_barrier(t);
#ifdef BSGP_PHASE_PROF
  // (phase profile: the member's own waves, then the other members)
  const unsigned long long tr1 = __builtin_amdgcn_s_memtime();
  if (ph >= 0 && threadIdx.x == 0) atomicAdd(&g_phase[ph], tr1 - tr0);
#endif
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    double s[NV + 1], m[NM];
    unsigned int spins = 0;
    red_wait_last(t, slot, NV + NM - 1);
    for (;;) {
      bool ok = true;
#pragma unroll
      for (int i = 0; i < NV; ++i) s[i] = 0.0;
#pragma unroll
      for (int k = 0; k < NM; ++k) m[k] = -INFINITY;
      for (int mm = lane; mm < t.T; mm += 64) {
        const double* q = slot + (size_t)mm * kMaxRed;
#pragma unroll
        for (int i = 0; i < NV; ++i) {
          const double u = ld_sc1(q + i);
          ok &= !part_empty(u);
          s[i] += u;
        }
#pragma unroll
        for (int k = 0; k < NM; ++k) {
          const double u = ld_sc1(q + NV + k);
          ok &= !part_empty(u);
          m[k] = (u > m[k] || u != u) ? u : m[k];
        }
      }
      if (red_poll_done(t, ok, spins)) break;
    }
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const double r = wave_sum(s[i]);
      if (lane == 0) red[kWaves * kMaxRed + i] = r;
    }
#pragma unroll
    for (int k = 0; k < NM; ++k) {
      const double r = wave_max(m[k]);
      if (lane == 0) red[kWaves * kMaxRed + NV + k] = r;
    }
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < NV; ++i) v[i] = red[kWaves * kMaxRed + i];
#pragma unroll
  for (int k = 0; k < NM; ++k) mx[k] = red[kWaves * kMaxRed + NV + k];
  __syncthreads();
#ifdef BSGP_PHASE_PROF
  if (ph >= 0 && threadIdx.x == 0) atomicAdd(&g_phase[ph + 1], __builtin_amdgcn_s_memtime() - tr1);
#endif
  team_red_done(t);
}
template <int NV>
__device__ __forceinline__ void team_sum_max(double (&v)[NV], double& mx, double* red, Team& t,
                                             int ph = -1) {
  double m[1] = {mx};
  team_reduce<NV, 1>(v, m, red, t, ph);
  mx = m[0];
}

// Team max / min (NaN propagates, like np.max / np.min)
template <bool MAX>
__device__ __forceinline__ double team_ext(double v, double* red, Team& t) {
  v = MAX ? block_max(v, red) : block_min(v, red);
  if (t.T == 1) return v;
  if (t.flags == 2) {  // min as -max(-v): the same value, NaN propagating
    double m1[1] = {MAX ? v : -v};
    team_reduce_hier<0, 1>(nullptr, m1, red, t);
    return MAX ? m1[0] : -m1[0];
  }
  double* slot = red_slot(t);
  if (threadIdx.x == 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's refills first (flags)
    if (v != v) v = __longlong_as_double(0x7ff8000000000000ll);  // never kPartEmpty
    st_sc1(slot + (size_t)t.m * kMaxRed, v);
  }
  team_red_barrier(t);
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    double s;
    unsigned int spins = 0;
    for (;;) {
      bool ok = true;
      s = MAX ? -INFINITY : INFINITY;
      for (int mm = lane; mm < t.T; mm += 64) {
        const double u = ld_sc1(slot + (size_t)mm * kMaxRed);
        ok &= !part_empty(u);
        s = MAX ? ((u > s || u != u) ? u : s) : ((u < s || u != u) ? u : s);
      }
      if (red_poll_done(t, ok, spins)) break;
    }
    s = MAX ? wave_max(s) : wave_min(s);
    if (lane == 0) red[kWaves * kMaxRed] = s;
  }
  __syncthreads();
  const double r = red[kWaves * kMaxRed];
  __syncthreads();
  team_red_done(t);
  return r;
}
__device__ __forceinline__ double team_max(double v, double* red, Team& t) {
  return team_ext<true>(v, red, t);
}
__device__ __forceinline__ double team_min(double v, double* red, Team& t) {
  return team_ext<false>(v, red, t);
}

// x**a for the divergence terms: fast_exp(a*fast_log(x)) (bsgp_math.hpp).  For the
// exponents of this path (|a| = |beta-1| <~ 1, scaled data so |log x| <~ 20)
// the error is a few ulp at most, at ~1/2.6 the cost of the general pow();
// x <= 0 follows pow for the cases the iteration can produce.
#ifndef BSGP_FAST_EXP
#define BSGP_FAST_EXP 0  // measured: ocml exp is faster at k_ls's occupancy (A/B -2 %)
#endif
__device__ __forceinline__ double fpow(double x, double a) {
#ifdef BSGP_VALU_X2  // diagnostic: twice the pow work, same values
  const double x2 = x + 0.0 * a * x;
  const double r1 = exp(a * fast_log(x));
  const double r2 = exp(a * fast_log(x2));
  return r1 == r2 ? r1 : r2;
#else
  return BSGP_FAST_EXP ? fast_exp(a * fast_log(x)) : exp(a * fast_log(x));
#endif
}

// numpy-like max/min of two scalars (np.max([a, b]): NaN propagates)
__device__ __forceinline__ double np_max2(double a, double b) {
  return (a != a || b != b) ? (a + b) : (a > b ? a : b);
}
__device__ __forceinline__ double np_min2(double a, double b) {
  return (a != a || b != b) ? (a + b) : (a < b ? a : b);
}
// Python builtin max(a, b) / min(a, b): first argument unless the second compares greater/less
__device__ __forceinline__ double py_max2(double a, double b) { return (b > a) ? b : a; }
__device__ __forceinline__ double py_min2(double a, double b) { return (b < a) ? b : a; }

// --------------------------------------------------------------- conv passes
// Spectrum scratch of one image is COLUMN-major: spec[k * ld + p] for stored
// column k < Qh and row p < ld (ld = H: the zero-filled rows H..P-1 of the
// padded grid are never stored).  A column is contiguous, so the column pass
// streams it with coalesced 16-B loads straight into one wave's LDS buffer;
// the row passes write/read (r, r+1) pairs, 32 contiguous bytes per column,
// which the L2 merges across the workgroup's waves (rows 2w.. of wave w).
struct alignas(32) CPair {
  cd a, b;
};

__device__ __forceinline__ void store_pair(cd* col, bool two, bool pair_ok, cd ak, cd bk) {
  if (two && pair_ok) {
    CPair v;
    v.a = ak;
    v.b = bk;
    *reinterpret_cast<CPair*>(col) = v;
  } else {
    col[0] = ak;
    if (two) col[1] = bk;
  }
}

// Memory-level parallelism of the row and column passes: every global load a
// wave needs for one row pair (or column) is issued before any of it is
// used, so a row pair costs about one memory round trip instead of one per
// 64-pixel step.  Operand loads go through a loader lambda `ld(r, j) -> V`
// that only loads; the lambda that uses them (and may store) runs after the
// whole batch is in registers.
constexpr int kJCH = 4;  // pixels per lane per row in one load batch (W <= 256: one batch)
constexpr int kGCH = 3;  // stored spectrum columns per lane in one gather batch (Qh <= 192)
constexpr int kPCH = 5;  // column elements per lane in one batch (P <= 320: one batch)

// Issue the loads of one batch of row pixels j0 + lane + 64u (u < kJCH) of
// rows r and r+1.  Branch-free: a lane past the row end reloads the last
// pixel and a missing row r+1 reloads row r (the values go unused).  A load
// under a condition would end in a join where the compiler waits for every
// outstanding load (s_waitcnt vmcnt(0)), defeating batches kept in flight.
template <int JCH, class LD, class V>
__device__ __forceinline__ void load_rows(LD& ld, int r, bool two, int j0, int lane, int ncols,
                                          V (&v0)[JCH], V (&v1)[JCH]) {
  const int r1 = two ? r + 1 : r;
#pragma unroll
  for (int u = 0; u < JCH; ++u) {
    const int j = min(j0 + lane + 64 * u, ncols - 1);
    v0[u] = ld(r, j);
    v1[u] = ld(r1, j);
  }
}

// ---------------------------------------------------- cooperative passes
// Geo::coop: transforms too long for one wave's share of the LDS (the 2048-point
// rows and columns of config C4, the 400/480-point grids of the application's
// subdivisions) run on the whole workgroup or on thread groups of it.
//
// One group (Part::nf == 1; C4's 2048-point transforms): one row pair or
// column at a time, all kBlock lanes per Stockham stage and a workgroup
// barrier per stage; member m owns row pairs / columns m, m + T, ...
//
// Thread groups (nf = 2 or 4; shorter transforms, bsgp_plan_create): nf groups
// of kBlock/nf threads (whole waves), each with its own pair of LDS buffers,
// run one row pair or column each; all groups take the same steps through the
// same barriers (a group with no row pair left in a step transforms its stale
// buffer and stores nothing).  Worker gw0 + g of the team partition is group
// g.  A 400-point radix-4 stage has 100 butterflies: one transform per
// 512-thread workgroup left 80 % of the lanes idle in every stage and ran the
// row pairs one after the other through the whole latency chain (375^2
// subdivision tiles: 31.3 k -> 58.6 k image-it/s with four groups, A/B).
struct BlockSync {
  __device__ __forceinline__ void operator()() const { __syncthreads(); }
};
constexpr int kCCH = 4;  // elements per thread per load batch


template <class LD, class MK>
__device__ __forceinline__ void coop_row_fwd_1(const Geo& G, const Part& D, int nrows, int ncols,
                                             int ldim, cd* spec, cd* lds, LD& ld, MK& mk) {
  using V = decltype(ld(0, 0));
  const int t = threadIdx.x;
  const bool pair_ok = (ldim & 1) == 0;
  cd* a = lds;
  cd* b = lds + G.lpad;
  for (int r = 2 * D.gw0; r < nrows; r += 2 * D.gws) {
    const bool two = (r + 1) < nrows;
    for (int j0 = 0; j0 < G.Q; j0 += kBlock * kCCH) {
      V v0[kCCH], v1[kCCH];
#pragma unroll
      for (int u = 0; u < kCCH; ++u) {  // clamped, branch-free (load_rows)
        const int j = min(j0 + t + kBlock * u, ncols - 1);
        v0[u] = ld(r, j);
        v1[u] = ld(two ? r + 1 : r, j);
      }
#pragma unroll
      for (int u = 0; u < kCCH; ++u) {
        const int j = j0 + t + kBlock * u;
        if (j < G.Q) {
          double va = 0.0, vb = 0.0;
          if (j < ncols) {
            va = mk(r, j, v0[u]);
            if (two) vb = mk(r + 1, j, v1[u]);
          }
          a[j] = cmk(va, vb);
        }
      }
    }
    __syncthreads();
    cd* Z = fft_wide(a, b, G.fq, false, t, kBlock, BlockSync());
    for (int k = t; k < G.Qh; k += kBlock) {
      cd ak, bk;
      r2c_split(Z, G.Q, k, &ak, &bk);
      store_pair(spec + (size_t)k * ldim + r, two, pair_ok, ak, bk);
    }
    __syncthreads();
  }
}

__device__ __forceinline__ void coop_gather_1(const Geo& G, const cd* spec, int r, bool two, cd* a) {
  const int t = threadIdx.x;
  for (int k0 = 0; k0 < G.Qh; k0 += kBlock * kCCH) {
    cd A[kCCH], B[kCCH];
#pragma unroll
    for (int u = 0; u < kCCH; ++u) {  // clamped, branch-free
      const int k = min(k0 + t + kBlock * u, G.Qh - 1);
      const cd* col = spec + (size_t)k * G.sld + r;
      A[u] = col[0];
      const cd b = col[two ? 1 : 0];
      B[u] = two ? b : cmk(0.0, 0.0);
    }
#pragma unroll
    for (int u = 0; u < kCCH; ++u) {
      const int k = k0 + t + kBlock * u;
      if (k < G.Qh) {
        a[k] = cmk(A[u].x - B[u].y, A[u].y + B[u].x);
        if (k > 0 && G.Q - k >= G.Qh) a[G.Q - k] = cmk(A[u].x + B[u].y, B[u].x - A[u].y);
      }
    }
  }
  __syncthreads();
}

template <class LD, class USE>
__device__ __forceinline__ void coop_row_inv_1(const Geo& G, const Part& D, const cd* spec, cd* lds,
                                             LD& ld, USE& use) {
  using V = decltype(ld(0, 0));
  const int t = threadIdx.x;
  cd* a = lds;
  cd* b = lds + G.lpad;
  for (int r = 2 * D.gw0; r < G.H; r += 2 * D.gws) {
    const bool two = (r + 1) < G.H;
    coop_gather_1(G, spec, r, two, a);
    cd* Z = fft_wide(a, b, G.fq, true, t, kBlock, BlockSync());
    for (int j0 = 0; j0 < G.W; j0 += kBlock * kCCH) {
      V v0[kCCH], v1[kCCH];
#pragma unroll
      for (int u = 0; u < kCCH; ++u) {  // clamped, branch-free
        const int j = min(j0 + t + kBlock * u, G.W - 1);
        v0[u] = ld(r, j);
        v1[u] = ld(two ? r + 1 : r, j);
      }
#pragma unroll
      for (int u = 0; u < kCCH; ++u) {
        const int j = j0 + t + kBlock * u;
        if (j < G.W) {
          const cd z = Z[j];
          use(r, j, z.x, v0[u]);
          if (two) use(r + 1, j, z.y, v1[u]);
        }
      }
    }
    __syncthreads();
  }
}

template <class CP>
__device__ __forceinline__ void coop_row_inv_fwd_1(const Geo& G, const Part& D, cd* spec, cd* lds,
                                                 CP& cp) {
  const int t = threadIdx.x;
  const bool pair_ok = (G.sld & 1) == 0;
  cd* a = lds;
  cd* b = lds + G.lpad;
  for (int r = 2 * D.gw0; r < G.H; r += 2 * D.gws) {
    const bool two = (r + 1) < G.H;
    coop_gather_1(G, spec, r, two, a);
    cd* Z = fft_wide(a, b, G.fq, true, t, kBlock, BlockSync());
    cd* in2 = (Z == a) ? b : a;
    for (int j = t; j < G.Q; j += kBlock) {
      double va = 0.0, vb = 0.0;
      if (j < G.W) {
        const cd z = Z[j];
        va = cp(r, j, z.x);
        if (two) vb = cp(r + 1, j, z.y);
      }
      in2[j] = cmk(va, vb);
    }
    __syncthreads();
    cd* Y = fft_wide(in2, Z, G.fq, false, t, kBlock, BlockSync());
    for (int k = t; k < G.Qh; k += kBlock) {
      cd ak, bk;
      r2c_split(Y, G.Q, k, &ak, &bk);
      store_pair(spec + (size_t)k * G.sld + r, two, pair_ok, ak, bk);
    }
    __syncthreads();
  }
}

// Columns 0 and Q/2 (Q even) of the half spectrum of real rows are real
// sequences (each row's DC and Nyquist terms), and so are their convolved
// columns (the transfer functions of a real kernel are Hermitian along p):
// they share one complex transform pair, z = c0 + i cN in and out, with the
// two spectra split by Hermitian symmetry before the transfer functions
// (r2c_split).  C4's 1025 stored columns then make 1024 transforms, two
// rounds of the column kernel's 512 resident workgroups instead of a third
// round for one leftover column.
#ifndef BSGP_COL_PAIR_NYQ
#define BSGP_COL_PAIR_NYQ 1
#endif
// The column transforms' plan: BSGP_COL_TW2 0 (default) keeps them on the
// global twiddle table, the row passes take the LDS two-level table.  With
// the LDS table the column kernel needed 168 VGPRs (one 512-thread workgroup
// per CU) or spilled at 128; on the global table it keeps two per CU.  C4 A/B
// (profiles/r05/ab_round5.txt): global columns 1802 it/s, LDS columns at 128
// VGPRs 1781, at 168 VGPRs 1770, no LDS table anywhere 1700.
#ifndef BSGP_COL_TW2
#define BSGP_COL_TW2 0
#endif
// (a template flag, not a modified copy of the plan: a copy of FftPlan lived
// in scratch memory and every stage of k_col read its fields from there)
// Column transforms: fft_wide's paths, the 2048-point one reading its
// second and third stages' twiddles from the LDS stage tables (Geo::twmix,
// loaded by load_tw_lds; bitwise the global table's values).
#ifndef BSGP_COL_TWMIX
#define BSGP_COL_TWMIX 1
#endif
// (every cooperative 2048-point plan has the tables: bsgp_plan_create)
__device__ __forceinline__ cd* col_fft(cd* a, cd* b, const Geo& G, bool inv, int t) {
  if constexpr (BSGP_COL_TWMIX && !BSGP_COL_TW2) {
    if (G.fp.n == 2048)
      return fft_run_static<2048, true, true>(a, b, TwMixL{G.twmix, G.fp.tw}, inv, t, kBlock,
                                              BlockSync());
    return fft_run(a, b, G.fp, inv, t, kBlock, BlockSync());
  }
  return fft_wide<BSGP_COL_TW2>(a, b, G.fp, inv, t, kBlock, BlockSync());
}
__device__ __forceinline__ void coop_col_pair_nyq(const Geo& G, cd* spec, const cd* tf, cd* a,
                                                  cd* b) {
  const int t = threadIdx.x;
  cd* c0 = spec;
  cd* cN = spec + (size_t)(G.Qh - 1) * G.sld;
  const cd* t0 = tf;
  const cd* tN = tf + (size_t)(G.Qh - 1) * G.P;
  for (int p0 = 0; p0 < G.P; p0 += kBlock * kCCH) {
    double x0[kCCH], xN[kCCH];
#pragma unroll
    for (int u = 0; u < kCCH; ++u) {  // clamped, branch-free
      const int pc = min(p0 + t + kBlock * u, G.H - 1);
      x0[u] = c0[pc].x;
      xN[u] = cN[pc].x;
    }
#pragma unroll
    for (int u = 0; u < kCCH; ++u) {
      const int p = p0 + t + kBlock * u;
      if (p < G.P) a[p] = p < G.H ? cmk(x0[u], xN[u]) : cmk(0.0, 0.0);
    }
  }
  __syncthreads();
  cd* Z = col_fft(a, b, G, false, t);
  cd* o = (Z == a) ? b : a;
  for (int p = t; p < G.P; p += kBlock) {
    cd A, B;
    r2c_split(Z, G.P, p, &A, &B);
    const cd X = cmul(A, t0[p]), W = cmul(B, tN[p]);
    o[p] = cmk(X.x - W.y, X.y + W.x);  // X + i W
  }
  __syncthreads();
  cd* Y = col_fft(o, Z, G, true, t);
  for (int p = t; p < G.H; p += kBlock) {
    c0[p] = cmk(Y[p].x, 0.0);
    cN[p] = cmk(Y[p].y, 0.0);
  }
  __syncthreads();
}

__device__ __forceinline__ void coop_col_conv_1(const Geo& G, const Part& D, cd* spec, const cd* tf,
                                              cd* lds) {
  const int t = threadIdx.x;
  cd* a = lds;
  cd* b = lds + G.lpad;
  const bool pair = BSGP_COL_PAIR_NYQ && (G.Q % 2) == 0 && G.Qh > 1;
  const int kend = pair ? G.Qh - 1 : G.Qh;
  for (int k = D.gw0; k < kend; k += D.gws) {
    if (pair && k == 0) {
      coop_col_pair_nyq(G, spec, tf, a, b);
      continue;
    }
    cd* col = spec + (size_t)k * G.sld;
    const cd* tk = tf + (size_t)k * G.P;
    for (int p0 = 0; p0 < G.P; p0 += kBlock * kCCH) {
      cd cv[kCCH];
#pragma unroll
      for (int u = 0; u < kCCH; ++u) {  // clamped, branch-free
        const int p = p0 + t + kBlock * u;
        const cd c = col[min(p, G.H - 1)];
        cv[u] = (p < G.H) ? c : cmk(0.0, 0.0);
      }
#pragma unroll
      for (int u = 0; u < kCCH; ++u) {
        const int p = p0 + t + kBlock * u;
        if (p < G.P) a[p] = cv[u];
      }
    }
    __syncthreads();
    cd* Z = col_fft(a, b, G, false, t);
    for (int p0 = 0; p0 < G.P; p0 += kBlock * kCCH) {
      cd tv[kCCH];
#pragma unroll
      for (int u = 0; u < kCCH; ++u) tv[u] = tk[min(p0 + t + kBlock * u, G.P - 1)];
#pragma unroll
      for (int u = 0; u < kCCH; ++u) {
        const int p = p0 + t + kBlock * u;
        if (p < G.P) Z[p] = cmul(Z[p], tv[u]);
      }
    }
    __syncthreads();
    cd* Y = col_fft(Z, (Z == a) ? b : a, G, true, t);
    for (int p = t; p < G.H; p += kBlock) col[p] = Y[p];
    __syncthreads();
  }
}


struct CGrp {
  int g, t, nt;  // group, thread in the group, threads per group
};
__device__ __forceinline__ CGrp coop_grp(int nf) {
  const int nt = kBlock / nf;
  return CGrp{(int)threadIdx.x / nt, (int)threadIdx.x % nt, nt};
}

template <class LD, class MK>
__device__ __forceinline__ void coop_row_fwd_g(const Geo& G, const Part& D, int nrows, int ncols,
                                               int ldim, cd* spec, cd* lds, LD& ld, MK& mk) {
  using V = decltype(ld(0, 0));
  const CGrp c = coop_grp(D.nf);
  const int t = c.t;
  const bool pair_ok = (ldim & 1) == 0;
  cd* a = lds + c.g * 2 * G.lpad;
  cd* b = a + G.lpad;
  for (int r0 = 2 * D.gw0; r0 < nrows; r0 += 2 * D.gws) {
    const int r = r0 + 2 * c.g;
    const bool act = r < nrows;  // uniform in the group
    const bool two = (r + 1) < nrows;
    PH_T(tq0);
    if (act) {
      for (int j0 = 0; j0 < G.Q; j0 += c.nt * kCCH) {
        V v0[kCCH], v1[kCCH];
#pragma unroll
        for (int u = 0; u < kCCH; ++u) {  // clamped, branch-free (load_rows)
          const int j = min(j0 + t + c.nt * u, ncols - 1);
          v0[u] = ld(r, j);
          v1[u] = ld(two ? r + 1 : r, j);
        }
#pragma unroll
        for (int u = 0; u < kCCH; ++u) {
          const int j = j0 + t + c.nt * u;
          if (j < G.Q) {
            double va = 0.0, vb = 0.0;
            if (j < ncols) {
              va = mk(r, j, v0[u]);
              if (two) vb = mk(r + 1, j, v1[u]);
            }
            a[j] = cmk(va, vb);
          }
        }
      }
    }
    __syncthreads();
    PH_ADD(27, tq0);
    PH_T(tq1);
    cd* Z = fft_wide(a, b, G.fq, false, t, c.nt, BlockSync());
    PH_ADD(26, tq1);
    PH_T(tq2);
    if (act) {
      for (int k = t; k < G.Qh; k += c.nt) {
        cd ak, bk;
        r2c_split(Z, G.Q, k, &ak, &bk);
        store_pair(spec + (size_t)k * ldim + r, two, pair_ok, ak, bk);
      }
    }
    __syncthreads();
    PH_ADD(28, tq2);
  }
}

// The full-length spectrum of row pair (r, r+1) from the stored half spectra
// into `a` (the group's threads); no barrier.
__device__ __forceinline__ void coop_gather_g(const Geo& G, const cd* spec, int r, bool two, cd* a,
                                              const CGrp& c) {
  const int t = c.t;
  for (int k0 = 0; k0 < G.Qh; k0 += c.nt * kCCH) {
    cd A[kCCH], B[kCCH];
#pragma unroll
    for (int u = 0; u < kCCH; ++u) {  // clamped, branch-free
      const int k = min(k0 + t + c.nt * u, G.Qh - 1);
      const cd* col = spec + (size_t)k * G.sld + r;
      A[u] = col[0];
      const cd b = col[two ? 1 : 0];
      B[u] = two ? b : cmk(0.0, 0.0);
    }
#pragma unroll
    for (int u = 0; u < kCCH; ++u) {
      const int k = k0 + t + c.nt * u;
      if (k < G.Qh) {
        a[k] = cmk(A[u].x - B[u].y, A[u].y + B[u].x);
        if (k > 0 && G.Q - k >= G.Qh) a[G.Q - k] = cmk(A[u].x + B[u].y, B[u].x - A[u].y);
      }
    }
  }
}

template <class LD, class USE>
__device__ __forceinline__ void coop_row_inv_g(const Geo& G, const Part& D, const cd* spec,
                                               cd* lds, LD& ld, USE& use) {
  using V = decltype(ld(0, 0));
  const CGrp c = coop_grp(D.nf);
  const int t = c.t;
  cd* a = lds + c.g * 2 * G.lpad;
  cd* b = a + G.lpad;
  for (int r0 = 2 * D.gw0; r0 < G.H; r0 += 2 * D.gws) {
    const int r = r0 + 2 * c.g;
    const bool act = r < G.H;
    const bool two = (r + 1) < G.H;
    PH_T(tq0);
    if (act) coop_gather_g(G, spec, r, two, a, c);
    __syncthreads();
    PH_ADD(25, tq0);
    PH_T(tq1);
    cd* Z = fft_wide(a, b, G.fq, true, t, c.nt, BlockSync());
    PH_ADD(26, tq1);
    PH_T(tq2);
    if (act) {
      for (int j0 = 0; j0 < G.W; j0 += c.nt * kCCH) {
        V v0[kCCH], v1[kCCH];
#pragma unroll
        for (int u = 0; u < kCCH; ++u) {  // clamped, branch-free
          const int j = min(j0 + t + c.nt * u, G.W - 1);
          v0[u] = ld(r, j);
          v1[u] = ld(two ? r + 1 : r, j);
        }
#pragma unroll
        for (int u = 0; u < kCCH; ++u) {
          const int j = j0 + t + c.nt * u;
          if (j < G.W) {
            const cd z = Z[j];
            use(r, j, z.x, v0[u]);
            if (two) use(r + 1, j, z.y, v1[u]);
          }
        }
      }
    }
    __syncthreads();
    PH_ADD(27, tq2);
  }
}

template <class CP>
__device__ __forceinline__ void coop_row_inv_fwd_g(const Geo& G, const Part& D, cd* spec, cd* lds,
                                                   CP& cp) {
  const CGrp c = coop_grp(D.nf);
  const int t = c.t;
  const bool pair_ok = (G.sld & 1) == 0;
  cd* a = lds + c.g * 2 * G.lpad;
  cd* b = a + G.lpad;
  for (int r0 = 2 * D.gw0; r0 < G.H; r0 += 2 * D.gws) {
    const int r = r0 + 2 * c.g;
    const bool act = r < G.H;
    const bool two = (r + 1) < G.H;
    PH_T(tq0);
    if (act) coop_gather_g(G, spec, r, two, a, c);
    __syncthreads();
    PH_ADD(25, tq0);
    PH_T(tq1);
    cd* Z = fft_wide(a, b, G.fq, true, t, c.nt, BlockSync());
    cd* in2 = (Z == a) ? b : a;
    if (act) {
      for (int j = t; j < G.Q; j += c.nt) {
        double va = 0.0, vb = 0.0;
        if (j < G.W) {
          const cd z = Z[j];
          va = cp(r, j, z.x);
          if (two) vb = cp(r + 1, j, z.y);
        }
        in2[j] = cmk(va, vb);
      }
    }
    __syncthreads();
    cd* Y = fft_wide(in2, Z, G.fq, false, t, c.nt, BlockSync());
    PH_ADD(26, tq1);
    PH_T(tq2);
    if (act) {
      for (int k = t; k < G.Qh; k += c.nt) {
        cd ak, bk;
        r2c_split(Y, G.Q, k, &ak, &bk);
        store_pair(spec + (size_t)k * G.sld + r, two, pair_ok, ak, bk);
      }
    }
    __syncthreads();
    PH_ADD(28, tq2);
  }
}

__device__ __forceinline__ void coop_col_conv_g(const Geo& G, const Part& D, cd* spec,
                                                const cd* tf, cd* lds) {
  const CGrp c = coop_grp(D.nf);
  const int t = c.t;
  cd* a = lds + c.g * 2 * G.lpad;
  cd* b = a + G.lpad;
  for (int k0 = D.gw0; k0 < G.Qh; k0 += D.gws) {
    const int k = k0 + c.g;
    const bool act = k < G.Qh;
    cd* col = spec + (size_t)k * G.sld;
    const cd* tk = tf + (size_t)k * G.P;
    PH_T(tq0);
    if (act) {
      for (int p0 = 0; p0 < G.P; p0 += c.nt * kCCH) {
        cd cv[kCCH];
#pragma unroll
        for (int u = 0; u < kCCH; ++u) {  // clamped, branch-free
          const int p = p0 + t + c.nt * u;
          const cd v = col[min(p, G.H - 1)];
          cv[u] = (p < G.H) ? v : cmk(0.0, 0.0);
        }
#pragma unroll
        for (int u = 0; u < kCCH; ++u) {
          const int p = p0 + t + c.nt * u;
          if (p < G.P) a[p] = cv[u];
        }
      }
    }
    __syncthreads();
    PH_ADD(29, tq0);
    PH_T(tq1);
    cd* Z = fft_wide<BSGP_COL_TW2>(a, b, G.fp, false, t, c.nt, BlockSync());
    if (act) {
      for (int p0 = 0; p0 < G.P; p0 += c.nt * kCCH) {
        cd tv[kCCH];
#pragma unroll
        for (int u = 0; u < kCCH; ++u) tv[u] = tk[min(p0 + t + c.nt * u, G.P - 1)];
#pragma unroll
        for (int u = 0; u < kCCH; ++u) {
          const int p = p0 + t + c.nt * u;
          if (p < G.P) Z[p] = cmul(Z[p], tv[u]);
        }
      }
    }
    __syncthreads();
    cd* Y = fft_wide<BSGP_COL_TW2>(Z, (Z == a) ? b : a, G.fp, true, t, c.nt, BlockSync());
    if (act)
      for (int p = t; p < G.H; p += c.nt) col[p] = Y[p];
    __syncthreads();
    PH_ADD(30, tq1);
  }
}

// one group: the whole-workgroup passes; groups: the grouped ones
template <class LD, class MK>
__device__ __forceinline__ void coop_row_fwd(const Geo& G, const Part& D, int nrows, int ncols,
                                             int ldim, cd* spec, cd* lds, LD& ld, MK& mk) {
  if (D.nf == 1)
    coop_row_fwd_1(G, D, nrows, ncols, ldim, spec, lds, ld, mk);
  else
    coop_row_fwd_g(G, D, nrows, ncols, ldim, spec, lds, ld, mk);
}
template <class LD, class USE>
__device__ __forceinline__ void coop_row_inv(const Geo& G, const Part& D, const cd* spec, cd* lds,
                                             LD& ld, USE& use) {
  if (D.nf == 1)
    coop_row_inv_1(G, D, spec, lds, ld, use);
  else
    coop_row_inv_g(G, D, spec, lds, ld, use);
}
template <class CP>
__device__ __forceinline__ void coop_row_inv_fwd(const Geo& G, const Part& D, cd* spec, cd* lds,
                                                 CP& cp) {
  if (D.nf == 1)
    coop_row_inv_fwd_1(G, D, spec, lds, cp);
  else
    coop_row_inv_fwd_g(G, D, spec, lds, cp);
}
__device__ __forceinline__ void coop_col_conv(const Geo& G, const Part& D, cd* spec, const cd* tf,
                                              cd* lds) {
  if (D.nf == 1)
    coop_col_conv_1(G, D, spec, tf, lds);
  else
    coop_col_conv_g(G, D, spec, tf, lds);
}

// row_fwd2: for every pair of image rows (r, r+1) one wave FFTs z = a + i b
// (a, b real rows of length ncols zero-padded to Q) and stores the two half
// spectra into column-major spec with leading dimension ld (>= nrows).
// The input pixel is mk(r, j, ld(r, j)) (fused producer).
// PF: the first operand batch of the wave's next row pair is issued before
// the FFT of the current one (its latency hides under the FFT; the batch
// registers stay live across it).
// PIPE: the operand batch j0 + 64*JCH is issued before batch j0 is computed
// (two batches in flight per wave instead of one round trip per batch; costs
// a second set of batch registers outside the FFT).
template <int JCH = kJCH, bool PF = false, bool COMP = BSGP_FFT_COMPOSITE, bool COOP = false,
          bool PIPE = false, int PHS = -1, class LD, class MK>
__device__ __forceinline__ void row_fwd2(const Geo& G, const Part& D, int nrows, int ncols,
                                         int ldim, cd* spec, cd* lds, LD&& ld, MK&& mk) {
  if constexpr (COOP) {
    coop_row_fwd(G, D, nrows, ncols, ldim, spec, lds, ld, mk);
    return;
  }
  using V = decltype(ld(0, 0));
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const bool pair_ok = (ldim & 1) == 0;
  if (w < G.nfw) {
    cd* a = lds + w * 2 * G.lpad;
    cd* b = a + G.lpad;
    int r = 2 * (D.gw0 + w);
    V v0[JCH], v1[JCH];
    if (PF && r < nrows) load_rows<JCH>(ld, r, (r + 1) < nrows, 0, lane, ncols, v0, v1);
    PH_SUB_T(tph);
    for (; r < nrows; r += 2 * D.gws) {
      const bool two = (r + 1) < nrows;
      auto put = [&](int j0, const V (&w0)[JCH], const V (&w1)[JCH]) __attribute__((always_inline)) {
#pragma unroll
        for (int u = 0; u < JCH; ++u) {
          const int j = j0 + lane + 64 * u;
          if (j < G.Q) {
            double va = 0.0, vb = 0.0;
            if (j < ncols) {
              va = mk(r, j, w0[u]);
              if (two) vb = mk(r + 1, j, w1[u]);
            }
            a[j] = cmk(va, vb);
          }
        }
      };
      if constexpr (PIPE) {
        constexpr int S = 64 * JCH;
        V u0[JCH], u1[JCH];
        if (!PF) load_rows<JCH>(ld, r, two, 0, lane, ncols, v0, v1);
        // (loads past the row end are clamped, not skipped: a skipped load
        // would be a branch whose join waits for every load in flight)
        for (int j0 = 0; j0 < G.Q; j0 += 2 * S) {
          // (no loads for batches wholly in the zero padding, j >= ncols)
          if (j0 + S < ncols) load_rows<JCH>(ld, r, two, j0 + S, lane, ncols, u0, u1);
          put(j0, v0, v1);
          if (j0 + S < G.Q) {
            if (j0 + 2 * S < ncols) load_rows<JCH>(ld, r, two, j0 + 2 * S, lane, ncols, v0, v1);
            put(j0 + S, u0, u1);
          }
        }
      } else {
        for (int j0 = 0; j0 < G.Q; j0 += 64 * JCH) {
          // batches wholly in the zero padding (j0 >= ncols: the 256..269 of a
          // 270-point row) load nothing: put() writes zeros there
          if ((!PF || j0 > 0) && j0 < ncols) load_rows<JCH>(ld, r, two, j0, lane, ncols, v0, v1);
          put(j0, v0, v1);
        }
      }
      const int rn = r + 2 * D.gws;
      if (PF && rn < nrows) load_rows<JCH>(ld, rn, (rn + 1) < nrows, 0, lane, ncols, v0, v1);
      wave_sync();
      PH_SUB(PHS, tph);
      cd* Z = fft_any<COMP>(a, b, G.fq, false, lane, 64, WaveSync());
      PH_SUB(PHS + 1, tph);
      for (int k = lane; k < G.Qh; k += 64) {
        cd ak, bk;
        r2c_split(Z, G.Q, k, &ak, &bk);
        store_pair(spec + (size_t)k * ldim + r, two, pair_ok, ak, bk);
      }
      wave_sync();
      PH_SUB(PHS + 2, tph);
    }
  }
}

// row_fwd: producer form, `prod(r, j)` returns the input pixel.
template <bool COOP = false, class Prod>
__device__ __forceinline__ void row_fwd(const Geo& G, const Part& D, int nrows, int ncols, int ldim,
                                        cd* spec, cd* lds, Prod&& prod) {
  row_fwd2<kJCH, false, BSGP_FFT_COMPOSITE, COOP>(G, D, nrows, ncols, ldim, spec, lds, prod,
                                                  [](int, int, double v) { return v; });
}

// Rebuild the full-length spectrum of row pair (r, r+1) into `a`: each
// stored column k < Qh is loaded once and yields Z_k and Z_{Q-k}.
__device__ __forceinline__ void gather_pair(const Geo& G, const cd* spec, int ld, int r, bool two,
                                            cd* a, int lane) {
  for (int k0 = lane; k0 < G.Qh; k0 += 64 * kGCH) {
    cd A[kGCH], B[kGCH];
#pragma unroll
    for (int u = 0; u < kGCH; ++u) {  // clamped, branch-free
      const int k = min(k0 + 64 * u, G.Qh - 1);
      const cd* col = spec + (size_t)k * ld + r;
      A[u] = col[0];
      const cd bk = col[two ? 1 : 0];
      B[u] = two ? bk : cmk(0.0, 0.0);
    }
#pragma unroll
    for (int u = 0; u < kGCH; ++u) {
      const int k = k0 + 64 * u;
      if (k < G.Qh) {
        a[k] = cmk(A[u].x - B[u].y, A[u].y + B[u].x);
        if (k > 0 && G.Q - k >= G.Qh) a[G.Q - k] = cmk(A[u].x + B[u].y, B[u].x - A[u].y);
      }
    }
  }
}

// LDS-DMA staging of one row pair's stored spectrum: F[k] = spec[k][r] and
// F[Qh + k] = spec[k][r + 1] for k < Qh (global_load_lds_dwordx4: the LDS
// destination is the wave-uniform base + 16 B * lane).  Needs lpad >= 2*Qh.
typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) void gbl_void_t;
__device__ __forceinline__ void stage_pair(const Geo& G, const cd* spec, int ld, int r, bool two,
                                           cd* F, int lane) {
  for (int k0 = 0; k0 < G.Qh; k0 += 64) {
    const int k = k0 + lane;
    if (k < G.Qh) {
      const cd* col = spec + (size_t)k * ld + r;
      __builtin_amdgcn_global_load_lds((gbl_void_t*)col, (lds_void_t*)(F + k0), 16, 0, 0);
      if (two)
        __builtin_amdgcn_global_load_lds((gbl_void_t*)(col + 1), (lds_void_t*)(F + G.Qh + k0), 16,
                                         0, 0);
    }
  }
}
// Full-length spectrum of the staged pair into `a` (as gather_pair).
__device__ __forceinline__ void unpack_pair(const Geo& G, const cd* F, bool two, cd* a, int lane) {
  for (int k = lane; k < G.Qh; k += 64) {
    const cd A = F[k];
    const cd B = two ? F[G.Qh + k] : cmk(0.0, 0.0);
    a[k] = cmk(A.x - B.y, A.y + B.x);
    if (k > 0 && G.Q - k >= G.Qh) a[G.Q - k] = cmk(A.x + B.y, B.x - A.y);
  }
}

// row_inv2: inverse row transforms; use(r, j, value, ld(r, j)) consumes each
// output pixel (j < W) of rows [0, H).  The 1/(P*Q) scale is folded into the
// TF.  Software pipeline per wave: while row pair r is consumed, the stored
// spectrum of the wave's next row pair streams into the buffer the FFT of r
// left free (LDS-DMA), so its latency overlaps the operand loads and the
// consumer of r; the first pair is gathered through registers.
// PRE: the first operand batch is issued before the FFT (costs its registers
// across the FFT).
// PIPE: as row_fwd2 (batch j0 + 64*JCH in flight while batch j0 is consumed).
template <bool PRE, int JCH = kJCH, bool COMP = BSGP_FFT_COMPOSITE, bool COOP = false,
          bool PIPE = false, int PHS = -1, class LD, class USE>
__device__ __forceinline__ void row_inv2(const Geo& G, const Part& D, const cd* spec, cd* lds,
                                         LD&& ld, USE&& use) {
  if constexpr (COOP) {
    coop_row_inv(G, D, spec, lds, ld, use);
    return;
  }
  using V = decltype(ld(0, 0));
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (w < G.nfw) {
    cd* in = lds + w * 2 * G.lpad;
    cd* other = in + G.lpad;
    int r = 2 * (D.gw0 + w);
    PH_SUB_T(tph);
    if (r < G.H) gather_pair(G, spec, G.sld, r, (r + 1) < G.H, in, lane);
    for (; r < G.H; r += 2 * D.gws) {
      const bool two = (r + 1) < G.H;
      V v0[JCH], v1[JCH];
      if (PRE) load_rows<JCH>(ld, r, two, 0, lane, G.W, v0, v1);
      wave_sync();
      PH_SUB(PHS + 2, tph);
      cd* Z = fft_any<COMP>(in, other, G.fq, true, lane, 64, WaveSync());
      PH_SUB(PHS + 1, tph);
      cd* F = (Z == in) ? other : in;
      const int rn = r + 2 * D.gws;
      const bool next = rn < G.H, two_n = (rn + 1) < G.H;
      if (next) stage_pair(G, spec, G.sld, rn, two_n, F, lane);
      auto eat = [&](int j0, const V (&w0)[JCH], const V (&w1)[JCH]) __attribute__((always_inline)) {
#pragma unroll
        for (int u = 0; u < JCH; ++u) {
          const int j = j0 + lane + 64 * u;
          if (j < G.W) {
            const cd z = Z[j];
            use(r, j, z.x, w0[u]);
            if (two) use(r + 1, j, z.y, w1[u]);
          }
        }
      };
      if constexpr (PIPE) {
        constexpr int S = 64 * JCH;
        V u0[JCH], u1[JCH];
        if (!PRE) load_rows<JCH>(ld, r, two, 0, lane, G.W, v0, v1);
        for (int j0 = 0; j0 < G.W; j0 += 2 * S) {
          load_rows<JCH>(ld, r, two, j0 + S, lane, G.W, u0, u1);  // clamped (see row_fwd2)
          eat(j0, v0, v1);
          if (j0 + S < G.W) {
            load_rows<JCH>(ld, r, two, j0 + 2 * S, lane, G.W, v0, v1);
            eat(j0 + S, u0, u1);
          }
        }
      } else {
        for (int j0 = 0; j0 < G.W; j0 += 64 * JCH) {
          if (!PRE || j0 > 0) load_rows<JCH>(ld, r, two, j0, lane, G.W, v0, v1);
          eat(j0, v0, v1);
        }
      }
      PH_SUB(PHS, tph);
      if (next) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // staged pair landed
        wave_sync();                                       // and Z fully consumed
        unpack_pair(G, F, two_n, Z, lane);
        in = Z;
        other = F;
      }
    }
    wave_sync();
  }
}

// row_inv: consumer form, `cons(r, j, value)` (loads, if any, inside).
template <bool COOP = false, class Cons>
__device__ __forceinline__ void row_inv(const Geo& G, const Part& D, const cd* spec, cd* lds,
                                        Cons&& cons) {
  row_inv2<false, kJCH, BSGP_FFT_COMPOSITE, COOP>(
      G, D, spec, lds, [](int, int) { return 0; },
      [&](int r, int j, double v, int) { cons(r, j, v); });
}

// row_inv_fwd: inverse rows of one convolution, then (same rows, same wave)
// forward rows of the next one: `cp(r, j, value)` consumes the output pixel
// and returns the next convolution's input pixel.  The spectrum is updated in
// place (only this wave touches rows r, r+1).
template <bool COOP = false, class CP>
__device__ __forceinline__ void row_inv_fwd(const Geo& G, const Part& D, cd* spec, cd* lds,
                                            CP&& cp) {
  if constexpr (COOP) {
    coop_row_inv_fwd(G, D, spec, lds, cp);
    return;
  }
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const bool pair_ok = (G.sld & 1) == 0;
  if (w < G.nfw) {
    cd* a = lds + w * 2 * G.lpad;
    cd* b = a + G.lpad;
    for (int r = 2 * (D.gw0 + w); r < G.H; r += 2 * D.gws) {
      const bool two = (r + 1) < G.H;
      gather_pair(G, spec, G.sld, r, two, a, lane);
      wave_sync();
      cd* Z = fft_any(a, b, G.fq, true, lane, 64, WaveSync());
      cd* in2 = (Z == a) ? b : a;
      for (int j = lane; j < G.Q; j += 64) {
        double va = 0.0, vb = 0.0;
        if (j < G.W) {
          const cd z = Z[j];
          va = cp(r, j, z.x);
          if (two) vb = cp(r + 1, j, z.y);
        }
        in2[j] = cmk(va, vb);
      }
      wave_sync();
      cd* Y = fft_any(in2, Z, G.fq, false, lane, 64, WaveSync());
      for (int k = lane; k < G.Qh; k += 64) {
        cd ak, bk;
        r2c_split(Y, G.Q, k, &ak, &bk);
        store_pair(spec + (size_t)k * G.sld + r, two, pair_ok, ak, bk);
      }
      wave_sync();
    }
  }
}

// measured on C3 (A/B): the TF loaded after the forward FFT keeps k_col at
// 111 VGPRs (4 waves/SIMD) and runs 8 % faster than batching it with the column
#ifndef BSGP_COL_TFPRE
#define BSGP_COL_TFPRE false
#endif
// col_conv: every wave owns whole columns: it streams stored column k
// (contiguous, H rows) into its LDS buffer, zero-fills rows H..P-1, runs the
// forward P-point FFT, multiplies by tf[k][:], runs the inverse FFT and
// writes rows [0, H) back.  No workgroup barrier inside the pass.
template <bool COOP = false>
__device__ __forceinline__ void col_conv(const Geo& G, const Part& D, cd* spec, const cd* tf,
                                         cd* lds) {
  if constexpr (COOP) {
    coop_col_conv(G, D, spec, tf, lds);
    return;
  }
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (w < G.nfw) {
    cd* a = lds + w * 2 * G.lpad;
    cd* b = a + G.lpad;
    // column and TF loads in one batch before the forward FFT (the TF stays
    // in registers across it), or the TF loaded after the FFT
    const bool one = BSGP_COL_TFPRE && G.P <= 64 * kPCH;
    for (int k = D.gw0 + w; k < G.Qh; k += D.gws) {
      cd* col = spec + (size_t)k * G.sld;
      const cd* t = tf + (size_t)k * G.P;
      cd tv[kPCH];
      for (int p0 = 0; p0 < G.P; p0 += 64 * kPCH) {
        cd cv[kPCH];
#pragma unroll
        for (int u = 0; u < kPCH; ++u) {
          // branch-free (a conditional load ends in a join that waits for every
          // load in flight): clamp the index, select after the load
          const int p = p0 + lane + 64 * u;
          const cd c = col[min(p, G.H - 1)];
          cv[u] = p < G.H ? c : cmk(0.0, 0.0);
          if (one) tv[u] = t[min(p, G.P - 1)];
        }
#pragma unroll
        for (int u = 0; u < kPCH; ++u) {
          const int p = p0 + lane + 64 * u;
          if (p < G.P) a[p] = cv[u];
        }
      }
      wave_sync();
      cd* Z = fft_any(a, b, G.fp, false, lane, 64, WaveSync());
      if (one) {
#pragma unroll
        for (int u = 0; u < kPCH; ++u) {
          const int p = lane + 64 * u;
          if (p < G.P) Z[p] = cmul(Z[p], tv[u]);
        }
      } else if (G.P <= 64 * kPCH) {
        // the TF column in one load batch after the FFT (one round trip)
#pragma unroll
        for (int u = 0; u < kPCH; ++u) tv[u] = t[min(lane + 64 * u, G.P - 1)];
#pragma unroll
        for (int u = 0; u < kPCH; ++u) {
          const int p = lane + 64 * u;
          if (p < G.P) Z[p] = cmul(Z[p], tv[u]);
        }
      } else {
        for (int p = lane; p < G.P; p += 64) Z[p] = cmul(Z[p], t[p]);
      }
      wave_sync();
      cd* Y = fft_any(Z, (Z == a) ? b : a, G.fp, true, lane, 64, WaveSync());
      for (int p = lane; p < G.H; p += 64) col[p] = Y[p];
      wave_sync();
    }
  }
  __syncthreads();
}

// --------------------------------------------------------------- projection
// flux_conserve_proj.projectDF (flux_conserve_proj.py:7-144) for one image:
// find lambda with |sum(x(lambda)) - b| <= 1e-11*b, x(lambda) =
// min(max(0, (c + lambda)/dia), sat/scaling - eps).  `cdf(i, c, dia)` yields the
// per-pixel (c, dia) on the fly.  Returns the final lambda; x(lambda) is
// recomputed by the caller pixel by pixel (same arithmetic, same bits).
struct ProjOut {
  double lam;
  int evals;
  int biter;
  int siter;
};

struct ProjClip {
  bool has_sat;
  double satv;  // ccd_sat_level/scaling - EPSILON
  __device__ __forceinline__ double operator()(double c, double dia, double lam) const {
    double v = (c + lam) / dia;
    v = (0.0 > v) ? 0.0 : v;  // np.maximum(0, v) (NaN stays NaN)
    if (has_sat) v = (satv < v) ? satv : v;  // np.minimum(satv, v)
    return v;
  }
};

template <class CDF>
__device__ __forceinline__ double proj_sum(int N, CDF& cdf, const ProjClip& clip, double lam, double* red) {
  double s[1] = {0.0};
  for (int i = threadIdx.x; i < N; i += kBlock) {
    double c, dia;
    cdf(i, c, dia);
    s[0] += clip(c, dia, lam);
  }
  block_sum<1>(s, red);
  return s[0];
}

// The reference's multiplier search as a stepper: `lam` is the multiplier
// whose sum is wanted next; feed(sum_i x_i(lam)) advances the search and
// returns false once it has finished (result in `lam`).  One evaluation site
// in the caller's loop keeps the (large, fused) evaluation code inlined once.
//   phase 0: first evaluation (:22-28)
//   phase 1: r < 0 bracketing loop (:30-53)
//   phase 2: r > 0 bracketing loop (:55-81), with the np.errstate overflow break
//   phase 3: secant loop (:96-142), including the :122 slip (x assigned, not s)
struct ProjDF {
  static constexpr int kCap = 200000;  // hard bound: the reference's r<0 bracket can spin forever
  double b, tol_r, tol_lam;
  double lam, dlam, laml, lamu, rl, ru, s, r;
  int biter, siter, nev, maxit_s, max_projs, phase;

  __device__ __forceinline__ void init(double b_, double lambda_, double dlambda_, double tol_lam_,
                                       int biter_, int siter_, int max_projs_) {
    b = b_;
    tol_r = 1e-11 * b_;
    tol_lam = tol_lam_;
    lam = lambda_;
    dlam = dlambda_;
    laml = lamu = rl = ru = s = r = 0.0;
    biter = biter_;
    siter = siter_;
    max_projs = max_projs_;
    maxit_s = 0;
    nev = 0;
    phase = 0;
  }
  __device__ __forceinline__ bool finish(double l) {
    lam = l;
    phase = 4;
    return false;
  }
  __device__ __forceinline__ bool secant_start() {
    if (fabs(ru) < tol_r) return finish(lamu);  // :84-88
    if (fabs(rl) < tol_r) return finish(laml);  // :89-93
    s = 1 - rl / ru;                            // :96-102
    dlam = dlam / s;
    lam = lamu - dlam;
    maxit_s = max_projs - biter;
    phase = 3;
    return true;
  }
  __device__ __forceinline__ bool feed(double S) {
    r = S - b;
    ++nev;
    if (phase == 0) {
      if (fabs(r) < tol_r) return finish(lam);
      if (r < 0) {
        laml = lam;
        rl = r;
        lam = lam + dlam;
        phase = 1;
      } else {
        lamu = lam;
        ru = r;
        lam = lam - dlam;
        phase = 2;
      }
      return true;
    }
    if (phase == 1) {
      if (r < 0 && nev < kCap) {
        biter = biter + 1;
        laml = lam;
        s = np_max2(rl / r - 1, 0.1);
        dlam = dlam + dlam / s;
        lam = lam + dlam;
        rl = r;
        return true;
      }
      lamu = lam;
      ru = r;
      return secant_start();
    }
    if (phase == 2) {
      if (r > 0 && nev < kCap) {
        biter = biter + 1;
        lamu = lam;
        s = np_max2(ru / r - 1, 0.1);
        // np.errstate(all='raise') around dlambda_ + dlambda_/s: overflow -> break
        const double q = dlam / s;
        const double nd = dlam + q;
        const bool fin_in = isfinite(dlam) && isfinite(s);
        if (!(fin_in && (!isfinite(q) || !isfinite(nd) || s == 0.0))) {
          dlam = nd;
          lam = lam - dlam;
          ru = r;
          return true;
        }
      }
      laml = lam;
      rl = r;
      return secant_start();
    }
    // phase 3: loop condition, then one secant step
    if (!(fabs(r) > tol_r && dlam > tol_lam * (1 + fabs(lam)) && siter < maxit_s && nev < kCap))
      return finish(lam);
    siter = siter + 1;
    if (r > 0) {
      if (s <= 2) {
        lamu = lam;
        ru = r;
        s = 1 - rl / ru;
        dlam = (lamu - laml) / s;
        lam = lamu - dlam;
      } else {
        s = np_max2(ru / r - 1, 0.1);
        dlam = (lamu - lam) / s;
        const double lam_new = np_max2(lam - dlam, 0.75 * laml + 0.25 * lam);
        lamu = lam;
        ru = r;
        lam = lam_new;
        // flux_conserve_proj.py:122 assigns x, not s: s keeps the value above
      }
    } else {
      if (s >= 2) {
        laml = lam;
        rl = r;
        s = 1 - rl / ru;
        dlam = (lamu - laml) / s;
        lam = lamu - dlam;
      } else {
        s = np_max2(rl / r - 1, 0.1);
        dlam = (lam - laml) / s;
        const double lam_new = np_min2(lam + dlam, 0.75 * lamu + 0.25 * lam);
        laml = lam;
        rl = r;
        lam = lam_new;
        s = (lamu - laml) / (lamu - lam);
      }
    }
    return true;
  }
  __device__ __forceinline__ ProjOut out() const {
    ProjOut o;
    o.lam = lam;
    o.evals = nev;
    o.biter = biter;
    o.siter = siter;
    return o;
  }
};

// `sumf(lambda)` returns sum_i x_i(lambda) over the image (a workgroup
// reduction); every thread runs the identical scalar search.
template <class SUMF>
__device__ __forceinline__ ProjOut project_df_fn(SUMF&& sumf, double b, double lambda_,
                                                 double dlambda_, double tol_lam, int biter,
                                                 int siter, int max_projs) {
  ProjDF pd;
  pd.init(b, lambda_, dlambda_, tol_lam, biter, siter, max_projs);
  while (pd.feed(sumf(pd.lam))) {
  }
  return pd.out();
}


template <class CDF>
__device__ __forceinline__ ProjOut project_df(int N, CDF&& cdf, const ProjClip& clip, double b,
                                              double lambda_, double dlambda_, double tol_lam,
                                              int biter, int siter, int max_projs, double* red) {
  return project_df_fn([&](double lam) { return proj_sum(N, cdf, clip, lam, red); }, b, lambda_,
                       dlambda_, tol_lam, biter, siter, max_projs);
}

// --------------------------------------------------------------- divergences
// Objective of one line-search trial as (up to) three partial sums, combined
// exactly as the reference combines its np.sum calls:
//   KL   (sgp.py:334):      T0 = sum gn*log(gn/den), T1 = sum x_tf_try;  f = T0 + T1 - flux
//   beta=0 (sgp.py:453):    T0 = sum gn/den, T1 = sum log(gn/den);        f = T0 - T1 - N
//   beta=1 (sgp.py:455):    T0 = sum gn*log(gn/den), T1 = sum gn, T2 = sum den;  f = T0 - T1 + T2
//   else  (sgp.py:457-458): T0 = sum s*gn^b, T1 = sum s(b-1)*den^b, T2 = sum s*b*gn*den^(b-1);
//                           f = T0 + T1 - T2
struct Objective {
  int variant;  // 0 KL, 1 beta
  double beta;
  double scal, c1, c2;  // s, s*(b-1), s*b
  int mode;             // 0 KL, 1 beta=0, 2 beta=1, 3 general
  // float32 observed image (params.gn_f32): numpy 1.x evaluates (s*b)*gn as
  // float32(s*b) * gn in float32 before the float64 multiply (sgp.py:458)
  bool f32g = false;
  float c2f = 0.0f;
  __device__ __forceinline__ void set_beta(double b) {
    beta = b;
    if (variant == 0) {
      mode = 0;
    } else if (b == 0.0) {
      mode = 1;
    } else if (b == 1.0) {
      mode = 2;
    } else {
      mode = 3;
      scal = 1 / (b * (b - 1));
      c1 = scal * (b - 1);
      c2 = scal * b;
      c2f = (float)c2;
    }
  }
  // the gn factor of the third sum: (s*b)*gn, or its float32 rounding
  __device__ __forceinline__ double c2g(double gnv) const {
    return f32g ? (double)(c2f * (float)gnv) : c2 * gnv;
  }
  // constant-in-lambda part for one pixel (mode 2: gn; mode 3: s*gn^b)
  __device__ __forceinline__ double konst(double gnv) const {
    if (mode == 2) return gnv;
    if (mode == 3) return scal * fpow(gnv, beta);
    return 0.0;
  }
  // lambda-dependent parts for one pixel with the mode fixed at compile time
  // (MODE < 0: runtime mode)
  template <int MODE>
  __device__ __forceinline__ void terms_m(double xtf_try, double den, double gnv,
                                         double* t) const {
    if constexpr (MODE == 0) {
      t[0] += gnv * fast_log(gnv / den);
      t[1] += xtf_try;
    } else if constexpr (MODE == 3) {
      const double p = fpow(den, beta - 1);
      t[0] += c1 * (den * p);
      t[1] += (c2 * gnv) * p;
    } else if constexpr (MODE == 4) {  // general beta, float32 observed image
      const double p = fpow(den, beta - 1);
      t[0] += c1 * (den * p);
      t[1] += (double)(c2f * (float)gnv) * p;
    } else {
      terms(xtf_try, den, gnv, t);
    }
  }
  // lambda-dependent parts for one pixel: adds to t[0..1]
  __device__ __forceinline__ void terms(double xtf_try, double den, double gnv, double* t) const {
    if (mode == 0) {
      t[0] += gnv * fast_log(gnv / den);
      t[1] += xtf_try;
    } else if (mode == 1) {
      const double q = gnv / den;
      t[0] += q;
      t[1] += fast_log(q);
    } else if (mode == 2) {
      t[0] += gnv * fast_log(gnv / den);
      t[1] += den;
    } else {
      const double p = fpow(den, beta - 1);
      t[0] += c1 * (den * p);
      t[1] += c2g(gnv) * p;
    }
  }
  // f from the constant sum K and the two lambda sums
  __device__ __forceinline__ double combine(double K, double t0, double t1, double flux,
                                            double N) const {
    if (mode == 0) return t0 + t1 - flux;
    if (mode == 1) return t0 - t1 - N;
    if (mode == 2) return t0 - K + t1;
    return K + t0 - t1;
  }
  // gradient numerator w (input of AT) and the first gradient term g1:
  // KL: g = 1 - AT(gn/den)               (sgp.py:263,342)
  // beta: g = den^(b-1) - AT(gn*den^(b-2)) (sgp.py:498-499)
  __device__ __forceinline__ double grad_w(double den, double gnv) const {
    if (variant == 0) return gnv / den;
    return gnv * (fpow(den, beta - 1) / den);
  }
  __device__ __forceinline__ double grad_g1(double den) const {
    if (variant == 0) return 1.0;
    return fpow(den, beta - 1);
  }
};

// d betaDiv / d beta for one pixel (sgp.py:495), y = den, x = gn
__device__ __forceinline__ double beta_deriv_px(double y, double x, double b) {
  const double ly = fast_log(y), lx = fast_log(x);
  const double yb1 = fast_exp((b - 1) * ly);
  const double yb = fast_exp(b * ly);
  const double xb = fast_exp(b * lx);
  double t = -x * yb1 * ly / (b - 1);
  t = t + x * yb1 / ((b - 1) * (b - 1));
  t = t + xb * lx / (b * (b - 1));
  t = t - xb / (b * ((b - 1) * (b - 1)));
  t = t + yb * ly / b;
  t = t - xb / ((b * b) * (b - 1));
  t = t - yb / (b * b);
  return t;
}

// The same for a float32 observed image (params.gn_f32), as numpy 1.x
// evaluates sgp.py:495 with x = gn float32 and y = den float64: the terms in
// x**beta are float32 arrays (x**beta and np.log(x) in float32, their
// product and the divisions by the float64 scalars, cast to float32, rounded
// to float32), the others float64; the seven terms are added left to right,
// each float32 term widened as it is added.
// `xb_out` (optional) receives the float32 power x**beta, which the same
// trial's K = sum(s * x**beta) (float32, numpy's order) needs again.
__device__ __forceinline__ double beta_deriv_px_f32(double y, double x, double b,
                                                    float* xb_out = nullptr) {
  const double ly = fast_log(y);
  const double yb1 = fast_exp((b - 1) * ly);
  const double yb = fast_exp(b * ly);
  const float xf = (float)x;
  const float xb = libm_powf(xf, (float)b);  // x**beta (float32)
  if (xb_out) *xb_out = xb;
  const float lx = libm_logf(xf);            // np.log(x) (float32)
  const float c3 = (float)(b * (b - 1));
  const float c4 = (float)(b * ((b - 1) * (b - 1)));
  const float c6 = (float)((b * b) * (b - 1));
  double t = -x * yb1 * ly / (b - 1);
  t = t + x * yb1 / ((b - 1) * (b - 1));
  t = t + (double)((xb * lx) / c3);
  t = t - (double)(xb / c4);
  t = t + yb * ly / b;
  t = t - (double)(xb / c6);
  t = t - yb / (b * b);
  return t;
}

}  // namespace bsgp
