// bsgp_fft.hpp — mixed-radix Stockham FFT core shared by the gfx950 kernels and
// the host-side unit test (tests/cpp/fft_core_test.cpp).
//
// This replaces numpy's pocketfft calls on the reference hot path:
//   restoration/sgp.py:109,113-115 (circular A/AT: fftn / ifftn of 2-D images)
//   restoration/sgp.py:138,157 -> astropy convolve_fft (linear A/AT, zero-filled)
//
// Design (MI355X-first):
//   * one 1-D transform is owned by ONE 64-lane wavefront and lives in LDS;
//     stages ping-pong between two per-wave LDS buffers, so a stage boundary
//     needs only a wave-level LDS sync, never a workgroup barrier;
//   * radix 2/3/4/5 butterflies are unrolled; any other prime factor goes
//     through a direct O(R^2) DFT stage (needed only for odd stamp sizes such
//     as the 31x31 star stamps of application_sgp_star_stamps.py);
//   * twiddles come from one table tw[k] = exp(-2*pi*i*k/n), k in [0,n),
//     computed once per plan on the host in long double.
//
// The stage formulation is the classic Stockham autosort (decimation in time):
//   for Ns = 1; Ns < n; Ns *= R:   out[(j/Ns)*Ns*R + j%Ns + r*Ns] =
//        DFT_R( in[j + r*n/R] * w^(r*(j%Ns)) ),  w = exp(-2*pi*i/(Ns*R)).
#pragma once

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define BSGP_HD __host__ __device__ __forceinline__
#else
#define BSGP_HD inline
#endif

namespace bsgp {

struct alignas(16) cd {
  double x, y;
};

BSGP_HD cd cmk(double x, double y) { cd r; r.x = x; r.y = y; return r; }
BSGP_HD cd cadd(cd a, cd b) { return cmk(a.x + b.x, a.y + b.y); }
BSGP_HD cd csub(cd a, cd b) { return cmk(a.x - b.x, a.y - b.y); }
BSGP_HD cd cmul(cd a, cd b) { return cmk(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x); }
// a * conj(w)
BSGP_HD cd cmulc(cd a, cd w) { return cmk(a.x * w.x + a.y * w.y, a.y * w.x - a.x * w.y); }
BSGP_HD cd cscale(cd a, double s) { return cmk(a.x * s, a.y * s); }
BSGP_HD cd cconj(cd a) { return cmk(a.x, -a.y); }
// multiply by -i (forward) or +i (inverse)
BSGP_HD cd mul_mi(cd a, bool inv) { return inv ? cmk(-a.y, a.x) : cmk(a.y, -a.x); }

constexpr int kMaxStages = 16;

// One 1-D transform length with its stage radices and twiddle table.
struct FftPlan {
  int n;
  int ns;
  int radix[kMaxStages];
  const cd* tw;  // n entries, exp(-2*pi*i*k/n)
  int lds_tw;    // device: byte offset of a copy of tw in dynamic LDS, or -1
  int lds_tw2;   // device: byte offset of the two-level table (Tw2) in dynamic LDS, or -1
};

// Lengths with a compile-time transform (the hot grid sizes: 256 for circular
// 256^2 images, 270 for 256^2 images with a 25x25 PSF in linear mode, and
// in builds with BSGP_FFT_STATIC_APP -- the persistent solver of
// bsgp_persist_app.hip -- the application's 375^2 / 450^2 subdivisions with
// the 31x31 DIAPL PSF in linear mode: 400 and 480).  Only that build inlines
// them: in every kernel the extra straight-line stages cost C3 0.7 % (A/B).
#ifndef BSGP_FFT_STATIC_APP
#define BSGP_FFT_STATIC_APP 0
#endif
BSGP_HD bool fft_static_len(int n) {
  return n == 256 || n == 270 || (BSGP_FFT_STATIC_APP && (n == 400 || n == 480));
}

BSGP_HD cd tw_at(const cd* tw, int k, bool inv) {
  cd w = tw[k];
  return inv ? cconj(w) : w;
}

// Two-level twiddle table of a length-n transform (n % 64 == 0, n <= 4096):
// t1[a] = w^a (a < 64) and t2[b] = w^(64 b) (b < n/64), both entries of the
// correctly rounded full table, so w^k = t1[k & 63] * t2[k >> 6] -- exact
// where either factor is 1, within ~1 ulp elsewhere.  (64 + n/64) entries
// (1.5 KiB for 2048) fit in LDS beside a workgroup-wide transform's buffers,
// where the full table (32 KiB) does not: the twiddles of every stage come
// from LDS instead of a global-memory round trip per stage.
struct Tw2 {
  const cd* t1;
  const cd* t2;
};
BSGP_HD cd tw_at(const Tw2& t, int k, bool inv) {
  const cd w = cmul(t.t1[k & 63], t.t2[k >> 6]);
  return inv ? cconj(w) : w;
}
template <int STEP, class TW>
BSGP_HD cd tw_step(const TW& tw, int m, bool inv) {
  return tw_at(tw, m * STEP, inv);
}


// ---- unrolled butterflies (forward: w = exp(-2 pi i / R); inverse: conj) ----
BSGP_HD void bfly2(cd* v) {
  cd a = v[0], b = v[1];
  v[0] = cadd(a, b);
  v[1] = csub(a, b);
}

BSGP_HD void bfly3(cd* v, bool inv) {
  const double h = 0.86602540378443864676;  // sin(2 pi / 3)
  cd s = cadd(v[1], v[2]);
  cd d = csub(v[1], v[2]);
  cd t = cmk(v[0].x - 0.5 * s.x, v[0].y - 0.5 * s.y);
  cd u = mul_mi(cscale(d, h), inv);  // -i*h*d (fwd)
  v[0] = cadd(v[0], s);
  v[1] = cadd(t, u);
  v[2] = csub(t, u);
}

BSGP_HD void bfly4(cd* v, bool inv) {
  cd s02 = cadd(v[0], v[2]), d02 = csub(v[0], v[2]);
  cd s13 = cadd(v[1], v[3]), d13 = mul_mi(csub(v[1], v[3]), inv);
  v[0] = cadd(s02, s13);
  v[2] = csub(s02, s13);
  v[1] = cadd(d02, d13);
  v[3] = csub(d02, d13);
}

BSGP_HD void bfly5(cd* v, bool inv) {
  const double c1 = 0.30901699437494742410;   // cos(2 pi / 5)
  const double c2 = -0.80901699437494742410;  // cos(4 pi / 5)
  const double s1 = 0.95105651629515357212;   // sin(2 pi / 5)
  const double s2 = 0.58778525229247312917;   // sin(4 pi / 5)
  cd b1 = cadd(v[1], v[4]), b2 = cadd(v[2], v[3]);
  cd d1 = csub(v[1], v[4]), d2 = csub(v[2], v[3]);
  cd a0 = v[0];
  cd t1 = cmk(a0.x + c1 * b1.x + c2 * b2.x, a0.y + c1 * b1.y + c2 * b2.y);
  cd t2 = cmk(a0.x + c2 * b1.x + c1 * b2.x, a0.y + c2 * b1.y + c1 * b2.y);
  cd u1 = mul_mi(cmk(s1 * d1.x + s2 * d2.x, s1 * d1.y + s2 * d2.y), inv);
  cd u2 = mul_mi(cmk(s2 * d1.x - s1 * d2.x, s2 * d1.y - s1 * d2.y), inv);
  v[0] = cadd(a0, cadd(b1, b2));
  v[1] = cadd(t1, u1);
  v[4] = csub(t1, u1);
  v[2] = cadd(t2, u2);
  v[3] = csub(t2, u2);
}

// exp(-2*pi*i*m/R) (forward) or its conjugate, for the internal twiddles of
// the composite butterflies (R = 6: m = 1, 2; R = 8: m = 1..3; R = 9: m = 1, 2,
// 4; R = 10: m = 1..4).
template <int R>
BSGP_HD cd unit_root(int m, bool inv) {
  double c = 1.0, s = 0.0;
  if (R == 6) {
    c = m == 1 ? 0.5 : -0.5;
    s = 0.86602540378443864676;
  } else if (R == 8) {
    const double h = 0.70710678118654752440;  // sqrt(2)/2
    c = m == 1 ? h : (m == 2 ? 0.0 : -h);
    s = m == 2 ? 1.0 : h;
  } else if (R == 10) {  // m = 1..4
    const double c36 = 0.80901699437494742410, s36 = 0.58778525229247312917;
    const double c72 = 0.30901699437494742410, s72 = 0.95105651629515357212;
    c = m == 1 ? c36 : (m == 2 ? c72 : (m == 3 ? -c72 : -c36));
    s = (m == 1 || m == 4) ? s36 : s72;
  } else if (R == 9) {
    if (m == 1) {
      c = 0.76604444311897803520;
      s = 0.64278760968653932632;
    } else if (m == 2) {
      c = 0.17364817766693034885;
      s = 0.98480775301220805936;
    } else {
      c = -0.93969262078590838405;
      s = 0.34202014332566873304;
    }
  }
  return cmk(c, inv ? s : -s);
}

template <int R>
BSGP_HD void bfly_r(cd* v, bool inv);

// Composite butterfly R = R1*R2 in registers (Cooley-Tukey, n = R2*n1 + n2,
// k = k1 + R1*k2): R2 DFTs of length R1, internal twiddles w_R^(n2*k1), R1
// DFTs of length R2.  One Stockham stage of radix 6 or 9 replaces two stages
// (2*3, 3*3), halving the LDS round trips of those factors.
template <int R1, int R2>
BSGP_HD void bfly_comp(cd* v, bool inv) {
  constexpr int R = R1 * R2;
  cd y[R];
#pragma unroll
  for (int n2 = 0; n2 < R2; ++n2) {
    cd t[R1];
#pragma unroll
    for (int n1 = 0; n1 < R1; ++n1) t[n1] = v[R2 * n1 + n2];
    bfly_r<R1>(t, inv);
#pragma unroll
    for (int k1 = 0; k1 < R1; ++k1) y[n2 * R1 + k1] = t[k1];
  }
#pragma unroll
  for (int n2 = 1; n2 < R2; ++n2)
#pragma unroll
    for (int k1 = 1; k1 < R1; ++k1)
      y[n2 * R1 + k1] = cmul(y[n2 * R1 + k1], unit_root<R>((n2 * k1) % R, inv));
#pragma unroll
  for (int k1 = 0; k1 < R1; ++k1) {
    cd t[R2];
#pragma unroll
    for (int n2 = 0; n2 < R2; ++n2) t[n2] = y[n2 * R1 + k1];
    bfly_r<R2>(t, inv);
#pragma unroll
    for (int k2 = 0; k2 < R2; ++k2) v[k1 + R1 * k2] = t[k2];
  }
}

template <int R>
BSGP_HD void bfly_r(cd* v, bool inv) {
  if constexpr (R == 2) bfly2(v);
  if constexpr (R == 3) bfly3(v, inv);
  if constexpr (R == 4) bfly4(v, inv);
  if constexpr (R == 5) bfly5(v, inv);
  if constexpr (R == 6) bfly_comp<3, 2>(v, inv);
  if constexpr (R == 8) bfly_comp<4, 2>(v, inv);
  if constexpr (R == 9) bfly_comp<3, 3>(v, inv);
  if constexpr (R == 10) bfly_comp<5, 2>(v, inv);
}

// One Stockham stage with a compile-time radix. `lane` in [0, nlanes).
template <int R>
BSGP_HD void stage_fixed(const cd* in, cd* out, int n, int Ns, const cd* tw, bool inv,
                         int lane, int nlanes) {
  const int nb = n / R;
  const int twstep = n / (Ns * R);
  for (int j = lane; j < nb; j += nlanes) {
    const int jm = j % Ns;
    cd v[R];
#pragma unroll
    for (int r = 0; r < R; ++r) v[r] = in[j + r * nb];
    if (Ns > 1) {
#pragma unroll
      for (int r = 1; r < R; ++r) v[r] = cmul(v[r], tw_at(tw, r * jm * twstep, inv));
    }
    if constexpr (R == 2) bfly2(v);
    if constexpr (R == 3) bfly3(v, inv);
    if constexpr (R == 4) bfly4(v, inv);
    if constexpr (R == 5) bfly5(v, inv);
    const int od = (j / Ns) * Ns * R + jm;
#pragma unroll
    for (int r = 0; r < R; ++r) out[od + r * Ns] = v[r];
  }
}

// Direct-DFT stage for any radix R (used for prime factors > 5, e.g. the
// single radix-31 stage of the 31x31 star stamps).  Parallel over the nb*R
// outputs, not over the nb butterflies: with n = R prime there is ONE
// butterfly, and a lane per butterfly left 63 of 64 lanes idle through R^2
// serial multiply-adds.  Each output keeps its summation order (r ascending).
BSGP_HD void stage_generic(const cd* in, cd* out, int n, int R, int Ns, const cd* tw, bool inv,
                           int lane, int nlanes) {
  const int nb = n / R;
  const int twstep = n / (Ns * R);
  const int rstep = n / R;  // tw[m*rstep] = exp(-2 pi i m / R)
#if defined(__HIP_DEVICE_COMPILE__)
  if (nlanes == 64 && 2 * nb * R <= 64) {
    // A stage that fills at most half the wave (a 31-point transform: 31
    // outputs): two lanes per output, one summing the even terms r and one
    // the odd ones, then their partials added (the same sum in both lanes of
    // the pair) -- half the serial chain, and the lanes that sat idle work.
    const int q = lane >> 1, half = lane & 1;
    const bool act = q < nb * R;
    const int k = act ? q / nb : 0, j = act ? q - k * nb : 0;
    const int jm = j % Ns;
    const int od = (j / Ns) * Ns * R + jm;
    const int k2 = (2 * k) % R;
    cd acc = cmk(0.0, 0.0);
    int m = half ? k : 0;  // (r * k) % R
    for (int r = half; r < R; r += 2) {
      cd v = in[j + r * nb];
      if (Ns > 1 && r > 0) v = cmul(v, tw_at(tw, r * jm * twstep, inv));
      acc = cadd(acc, cmul(v, tw_at(tw, m * rstep, inv)));
      m += k2;
      if (m >= R) m -= R;
    }
    acc.x += __shfl_xor(acc.x, 1);
    acc.y += __shfl_xor(acc.y, 1);
    if (act && half == 0) out[od + k * Ns] = acc;
    return;
  }
#endif
  for (int q = lane; q < nb * R; q += nlanes) {
    const int k = q / nb, j = q - k * nb;  // neighbouring lanes: neighbouring butterflies
    const int jm = j % Ns;
    const int od = (j / Ns) * Ns * R + jm;
    cd acc = cmk(0.0, 0.0);
    int m = 0;  // (r * k) % R
    for (int r = 0; r < R; ++r) {
      cd v = in[j + r * nb];
      if (Ns > 1 && r > 0) v = cmul(v, tw_at(tw, r * jm * twstep, inv));
      acc = cadd(acc, cmul(v, tw_at(tw, m * rstep, inv)));
      m += k;
      if (m >= R) m -= R;
    }
    out[od + k * Ns] = acc;
  }
}

BSGP_HD void fft_stage(const cd* in, cd* out, int n, int R, int Ns, const cd* tw, bool inv,
                       int lane, int nlanes) {
  switch (R) {
    case 2: stage_fixed<2>(in, out, n, Ns, tw, inv, lane, nlanes); break;
    case 3: stage_fixed<3>(in, out, n, Ns, tw, inv, lane, nlanes); break;
    case 4: stage_fixed<4>(in, out, n, Ns, tw, inv, lane, nlanes); break;
    case 5: stage_fixed<5>(in, out, n, Ns, tw, inv, lane, nlanes); break;
    default: stage_generic(in, out, n, R, Ns, tw, inv, lane, nlanes); break;
  }
}

// Run all stages of `p` on data in `a` (scratch `b`); returns the buffer that
// holds the result (a or b). `sync()` is called after every stage.
// `tw`: the plan's twiddle table or a copy of it (LDS); null = p.tw.
template <class Sync>
BSGP_HD cd* fft_run(cd* a, cd* b, const FftPlan& p, bool inv, int lane, int nlanes, Sync sync,
                    const cd* tw = nullptr) {
  cd* in = a;
  cd* out = b;
  int Ns = 1;
  if (!tw) tw = p.tw;
  for (int s = 0; s < p.ns; ++s) {
    const int R = p.radix[s];
    fft_stage(in, out, p.n, R, Ns, tw, inv, lane, nlanes);
    sync();
    Ns *= R;
    cd* t = in;
    in = out;
    out = t;
  }
  return in;
}

// ---- two real rows per complex transform -------------------------------------
// Forward: z = a + i*b (a, b real rows of length Q) was transformed to Z.
// Half spectra A_k = (Z_k + conj(Z_{-k}))/2, B_k = -i/2 (Z_k - conj(Z_{-k})).
BSGP_HD void r2c_split(const cd* Z, int Q, int k, cd* A, cd* B) {
  const cd zk = Z[k];
  const cd zm = Z[k == 0 ? 0 : Q - k];
  *A = cmk(0.5 * (zk.x + zm.x), 0.5 * (zk.y - zm.y));
  // Z_k - conj(Z_m) = (p, q);  -i/2 (p + i q) = (q/2, -p/2)
  const double p = zk.x - zm.x, q = zk.y + zm.y;
  *B = cmk(0.5 * q, -0.5 * p);
}

// Inverse: rebuild Z_k = A_k + i B_k over the full length from the stored
// half spectra (k < Qh); for k >= Qh use Hermitian symmetry of A and B.
BSGP_HD cd c2r_gather(const cd* A, const cd* B, int Q, int Qh, int k) {
  if (k < Qh) {
    const cd a = A[k], b = B[k];
    return cmk(a.x - b.y, a.y + b.x);
  }
  const cd a = A[Q - k], b = B[Q - k];
  return cmk(a.x + b.y, b.x - a.y);
}

// ---- compile-time transforms for the hot lengths ----------------------------
// Same Stockham stages, but with n, every radix and every span Ns known at
// compile time: the butterfly loops unroll, j % Ns and j / Ns become shifts or
// constant multiplies, and the stage sequence is straight-line code.
struct RadixList {
  int n;
  int r[kMaxStages];
};

#ifndef BSGP_FFT_COMPOSITE
#define BSGP_FFT_COMPOSITE 1
#endif
// Stage radices of a static transform: 4s, then a 2 paired with a 3 as one
// radix-6 stage, 3s paired as radix-9 stages, the rest, then 5s
// (270 = 6*9*5: three LDS passes instead of five).
// r8: radix-8 stages first (workgroup-wide transforms: 256 lanes, 2048 = 8*8*8*4).
constexpr RadixList factor_radices(int n, bool comp = BSGP_FFT_COMPOSITE, bool r8 = false) {
  RadixList L{0, {}};
  // one wave's 400- / 480-point transforms: three stages whose butterflies
  // fill the 64 lanes in 4 rounds in all (nb = 50, 40, 80 and 60, 80, 48)
  // instead of four radix-4/5/6 stages in 8 rounds
  if (comp && !r8 && n == 400) {
    L.n = 3; L.r[0] = 8; L.r[1] = 10; L.r[2] = 5;
    return L;
  }
  if (comp && !r8 && n == 480) {
    L.n = 3; L.r[0] = 8; L.r[1] = 6; L.r[2] = 10;
    return L;
  }
  int m = n;
  while (r8 && m % 8 == 0) { L.r[L.n++] = 8; m /= 8; }
  while (m % 4 == 0) { L.r[L.n++] = 4; m /= 4; }
  int c2 = 0, c3 = 0;
  while (m % 2 == 0) { ++c2; m /= 2; }
  while (m % 3 == 0) { ++c3; m /= 3; }
  while (comp && c2 > 0 && c3 > 0) { L.r[L.n++] = 6; --c2; --c3; }
  while (comp && c3 >= 2) { L.r[L.n++] = 9; c3 -= 2; }
  while (c2 > 0) { L.r[L.n++] = 2; --c2; }
  while (c3 > 0) { L.r[L.n++] = 3; --c3; }
  while (m % 5 == 0) { L.r[L.n++] = 5; m /= 5; }
  return L;
}

template <int R, int N, int Ns, class TW>
BSGP_HD void stage_static(const cd* in, cd* out, TW tw, bool inv, int lane, int nlanes) {
  constexpr int nb = N / R;
  constexpr int twstep = N / (Ns * R);
#pragma unroll 1
  for (int j0 = 0; j0 < nb; j0 += 64) {
    const int j = j0 + lane;
    if (nlanes == 64 ? (j < nb) : false) {
      const int jm = j % Ns;
      cd v[R];
#pragma unroll
      for (int r = 0; r < R; ++r) v[r] = in[j + r * nb];
      if constexpr (Ns > 1) {
#pragma unroll
        for (int r = 1; r < R; ++r) v[r] = cmul(v[r], tw_step<twstep>(tw, r * jm, inv));
      }
      bfly_r<R>(v, inv);
      const int od = (j / Ns) * Ns * R + jm;
#pragma unroll
      for (int r = 0; r < R; ++r) out[od + r * Ns] = v[r];
    }
  }
  if (nlanes != 64) {  // host test path: serial lanes
    for (int j = lane; j < nb; j += nlanes) {
      const int jm = j % Ns;
      cd v[R];
      for (int r = 0; r < R; ++r) v[r] = in[j + r * nb];
      if (Ns > 1)
        for (int r = 1; r < R; ++r) v[r] = cmul(v[r], tw_step<twstep>(tw, r * jm, inv));
      bfly_r<R>(v, inv);
      const int od = (j / Ns) * Ns * R + jm;
      for (int r = 0; r < R; ++r) out[od + r * Ns] = v[r];
    }
  }
}

template <int N, int S, int Ns, bool COMP, bool R8, class Sync, class TW>
BSGP_HD cd* stages_static(cd* in, cd* out, TW tw, bool inv, int lane, int nlanes,
                          Sync sync) {
  constexpr RadixList L = factor_radices(N, COMP, R8);
  if constexpr (S < L.n) {
    constexpr int R = L.r[S];
    stage_static<R, N, Ns>(in, out, tw, inv, lane, nlanes);
    sync();
    return stages_static<N, S + 1, Ns * R, COMP, R8>(out, in, tw, inv, lane, nlanes, sync);
  } else {
    return in;
  }
}

// Transform of compile-time length N (must be 2/3/5-smooth).  COMP: composite
// radix-6/9 stages (fewer LDS round trips, ~20 more VGPRs live in the stage);
// R8: radix-8 stages first (for 256-lane workgroup transforms).
template <int N, bool COMP = BSGP_FFT_COMPOSITE, bool R8 = false, class Sync, class TW>
BSGP_HD cd* fft_run_static(cd* a, cd* b, TW tw, bool inv, int lane, int nlanes, Sync sync) {
  static_assert(factor_radices(N).n > 0, "N must be 2/3/5-smooth");
  return stages_static<N, 0, 1, COMP, R8>(a, b, tw, inv, lane, nlanes, sync);
}

#if defined(__HIP_DEVICE_COMPILE__)
extern __shared__ __attribute__((aligned(16))) char bsgp_dyn_lds[];
#endif

// Stage tables of the 2048-point radix 8-8-8-4 transform of the cooperative
// column passes (Geo::twmix): its second stage reads the twiddles w^(32 m)
// (m < 64), its third w^(4 m) (m < 512), its last w^k.  The first two come
// from LDS copies of the full table's entries (9 KiB beside the two-level
// tables), the last from the global table: the same values (bitwise equal to
// the global table), one global-memory round trip per transform instead of
// three, and no extra products (the two-level table's product had taken the
// column kernel past 128 VGPRs).
struct TwMixL {
  int off;      // byte offset of the tables in dynamic LDS: [64] w^(32 m), then [512] w^(4 m)
  const cd* g;  // the global table
};
template <int STEP>
BSGP_HD cd tw_step(const TwMixL& t, int m, bool inv) {
#if defined(__HIP_DEVICE_COMPILE__)
  const cd* l = reinterpret_cast<const cd*>(bsgp_dyn_lds + t.off);
  const cd w = STEP == 32 ? l[m] : STEP == 4 ? l[64 + m] : t.g[m * STEP];
#else
  const cd w = t.g[m * STEP];
#endif
  return inv ? cconj(w) : w;
}

// Workgroup-wide transform (all kBlock-style lanes, `sync` = workgroup
// barrier): compile-time radix-8 plan for 2048 (config C4), runtime plan otherwise.
#ifndef BSGP_COOP_TW2
#define BSGP_COOP_TW2 1
#endif
// TW2 false: the global table even where the plan placed the LDS two-level
// table (the column kernel's register budget, bsgp_device.hpp col_tw2).
template <bool TW2 = true, class Sync>
BSGP_HD cd* fft_wide(cd* a, cd* b, const FftPlan& p, bool inv, int lane, int nlanes, Sync sync) {
  if (p.n == 2048) {
#if defined(__HIP_DEVICE_COMPILE__)
    // the two-level table in LDS (bsgp_plan_create places it for every
    // 2048-point plan when BSGP_COOP_TW2; load_tw_lds): a compile-time choice,
    // so the kernels carry one 2048-point transform, not both
    if constexpr (TW2 && BSGP_COOP_TW2) {
      const cd* t = reinterpret_cast<const cd*>(bsgp_dyn_lds + p.lds_tw2);
      return fft_run_static<2048, true, true>(a, b, Tw2{t, t + 64}, inv, lane, nlanes, sync);
    }
#endif
    return fft_run_static<2048, true, true>(a, b, p.tw, inv, lane, nlanes, sync);
  }
  return fft_run(a, b, p, inv, lane, nlanes, sync);
}

// Runtime length with compile-time fast paths for the hot grid sizes.  On the
// device every transform reads its twiddles from the LDS copy the kernel made
// when the plan placed one (plan.lds_tw >= 0; LDS latency instead of L1/L2
// latency in every butterfly round), else the global table.
template <bool COMP = BSGP_FFT_COMPOSITE, class Sync>
BSGP_HD cd* fft_any(cd* a, cd* b, const FftPlan& p, bool inv, int lane, int nlanes, Sync sync) {
#if defined(__HIP_DEVICE_COMPILE__)
  if (p.lds_tw >= 0) {
    const cd* t = reinterpret_cast<const cd*>(bsgp_dyn_lds + p.lds_tw);
    if (p.n == 256) return fft_run_static<256, COMP>(a, b, t, inv, lane, nlanes, sync);
    if (p.n == 270) return fft_run_static<270, COMP>(a, b, t, inv, lane, nlanes, sync);
#if BSGP_FFT_STATIC_APP
    if (p.n == 400) return fft_run_static<400, COMP>(a, b, t, inv, lane, nlanes, sync);
    if (p.n == 480) return fft_run_static<480, COMP>(a, b, t, inv, lane, nlanes, sync);
#endif
    return fft_run(a, b, p, inv, lane, nlanes, sync, t);
  }
#if BSGP_FFT_STATIC_APP
  if (p.n == 400) return fft_run_static<400, COMP>(a, b, p.tw, inv, lane, nlanes, sync);
  if (p.n == 480) return fft_run_static<480, COMP>(a, b, p.tw, inv, lane, nlanes, sync);
#endif
  return fft_run(a, b, p, inv, lane, nlanes, sync);
#else
  switch (p.n) {
    case 256: return fft_run_static<256, COMP>(a, b, p.tw, inv, lane, nlanes, sync);
    case 270: return fft_run_static<270, COMP>(a, b, p.tw, inv, lane, nlanes, sync);
    case 400: return fft_run_static<400, COMP>(a, b, p.tw, inv, lane, nlanes, sync);
    case 480: return fft_run_static<480, COMP>(a, b, p.tw, inv, lane, nlanes, sync);
    default: return fft_run(a, b, p, inv, lane, nlanes, sync);
  }
#endif
}

// Factor n into stage radices: 4s first, then 2, 3, 5, then remaining primes.
// Returns false when n needs more than kMaxStages stages or n < 1.
inline bool plan_radices(int n, int* radix, int* ns) {
  if (n < 1) return false;
  int k = 0;
  int m = n;
  while (m % 4 == 0) { if (k >= kMaxStages) return false; radix[k++] = 4; m /= 4; }
  while (m % 2 == 0) { if (k >= kMaxStages) return false; radix[k++] = 2; m /= 2; }
  while (m % 3 == 0) { if (k >= kMaxStages) return false; radix[k++] = 3; m /= 3; }
  while (m % 5 == 0) { if (k >= kMaxStages) return false; radix[k++] = 5; m /= 5; }
  for (int f = 7; m > 1; f += 2) {
    while (m % f == 0) { if (k >= kMaxStages) return false; radix[k++] = f; m /= f; }
  }
  *ns = k;
  return true;
}

// Smallest 5-smooth integer >= n (scipy.fft.next_fast_len semantics for
// complex transforms, which astropy.convolve_fft uses to size its pad).
inline int next_fast_len(int n) {
  if (n <= 6) return n < 1 ? 1 : n;
  for (int m = n;; ++m) {
    int t = m;
    while (t % 2 == 0) t /= 2;
    while (t % 3 == 0) t /= 3;
    while (t % 5 == 0) t /= 5;
    if (t == 1) return m;
  }
}

}  // namespace bsgp
