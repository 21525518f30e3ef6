// bsgp_solver.hip — the float64-storage builds of the batched beta-SGP phase
// kernels (bsgp_kernels.hpp), the standalone kernels behind include/bsgp.h
// (transfer functions, A/AT, projectDF, betaDiv family) and the dispatch of
// both storage builds.
//
// Reference hot path: restoration/sgp.py:41-438 (sgp, KL) and :506-895
// (sgp_betaDiv), restoration/flux_conserve_proj.py:7-144 (projectDF).
#include <hip/hip_runtime.h>

#include <map>
#include <mutex>
#include <type_traits>
#include <vector>

// pass 1 of the line search also sums the second trial (as in the float64
// persistent build, bsgp_persist.hip: the two stay bitwise equal; the
// cooperative kernels of this unit keep it off, bsgp_kernels.hpp)
#ifndef BSGP_LS1_K2
#define BSGP_LS1_K2 1
#endif
#include "bsgp_kernels.hpp"

namespace bsgp {

hipError_t phase_prof(unsigned long long* out, int n, int reset) {
#ifdef BSGP_PHASE_PROF
  if (n > kPhaseSlots) n = kPhaseSlots;
  hipError_t e = hipDeviceSynchronize();
  if (e == hipSuccess && out) e = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_phase), n * sizeof(unsigned long long));
  if (e == hipSuccess && reset) {
    unsigned long long z[kPhaseSlots] = {};
    e = hipMemcpyToSymbol(HIP_SYMBOL(g_phase), z, sizeof z);
  }
  // the cooperative 512-thread build keeps its own counters: add them
  if (e == hipSuccess && BSGP_COOP512) {
    unsigned long long c[kPhaseSlots] = {};
    e = bsgp_c512_phase_prof(c, n, reset);
    if (e == hipSuccess && out)
      for (int i = 0; i < n; ++i) out[i] += c[i];
  }
  // and so do the persistent solver's translation units
  if (e == hipSuccess) {
    unsigned long long c[kPhaseSlots] = {};
    e = persist_phase_prof(c, n, reset);
    if (e == hipSuccess && out)
      for (int i = 0; i < n; ++i) out[i] += c[i];
  }
  return e;
#else
  (void)out;
  (void)n;
  (void)reset;
  return hipErrorNotSupported;
#endif
}

// --------------------------------------------------------- TF construction
// tf[k][p] = FFT2(kc)[p][k] * scale (optionally conjugated); kc is P x Q real.
// Two launches over many workgroups (blockIdx.y = which kernel grid, for
// per-image PSFs): rows of every grid into the column-major half spectrum
// (ld = P), then the columns.  Cooperative plans transform each row/column
// with the whole workgroup, like the solver's passes.
template <bool COOP>
__global__ void __launch_bounds__(kBlock) tf_rows_kernel(Geo G, const double* kc,
                                                         size_t kc_stride, cd* spec,
                                                         size_t spec_stride) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  cd* lds = reinterpret_cast<cd*>(smem + G.tw2);
  kc += blockIdx.y * kc_stride;
  spec += blockIdx.y * spec_stride;
  load_tw_lds(G);
  Part D = solo_part(G.nfw);
  D.gw0 = blockIdx.x * G.nfw;
  D.gws = gridDim.x * G.nfw;
  row_fwd<COOP>(G, D, G.P, G.Q, G.P, spec, lds, [&](int r, int j) { return kc[r * G.Q + j]; });
}

template <bool COOP>
__global__ void __launch_bounds__(kBlock) tf_cols_kernel(Geo G, const cd* spec,
                                                         size_t spec_stride, cd* tf,
                                                         size_t tf_stride, double scale,
                                                         int conj) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  cd* lds = reinterpret_cast<cd*>(smem + G.tw2);
  spec += blockIdx.y * spec_stride;
  tf += blockIdx.y * tf_stride;
  load_tw_lds(G);
  if constexpr (COOP) {
    // thread groups as the solver's cooperative passes (coop_col_conv)
    const CGrp c = coop_grp(G.nfw);
    cd* a = lds + c.g * 2 * G.lpad;
    cd* b = a + G.lpad;
    for (int k0 = blockIdx.x * G.nfw; k0 < G.Qh; k0 += gridDim.x * G.nfw) {
      const int k = k0 + c.g;
      const bool act = k < G.Qh;
      const cd* col = spec + (size_t)k * G.P;
      if (act)
        for (int p = c.t; p < G.P; p += kBlock / G.nfw) a[p] = col[p];
      __syncthreads();
      cd* Z = fft_wide(a, b, G.fp, false, c.t, kBlock / G.nfw, BlockSync());
      cd* o = tf + (size_t)k * G.P;
      if (act)
        for (int p = c.t; p < G.P; p += kBlock / G.nfw) {
          const cd z = cscale(Z[p], scale);
          o[p] = conj ? cconj(z) : z;
        }
      __syncthreads();
    }
  } else {
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (w >= G.nfw) return;
    cd* a = lds + w * 2 * G.lpad;
    for (int k = blockIdx.x * G.nfw + w; k < G.Qh; k += gridDim.x * G.nfw) {
      const cd* col = spec + (size_t)k * G.P;
      for (int p = lane; p < G.P; p += 64) a[p] = col[p];
      wave_sync();
      cd* Z = fft_any(a, a + G.lpad, G.fp, false, lane, 64, WaveSync());
      cd* o = tf + (size_t)k * G.P;
      for (int p = lane; p < G.P; p += 64) {
        const cd z = cscale(Z[p], scale);
        o[p] = conj ? cconj(z) : z;
      }
      wave_sync();
    }
  }
}

// Per-image PSF stamps [n][kh][kw] -> circularly placed kernels for A and AT
// on the P x Q grid (kc: [n][2][P*Q], zero-filled by the caller), the same
// placement bsgp_plan_create makes on the host (bit-identical values: the
// linear-mode sum is the same serial row-major loop).  sums[b] = sum(psf_b).
__global__ void __launch_bounds__(kBlock) place_psfs_kernel(Geo G, const double* psfs, int kh,
                                                            int kw, int circ, double* kc,
                                                            double* sums) {
  __shared__ double s_sum;
  const double* psf = psfs + (size_t)blockIdx.x * kh * kw;
  const size_t PQ = (size_t)G.P * G.Q;
  double* kA = kc + (size_t)blockIdx.x * 2 * PQ;
  double* kAT = kA + PQ;
  if (threadIdx.x == 0) {
    double s = 0;
    for (int i = 0; i < kh * kw; ++i) s += psf[i];  // sgp.py:97-102 check / astropy normalisation
    s_sum = s;
    sums[blockIdx.x] = s;
  }
  __syncthreads();
  const double s = s_sum;
  for (int e = threadIdx.x; e < kh * kw; e += kBlock) {
    const int u = e / kw, v = e % kw;
    if (circ) {
      // fftshift (sgp.py:109): kA[i][j] = psf[(i - H//2) mod H][(j - W//2) mod W]
      const int i = (u + G.H / 2) % G.H, j = (v + G.W / 2) % G.W;
      kA[(size_t)i * G.W + j] = psf[e];
    } else {
      // kernel/sum centred at k//2; AT: psf.T (sgp.py:157)
      const double val = psf[e] / s;
      const int a = ((u - kh / 2) % G.P + G.P) % G.P, b = ((v - kw / 2) % G.Q + G.Q) % G.Q;
      kA[(size_t)a * G.Q + b] = val;
      const int at = ((v - kw / 2) % G.P + G.P) % G.P, bt = ((u - kh / 2) % G.Q + G.Q) % G.Q;
      kAT[(size_t)at * G.Q + bt] = val;
    }
  }
}

// ------------------------------------------------------ A / AT standalone
template <bool COOP>
__global__ void __launch_bounds__(kBlock) apply_op_kernel(Geo G, int B, int transpose,
                                                          const double* x, double* out,
                                                          cd* specws, size_t spec_stride) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  cd* lds = reinterpret_cast<cd*>(smem + G.tw2);
  const int N = G.H * G.W;
  cd* spec = specws + (size_t)blockIdx.x * spec_stride;
  load_tw_lds(G);
  for (int img = blockIdx.x; img < B; img += gridDim.x) {
    const double* xi = x + (size_t)img * N;
    double* oi = out + (size_t)img * N;
    const Part D = solo_part(G.nfw);
    row_fwd<COOP>(G, D, G.H, G.W, G.sld, spec, lds, [&](int r, int j) { return xi[r * G.W + j]; });
    __syncthreads();
    col_conv<COOP>(G, D, spec, tf_of(G, img, transpose), lds);
    row_inv<COOP>(G, D, spec, lds, [&](int r, int j, double v) { oi[r * G.W + j] = v; });
    __syncthreads();
  }
}

// A / AT for a few large images: three launches over many workgroups per
// image (blockIdx.y = image): rows, columns x TF, inverse rows.
template <bool COOP>
__global__ void __launch_bounds__(kBlock) op_rows_kernel(Geo G, const double* x, cd* specws,
                                                         size_t spec_stride) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  cd* lds = reinterpret_cast<cd*>(smem + G.tw2);
  const double* xi = x + (size_t)blockIdx.y * G.H * G.W;
  Part D = solo_part(G.nfw);
  D.gw0 = blockIdx.x * G.nfw;
  D.gws = gridDim.x * G.nfw;
  load_tw_lds(G);
  row_fwd<COOP>(G, D, G.H, G.W, G.sld, specws + blockIdx.y * spec_stride, lds,
                [&](int r, int j) { return xi[r * G.W + j]; });
}
template <bool COOP>
__global__ void __launch_bounds__(kBlock) op_cols_kernel(Geo G, int transpose, cd* specws,
                                                         size_t spec_stride) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  cd* lds = reinterpret_cast<cd*>(smem + G.tw2);
  Part D = solo_part(G.nfw);
  D.gw0 = blockIdx.x * G.nfw;
  D.gws = gridDim.x * G.nfw;
  load_tw_lds(G);
  col_conv<COOP>(G, D, specws + blockIdx.y * spec_stride, tf_of(G, blockIdx.y, transpose), lds);
}
template <bool COOP>
__global__ void __launch_bounds__(kBlock) op_rows_inv_kernel(Geo G, cd* specws,
                                                             size_t spec_stride, double* out) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  cd* lds = reinterpret_cast<cd*>(smem + G.tw2);
  double* oi = out + (size_t)blockIdx.y * G.H * G.W;
  Part D = solo_part(G.nfw);
  D.gw0 = blockIdx.x * G.nfw;
  D.gws = gridDim.x * G.nfw;
  load_tw_lds(G);
  row_inv<COOP>(G, D, specws + blockIdx.y * spec_stride, lds,
                [&](int r, int j, double v) { oi[r * G.W + j] = v; });
}

// ----------------------------------------------------------- projectDF
__global__ void __launch_bounds__(kBlock) project_df_kernel(int n, double b, const double* c,
                                                            const double* dia, ProjClip clip,
                                                            double lam0, double dlam0,
                                                            double tol_lam, int biter, int siter,
                                                            int max_projs, double* x,
                                                            double* info) {
  __shared__ double red[(kWaves + 1) * kMaxRed];
  ProjOut po = project_df(
      n, [&](int i, double& cc, double& dd) { cc = c[i]; dd = dia[i]; }, clip, b, lam0, dlam0,
      tol_lam, biter, siter, max_projs, red);
  for (int i = threadIdx.x; i < n; i += kBlock) x[i] = clip(c[i], dia[i], po.lam);
  if (threadIdx.x == 0) {
    info[0] = po.lam;
    info[1] = po.evals;
    info[2] = po.biter;
    info[3] = po.siter;
  }
}

// ------------------------------------------------------------ betaDiv family
__global__ void __launch_bounds__(kBlock) beta_div_kernel(int n, const double* y,
                                                          const double* x, double beta,
                                                          double* out) {
  __shared__ double red[(kWaves + 1) * kMaxRed];
  Objective o;
  o.variant = 1;
  o.set_beta(beta);
  double t[3] = {0.0, 0.0, 0.0};
  for (int i = threadIdx.x; i < n; i += kBlock) {
    t[0] += o.konst(x[i]);
    o.terms(y[i], y[i], x[i], &t[1]);
  }
  block_sum<3>(t, red);
  if (threadIdx.x == 0) out[0] = o.combine(t[0], t[1], t[2], 0.0, (double)n);
}

__global__ void beta_div_deriv_kernel(int64_t n, const double* y, const double* x, double beta,
                                      double* out) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    out[i] = beta_deriv_px(y[i], x[i], beta);
}

__global__ void grad_parts_kernel(int64_t n, const double* den, const double* gn, double beta,
                                  double* pow1, double* w) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    pow1[i] = pow(den[i], beta - 1);
    w[i] = gn[i] * pow(den[i], beta - 2);
  }
}

// ----------------------------------------------------------- launchers
// Kernels come in two builds: per-wave transforms (COOP = false) and, for long
// rows/columns (Geo::coop), workgroup-cooperative ones; separate instantiations
// keep each build's register allocation its own.
// ----------------------------------------------------------- launchers
hipError_t launch_setup(const SolveArgs& a, size_t lds, hipStream_t s) {
  if (a.g.coop && BSGP_COOP512) return bsgp_c512_launch_setup(&a, lds, s);
  if (a.storage == BSGP_STORAGE_F32) return launch_setup_f32(a, lds, s);
  return a.g.coop ? launch_setup_t<true, double>(a, lds, s) : launch_setup_t<false, double>(a, lds, s);
}
hipError_t launch_iteration(const SolveArgs& a, int K, size_t lds, hipStream_t s, hipEvent_t* ev) {
  if (a.g.coop && BSGP_COOP512) return bsgp_c512_launch_iteration(&a, K, lds, s, ev);
  if (a.storage == BSGP_STORAGE_F32) return launch_iteration_f32(a, K, lds, s, ev);
  return a.g.coop ? launch_iteration_t<true, double>(a, K, lds, s, ev)
                  : launch_iteration_t<false, double>(a, K, lds, s, ev);
}
hipError_t team_resident_per_cu(bool coop, int storage, size_t lds, int* per_cu) {
  if (coop && BSGP_COOP512) return bsgp_c512_team_resident(storage, lds, per_cu);
  std::vector<const void*> fns;
  if (storage == BSGP_STORAGE_F32)
    solver_kernels_f32(fns, coop);
  else if (coop)
    solver_kernels<true, double>(fns);
  else
    solver_kernels<false, double>(fns);
  return team_resident(fns, lds, per_cu);
}
hipError_t launch_track(const SolveArgs& a, int it, hipStream_t s) {
  if (a.storage == BSGP_STORAGE_F32) return launch_track_f32(a, it, s);
  return launch_track_t<double>(a, it, s);
}
hipError_t launch_build_tf(const Geo& g, const double* kc, cd* spec, cd* tf, double scale,
                           int conj, size_t lds, hipStream_t s) {
  return launch_build_tfs(g, 1, kc, 0, spec, 0, tf, 0, scale, conj, lds, s);
}
// grid.x: workgroups per kernel grid, enough to cover the rows / columns
// once the n grids share the device (the two launches are stream-ordered).
hipError_t launch_build_tfs(const Geo& g, int n, const double* kc, size_t kc_stride, cd* spec,
                            size_t spec_stride, cd* tf, size_t tf_stride, double scale, int conj,
                            size_t lds, hipStream_t s) {
  const int slots = 1024;  // ~resident workgroups of the device
  int per = slots / n;
  if (per < 1) per = 1;
  const int rp = (g.P + 1) / 2;  // row pairs
  const int nr = (rp + g.nfw - 1) / g.nfw, nc = (g.Qh + g.nfw - 1) / g.nfw;
  const dim3 gr(per < nr ? per : nr, n), gc(per < nc ? per : nc, n);
  if (g.coop) {
    hipLaunchKernelGGL((tf_rows_kernel<true>), gr, dim3(kBlock), lds, s, g, kc, kc_stride, spec,
                       spec_stride);
    hipLaunchKernelGGL((tf_cols_kernel<true>), gc, dim3(kBlock), lds, s, g, spec, spec_stride, tf,
                       tf_stride, scale, conj);
  } else {
    hipLaunchKernelGGL((tf_rows_kernel<false>), gr, dim3(kBlock), lds, s, g, kc, kc_stride, spec,
                       spec_stride);
    hipLaunchKernelGGL((tf_cols_kernel<false>), gc, dim3(kBlock), lds, s, g, spec, spec_stride,
                       tf, tf_stride, scale, conj);
  }
  return hipGetLastError();
}
hipError_t launch_place_psfs(const Geo& g, int n, const double* psfs, int kh, int kw, int circ,
                             double* kc, double* sums, hipStream_t s) {
  hipLaunchKernelGGL(place_psfs_kernel, dim3(n), dim3(kBlock), 0, s, g, psfs, kh, kw, circ, kc,
                     sums);
  return hipGetLastError();
}
hipError_t launch_apply_op(const Geo& g, int B, int transpose, const double* x, double* out,
                           cd* specws, size_t spec_stride, int grid, size_t lds, hipStream_t s) {
  if (g.coop)
    hipLaunchKernelGGL((apply_op_kernel<true>), dim3(grid), dim3(kBlock), lds, s, g, B, transpose,
                       x, out, specws, spec_stride);
  else
    hipLaunchKernelGGL((apply_op_kernel<false>), dim3(grid), dim3(kBlock), lds, s, g, B, transpose,
                       x, out, specws, spec_stride);
  return hipGetLastError();
}
template <bool COOP>
static void launch_apply_split_t(const Geo& g, int B, int transpose, const double* x, double* out,
                                 cd* specws, size_t spec_stride, int per, size_t lds,
                                 hipStream_t s) {
  const int rp = (g.H + 1) / 2;
  const int nr = (rp + g.nfw - 1) / g.nfw, nc = (g.Qh + g.nfw - 1) / g.nfw;
  const dim3 gr(per < nr ? per : nr, B), gc(per < nc ? per : nc, B);
  hipLaunchKernelGGL((op_rows_kernel<COOP>), gr, dim3(kBlock), lds, s, g, x, specws, spec_stride);
  hipLaunchKernelGGL((op_cols_kernel<COOP>), gc, dim3(kBlock), lds, s, g, transpose, specws,
                     spec_stride);
  hipLaunchKernelGGL((op_rows_inv_kernel<COOP>), gr, dim3(kBlock), lds, s, g, specws,
                     spec_stride, out);
}
hipError_t launch_apply_op_split(const Geo& g, int B, int transpose, const double* x,
                                 double* out, cd* specws, size_t spec_stride, int per, size_t lds,
                                 hipStream_t s) {
  if (g.coop)
    launch_apply_split_t<true>(g, B, transpose, x, out, specws, spec_stride, per, lds, s);
  else
    launch_apply_split_t<false>(g, B, transpose, x, out, specws, spec_stride, per, lds, s);
  return hipGetLastError();
}
hipError_t launch_project_df(int n, double b, const double* c, const double* dia, ProjClip clip,
                             double lam0, double dlam0, double tol_lam, int biter, int siter,
                             int max_projs, double* x, double* info, hipStream_t s) {
  hipLaunchKernelGGL(project_df_kernel, dim3(1), dim3(kBlock), 0, s, n, b, c, dia, clip, lam0,
                     dlam0, tol_lam, biter, siter, max_projs, x, info);
  return hipGetLastError();
}
hipError_t launch_beta_div(int n, const double* y, const double* x, double beta, double* out,
                           hipStream_t s) {
  hipLaunchKernelGGL(beta_div_kernel, dim3(1), dim3(kBlock), 0, s, n, y, x, beta, out);
  return hipGetLastError();
}
hipError_t launch_beta_div_deriv(int64_t n, const double* y, const double* x, double beta,
                                 double* out, hipStream_t s) {
  const int grid = (int)((n + 255) / 256 < 4096 ? (n + 255) / 256 : 4096);
  hipLaunchKernelGGL(beta_div_deriv_kernel, dim3(grid > 0 ? grid : 1), dim3(256), 0, s, n, y, x,
                     beta, out);
  return hipGetLastError();
}
hipError_t launch_grad_parts(int64_t n, const double* den, const double* gn, double beta,
                             double* pow1, double* w, hipStream_t s) {
  const int grid = (int)((n + 255) / 256 < 4096 ? (n + 255) / 256 : 4096);
  hipLaunchKernelGGL(grad_parts_kernel, dim3(grid > 0 ? grid : 1), dim3(256), 0, s, n, den, gn,
                     beta, pow1, w);
  return hipGetLastError();
}
// The dynamic-LDS limit is a per-function attribute shared by every plan: it
// only ever rises (per device), so creating a plan with a short transform
// after one with a long transform cannot lower the limit the first one's
// launches need.
hipError_t set_solver_lds_limit(size_t bytes) {
  static std::mutex mu;
  static std::map<int, size_t> applied;
  int dev = 0;
  hipError_t ge = hipGetDevice(&dev);
  if (ge != hipSuccess) return ge;
  std::lock_guard<std::mutex> lock(mu);
  if (applied[dev] >= bytes) return hipSuccess;
  std::vector<const void*> fns = {
      (const void*)k_col<false>, (const void*)k_col<true>,
      (const void*)apply_op_kernel<false>, (const void*)apply_op_kernel<true>,
      (const void*)tf_rows_kernel<false>, (const void*)tf_rows_kernel<true>,
      (const void*)tf_cols_kernel<false>, (const void*)tf_cols_kernel<true>,
      (const void*)op_rows_kernel<false>, (const void*)op_rows_kernel<true>,
      (const void*)op_cols_kernel<false>, (const void*)op_cols_kernel<true>,
      (const void*)op_rows_inv_kernel<false>, (const void*)op_rows_inv_kernel<true>};
  solver_kernels<false, double>(fns);
  solver_kernels<true, double>(fns);
  solver_kernels_f32(fns, false);
  solver_kernels_f32(fns, true);
  persist_kernels_all(fns);
  for (const void* f : fns) {
    hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
    if (e != hipSuccess) return e;
  }
  hipError_t e = BSGP_COOP512 ? bsgp_c512_set_lds_limit(bytes) : hipSuccess;
  if (e == hipSuccess && BSGP_COOP512) e = bsgp_c512_persist_set_lds_limit(bytes);
  if (e == hipSuccess) e = bsgp_app_persist_set_lds_limit(bytes);
  if (e == hipSuccess) applied[dev] = bytes;
  return e;
}

}  // namespace bsgp
