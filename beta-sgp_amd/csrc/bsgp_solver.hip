// bsgp_solver.hip — the persistent batched beta-SGP solve kernel for gfx950
// and the small standalone kernels behind include/bsgp.h.
//
// Reference hot path: restoration/sgp.py:41-438 (sgp, KL) and :506-895
// (sgp_betaDiv), restoration/flux_conserve_proj.py:7-144 (projectDF).
//
// One workgroup = one image for the whole solve (setup, every iteration,
// every inner loop).  Workgroups pull images from a device queue, so a batch
// of B images needs no host involvement between launch and completion.
#include <hip/hip_runtime.h>

#include "bsgp_device.hpp"
#include "bsgp_internal.hpp"

namespace bsgp {

// ------------------------------------------------------------------ helpers
__device__ __forceinline__ double clipX(double x, double lo, double hi) {
  // X[X < lo] = lo; X[X > hi] = hi  (sgp.py:355-357)
  double X = (x < lo) ? lo : x;
  return (X > hi) ? hi : X;
}

__device__ __forceinline__ double realtime_s() {
  return (double)__builtin_amdgcn_s_memrealtime() * 1e-8;  // 100 MHz constant clock
}

// Per-image scalar state, identical in every thread of the workgroup.
struct State {
  double scaling, flux, fv, alpha, tau, lr, init_lr, beta;
  double lo, hi;  // X bounds
  double Valpha[32];
  double Fold[32];
};

// --------------------------------------------------------------- the solver
__global__ void __launch_bounds__(kBlock) sgp_solve_kernel(SolveArgs A) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  cd* lds = reinterpret_cast<cd*>(smem);
  double* red = reinterpret_cast<double*>(smem + A.lds_fft_bytes);
  int& s_img = *reinterpret_cast<int*>(red + kWaves * kMaxRed);  // inside the dynamic carve

  const Geo& G = A.g;
  const bsgp_params& P = A.prm;
  const int N = G.H * G.W;
  const int tid = threadIdx.x;
  const bool bmap = P.bkg_is_map != 0;
  const bool beta_v = P.variant == BSGP_VARIANT_BETA;
  const int MAXIT1 = P.MAXIT + 1;

  double* ws = A.ws + (size_t)blockIdx.x * A.slot_stride;
  double* gns = ws;                 // scaled, null-fixed gn
  double* bks = gns + A.vec_stride; // scaled bkg map (bmap)
  double* xa = bks + A.vec_stride;  // x at iteration start
  double* xb = xa + A.vec_stride;   // x at iteration end
  double* ga = xb + A.vec_stride;
  double* gb = ga + A.vec_stride;
  double* xtf = gb + A.vec_stride;  // A(x)
  double* dtf = xtf + A.vec_stride; // A(d)
  cd* spec = reinterpret_cast<cd*>(dtf + A.vec_stride);

  for (;;) {
    if (tid == 0) s_img = atomicAdd(A.queue, 1);
    __syncthreads();
    const int img = s_img;
    __syncthreads();
    if (img >= A.B) break;

    const double* gn_in = A.in.gn + (size_t)img * N;
    const double* bk_in = bmap ? A.in.bkg + (size_t)img * N : nullptr;
    const double bk_scalar_raw = bmap ? 0.0 : A.in.bkg[img];
    const double t0 = realtime_s();

    State S;
    S.beta = A.in.beta0 ? A.in.beta0[img] : P.betaParam;
    S.lr = P.lr;
    S.init_lr = P.lr;
    S.tau = P.tau;
    S.alpha = P.alpha;
    int64_t E_p = 0, E_ls = 0, ls_passes = 0, status = 0;

    // ---- setup 1: raw statistics (sgp.py:174-177, 190, 193-194)
    double sc;
    {
      double v[2] = {0.0, 0.0};  // sum(gn - bkg), sum(gn)
      double mx = -INFINITY;
      for (int i = tid; i < N; i += kBlock) {
        const double g = gn_in[i];
        const double bkr = bmap ? bk_in[i] : bk_scalar_raw;
        v[0] += g - bkr;
        v[1] += g;
        mx = (g > mx || g != g) ? g : mx;
      }
      block_sum<2>(v, red);
      mx = block_max(mx, red);
      sc = P.scale_data == 2 ? P.prescaled_scaling : (P.scale_data ? mx : 1.0);
      S.scaling = sc;
      // init_recon 3 constant (before scaling), flux given or sum(gn - bkg)
      const double flux_in = A.in.flux ? A.in.flux[img] : 0.0;
      S.flux = A.in.flux ? flux_in : v[0];  // temporarily: raw flat-init numerator
      S.fv = v[1] / (double)N;              // temporarily: mean(gn) for stop rule 4
    }
    const double x3 = (S.flux / (double)N) * 1.0;  // np.sum(gn-bkg)/gn.size*ones
    const double tol4 = P.scale_data == 2 ? P.prescaled_tol4 : 1 + 1 / S.fv;
    const bool divide = P.scale_data == 1;  // device applies the scaling
    // ---- setup 2: scale, null-pixel minimum (sgp.py:193-204)
    const double bks_scalar = P.scale_data == 2 ? bk_scalar_raw : bk_scalar_raw / sc;
    {
      double vmin = INFINITY;
      for (int i = tid; i < N; i += kBlock) {
        const double g = divide ? gn_in[i] / sc : gn_in[i];
        gns[i] = g;
        if (g > 0 && g < vmin) vmin = g;
        if (bmap) bks[i] = divide ? bk_in[i] / sc : bk_in[i];
      }
      vmin = block_min(vmin, red);
      const double eps = 2.220446049250313e-16;
      const double fill = vmin * eps * eps;
      double v[1] = {0.0};
      for (int i = tid; i < N; i += kBlock) {
        double g = gns[i];
        if (g <= 0) {
          g = fill;
          gns[i] = g;
        }
        v[0] += g - (bmap ? bks[i] : bks_scalar);
        // initial x (sgp.py:166-177, 197), then the pflag==0 clamp (:248-249)
        double x;
        if (A.in.x0) {
          x = A.in.x0[(size_t)img * N + i];
        } else if (P.init_recon == 0) {
          x = 0.0;
        } else if (P.init_recon == 2) {
          x = gn_in[i];
        } else {
          x = x3;
        }
        if (divide) x = x / sc;
        if (P.proj_type == 0 && x < 0) x = 0;
        xa[i] = x;
      }
      block_sum<1>(v, red);
      // flux (sgp.py:208-211)
      S.flux = A.in.flux ? A.in.flux[img] / sc : v[0];
    }
    const double flux = S.flux;
    const ProjClip clip{P.has_sat != 0, P.ccd_sat_level / sc - 2.220446049250313e-16};
    __syncthreads();

    // ---- setup 3: initial projection with dia = 1 (sgp.py:250-253)
    if (P.proj_type == 1) {
      ProjOut po = project_df(
          N, [&](int i, double& c, double& dia) { c = xa[i]; dia = 1.0; }, clip, flux, 0.0, 1.0,
          1e-11, 0, 0, P.max_projs, red);
      for (int i = tid; i < N; i += kBlock) xa[i] = clip(xa[i], 1.0, po.lam);
      __syncthreads();
    }

    // ---- setup 4: x_tf = A(x), f, g (sgp.py:260-265 / 702-709)
    Objective obj;
    obj.variant = P.variant;
    obj.set_beta(S.beta);
    double fsum[3] = {0.0, 0.0, 0.0};  // K, T0, T1
    row_fwd(G, G.H, G.W, spec, lds, [&](int r, int j) { return xa[r * G.W + j]; });
    __syncthreads();
    col_conv(G, spec, G.tfA, lds);
    row_inv_fwd(G, spec, lds, [&](int r, int j, double v) {
      const int i = r * G.W + j;
      xtf[i] = v;
      const double den = v + (bmap ? bks[i] : bks_scalar);
      const double g = gns[i];
      fsum[0] += obj.konst(g);
      obj.terms(v, den, g, &fsum[1]);
      return obj.grad_w(den, g);
    });
    block_sum<3>(fsum, red);  // includes the barrier that publishes xtf / spec
    S.fv = obj.combine(fsum[0], fsum[1], fsum[2], flux, (double)N);
    col_conv(G, spec, G.tfAT, lds);
    row_inv(G, spec, lds, [&](int r, int j, double at) {
      const int i = r * G.W + j;
      const double den = xtf[i] + (bmap ? bks[i] : bks_scalar);
      ga[i] = obj.grad_g1(den) - at;
    });
    __syncthreads();
    // ---- setup 5: scaling-matrix bounds from AT(gn) (sgp.py:268-273)
    row_fwd(G, G.H, G.W, spec, lds, [&](int r, int j) { return gns[r * G.W + j]; });
    __syncthreads();
    col_conv(G, spec, G.tfAT, lds);
    {
      double ymin = INFINITY, ymax = -INFINITY;
      row_inv(G, spec, lds, [&](int r, int j, double at) {
        const int i = r * G.W + j;
        const double bkv = bmap ? bks[i] : bks_scalar;
        const double y = (flux / (flux + bkv)) * at;
        if (y > 0 && y < ymin) ymin = y;
        ymax = (y > ymax || y != y) ? y : ymax;
      });
      ymin = block_min(ymin, red);
      ymax = block_max(ymax, red);
      S.lo = ymin;
      S.hi = ymax;
      if (S.hi / S.lo < 50) {
        S.lo = S.lo / 10;
        S.hi = S.hi * 10;
      }
    }
    const double Dcoeff = 2 / (double)N * sc;
    double* discr = A.out.discr + (size_t)img * MAXIT1;
    if (tid == 0) {
      discr[0] = Dcoeff * S.fv;
      if (A.out.times) A.out.times[(size_t)img * MAXIT1] = 0.0;
      if (A.out.crit) A.out.crit[(size_t)img * MAXIT1] = 0.0;
      if (A.out.flags) A.out.flags[(size_t)img * MAXIT1] = 0;
    }
    for (int k = 0; k < P.M_alpha; ++k) S.Valpha[k] = P.alpha_max;
    for (int k = 0; k < P.M; ++k) S.Fold[k] = -1e30;
    double tol = P.tol_convergence;
    if (P.stop_criterion == 4) tol = tol4;
    if (P.verbose && P.stop_criterion == 2) tol = tol * tol;
    bool Xones = (P.init_recon == 0);  // X = ones until the first BB update (sgp.py:279-280)

    // ---- main loop (sgp.py:302-425 / 748-882)
    int iter_ = 1;
    int epoch = 0;
    const int K = P.adapt_beta && beta_v ? 1 : P.ls_spec;
    for (;;) {
      epoch += 1;
      for (int k = 0; k < P.M_alpha - 1; ++k) S.Valpha[k] = S.Valpha[k + 1];
      for (int k = 0; k < P.M - 1; ++k) S.Fold[k] = S.Fold[k + 1];
      S.Fold[P.M - 1] = S.fv;
      const double alpha = S.alpha;
      const double lo = S.lo, hi = S.hi;

      // direction y = x - alpha*X*g and its projection (sgp.py:311-316)
      auto ycd = [&](int i, double& c, double& dia) {
        const double x = xa[i];
        const double X = Xones ? 1.0 : clipX(x, lo, hi);
        const double D = 1 / X;
        const double y = x - alpha * (X * ga[i]);
        c = y * D;
        dia = D;
      };
      double lam_p = 0.0;
      if (P.proj_type == 1) {
        ProjOut po = project_df(N, ycd, clip, flux, 0.0, 1.0, 1e-11, 0, 0, P.max_projs, red);
        lam_p = po.lam;
        E_p += po.evals;
      }
      auto dir = [&](int i) {  // d = y - x (sgp.py:318)
        double y;
        if (P.proj_type == 1) {
          double c, dia;
          ycd(i, c, dia);
          y = clip(c, dia, lam_p);
        } else {
          const double x = xa[i];
          const double X = Xones ? 1.0 : clipX(x, lo, hi);
          y = x - alpha * (X * ga[i]);
          if (y < 0) y = 0;
        }
        return y - xa[i];
      };

      // d, gd = d.g, A(d) (sgp.py:318-325)
      double gd[1] = {0.0};
      row_fwd(G, G.H, G.W, spec, lds, [&](int r, int j) {
        const int i = r * G.W + j;
        const double d = dir(i);
        gd[0] += d * ga[i];
        return d;
      });
      block_sum<1>(gd, red);
      col_conv(G, spec, G.tfA, lds);

      // line search (sgp.py:328-349 / 776-801): K trial lambdas per pass
      double fr = S.Fold[0];
      for (int k = 1; k < P.M; ++k) fr = py_max2(fr, S.Fold[k]);
      double lam = 1.0;
      int accepted = -1;
      double f_acc = 0.0;
      bool first = true;
      int nls = 0;
      while (accepted < 0) {
        double lamk[8];
        lamk[0] = lam;
        for (int k = 1; k < K; ++k) lamk[k] = lamk[k - 1] * P.beta;
        double t[2 * 8 + 2];
        for (int k = 0; k < 2 * 8 + 2; ++k) t[k] = 0.0;
        const bool adapt = P.adapt_beta && beta_v;
        auto eval_px = [&](int i, double dt) {
          const double g = gns[i];
          const double bkv = bmap ? bks[i] : bks_scalar;
          const double x0 = xtf[i];
          t[2 * 8] += obj.konst(g);
          for (int k = 0; k < K; ++k) {
            const double xt = x0 + lamk[k] * dt;
            const double den = xt + bkv;
            obj.terms(xt, den, g, &t[2 * k]);
          }
          if (adapt) t[2 * 8 + 1] += beta_deriv_px(x0 + lamk[0] * dt + bkv, g, obj.beta);
        };
        if (first) {
          row_inv(G, spec, lds, [&](int r, int j, double v) {
            const int i = r * G.W + j;
            dtf[i] = v;
            eval_px(i, v);
          });
          first = false;
        } else {
          for (int i = tid; i < N; i += kBlock) eval_px(i, dtf[i]);
        }
        block_sum<2 * 8 + 2>(t, red);
        ++ls_passes;
        for (int k = 0; k < K; ++k) {
          const double fk = obj.combine(t[2 * 8], t[2 * k], t[2 * k + 1], flux, (double)N);
          ++nls;
          if (fk <= fr + P.gamma * lamk[k] * gd[0] || lamk[k] < 1e-12) {
            accepted = k;
            f_acc = fk;
            lam = lamk[k];
            break;
          }
        }
        if (accepted < 0) {
          lam = lamk[K - 1] * P.beta;
          if (adapt) {  // sgp.py:798-800: beta -= lr * mean(dDiv/dbeta)
            const double bgrad = (obj.beta == 0.0 || obj.beta == 1.0) ? 0.0 : t[2 * 8 + 1] / N;
            obj.set_beta(obj.beta - S.lr * bgrad);
          }
        }
        if (nls > 64) {  // unreachable: lam < 1e-12 forces acceptance by the 32nd trial
          status |= 1;
          accepted = 0;
          f_acc = 0.0;
        }
      }
      E_ls += nls;
      S.fv = f_acc;
      S.beta = obj.beta;
      const double lam_acc = lam;
      if (tid == 0 && A.out.flags)
        A.out.flags[(size_t)img * MAXIT1 + iter_] = (S.fv >= fr) ? 1 : 0;

      // accept: x_tf += lam*d_tf; w = gn/den or gn*den^(b-2); AT(w) (sgp.py:337-345)
      row_fwd(G, G.H, G.W, spec, lds, [&](int r, int j) {
        const int i = r * G.W + j;
        const double xt = xtf[i] + lam_acc * dtf[i];
        xtf[i] = xt;
        const double den = xt + (bmap ? bks[i] : bks_scalar);
        return obj.grad_w(den, gns[i]);
      });
      __syncthreads();
      col_conv(G, spec, G.tfAT, lds);
      // new gradient, x update, BB sums (sgp.py:337-365, 402)
      double bb[6] = {0, 0, 0, 0, 0, 0};  // bk, ck, sk2.sk2, yk2.yk2, sk.sk, x.x
      row_inv(G, spec, lds, [&](int r, int j, double at) {
        const int i = r * G.W + j;
        const double den = xtf[i] + (bmap ? bks[i] : bks_scalar);
        const double gnew = obj.grad_g1(den) - at;
        const double d = dir(i);
        const double sk = lam_acc * d;
        const double xn = xa[i] + lam_acc * d;
        const double yk = gnew - ga[i];
        const double X = clipX(xn, lo, hi);
        const double D = 1 / X;
        const double sk2 = sk * D;
        const double yk2 = yk * X;
        bb[0] += sk2 * yk;
        bb[1] += yk2 * sk;
        bb[2] += sk2 * sk2;
        bb[3] += yk2 * yk2;
        bb[4] += sk * sk;
        bb[5] += xn * xn;
        xb[i] = xn;
        gb[i] = gnew;
      });
      block_sum<6>(bb, red);

      // Barzilai-Borwein steps and the tau alternation (sgp.py:366-386)
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
      S.Valpha[P.M_alpha - 1] = alpha2;
      double vmin = S.Valpha[0];
      for (int k = 1; k < P.M_alpha; ++k) vmin = py_min2(vmin, S.Valpha[k]);
      if (iter_ <= 20) {
        S.alpha = vmin;
      } else if (alpha2 / alpha1 < S.tau) {
        S.alpha = vmin;
        S.tau = S.tau * 0.9;
      } else {
        S.alpha = alpha1;
        S.tau = S.tau * 1.1;
      }
      if (beta_v && P.schedule_lr) S.lr = S.init_lr * exp(-P.lr_exp_param * epoch);

      // stop rules (sgp.py:390-414)
      iter_ += 1;
      bool loop = true;
      double crit = 0.0;
      const double dk = Dcoeff * S.fv;
      if (P.stop_criterion == 2) {
        crit = bb[4] / bb[5];
        loop = crit > tol;
      } else if (P.stop_criterion == 3) {
        crit = (S.Fold[P.M - 1] - S.fv) / S.fv;
        loop = crit > tol && crit >= 0;
      } else if (P.stop_criterion == 4) {
        crit = dk;
        loop = dk > tol;
      }
      if (iter_ > P.MAXIT) loop = false;
      if (tid == 0) {
        discr[iter_ - 1] = dk;
        if (A.out.times) A.out.times[(size_t)img * MAXIT1 + iter_ - 1] = realtime_s() - t0;
        if (A.out.crit) A.out.crit[(size_t)img * MAXIT1 + iter_ - 1] = crit;
      }
      if (!loop) break;  // x reverts to prev_x = xa (sgp.py:424-425)
      double* t1 = xa;
      xa = xb;
      xb = t1;
      t1 = ga;
      ga = gb;
      gb = t1;
      Xones = false;
      __syncthreads();
    }

    // ---- outputs (sgp.py:428-438, 892-895)
    double* xo = A.out.x + (size_t)img * N;
    for (int i = tid; i < N; i += kBlock) xo[i] = xa[i] * sc;
    if (tid == 0) {
      A.out.iters[img] = iter_ - 1;
      if (A.out.beta_final) A.out.beta_final[img] = S.beta;
      if (A.out.counters) {
        int64_t* c = A.out.counters + (size_t)img * 4;
        c[0] = E_p;
        c[1] = E_ls;
        c[2] = ls_passes;
        c[3] = status;
      }
    }
    // restore slot pointers for the next image of this workgroup
    xa = bks + A.vec_stride;
    xb = xa + A.vec_stride;
    ga = xb + A.vec_stride;
    gb = ga + A.vec_stride;
    __syncthreads();
  }
}

// --------------------------------------------------------- TF construction
// tf[k][p] = FFT2(kc)[p][k] * scale (optionally conjugated); kc is P x Q real.
__global__ void __launch_bounds__(kBlock) build_tf_kernel(Geo G, const double* kc, cd* spec,
                                                          cd* tf, double scale, int conj) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  cd* lds = reinterpret_cast<cd*>(smem);
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  row_fwd(G, G.P, G.Q, spec, lds, [&](int r, int j) { return kc[r * G.Q + j]; });
  __syncthreads();
  const int C = G.nfw;
  const int stride = 2 * G.lpad;
  for (int k0 = 0; k0 < G.Qh; k0 += C) {
    for (int idx = threadIdx.x; idx < G.P * C; idx += kBlock) {
      const int p = idx / C, c = idx - p * C, k = k0 + c;
      lds[c * stride + p] = (k < G.Qh) ? spec[(size_t)p * G.Qh + k] : cmk(0.0, 0.0);
    }
    __syncthreads();
    if (w < C && k0 + w < G.Qh) {
      cd* a = lds + w * stride;
      cd* Z = fft_run(a, a + G.lpad, G.fp, false, lane, 64, WaveSync());
      cd* t = tf + (size_t)(k0 + w) * G.P;
      for (int p = lane; p < G.P; p += 64) {
        cd z = cscale(Z[p], scale);
        t[p] = conj ? cconj(z) : z;
      }
    }
    __syncthreads();
  }
}

// ------------------------------------------------------ A / AT standalone
__global__ void __launch_bounds__(kBlock) apply_op_kernel(Geo G, int B, int transpose,
                                                          const double* x, double* out,
                                                          cd* specws, size_t spec_stride) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  cd* lds = reinterpret_cast<cd*>(smem);
  const int N = G.H * G.W;
  cd* spec = specws + (size_t)blockIdx.x * spec_stride;
  for (int img = blockIdx.x; img < B; img += gridDim.x) {
    const double* xi = x + (size_t)img * N;
    double* oi = out + (size_t)img * N;
    row_fwd(G, G.H, G.W, spec, lds, [&](int r, int j) { return xi[r * G.W + j]; });
    __syncthreads();
    col_conv(G, spec, transpose ? G.tfAT : G.tfA, lds);
    row_inv(G, spec, lds, [&](int r, int j, double v) { oi[r * G.W + j] = v; });
    __syncthreads();
  }
}

// ----------------------------------------------------------- projectDF
__global__ void __launch_bounds__(kBlock) project_df_kernel(int n, double b, const double* c,
                                                            const double* dia, ProjClip clip,
                                                            double lam0, double dlam0,
                                                            double tol_lam, int biter, int siter,
                                                            int max_projs, double* x,
                                                            double* info) {
  __shared__ double red[kWaves * kMaxRed];
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
  __shared__ double red[kWaves * kMaxRed];
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
hipError_t launch_solve(const SolveArgs& a, int grid, size_t lds, hipStream_t s) {
  hipLaunchKernelGGL(sgp_solve_kernel, dim3(grid), dim3(kBlock), lds, s, a);
  return hipGetLastError();
}
hipError_t launch_build_tf(const Geo& g, const double* kc, cd* spec, cd* tf, double scale,
                           int conj, size_t lds, hipStream_t s) {
  hipLaunchKernelGGL(build_tf_kernel, dim3(1), dim3(kBlock), lds, s, g, kc, spec, tf, scale,
                     conj);
  return hipGetLastError();
}
hipError_t launch_apply_op(const Geo& g, int B, int transpose, const double* x, double* out,
                           cd* specws, size_t spec_stride, int grid, size_t lds, hipStream_t s) {
  hipLaunchKernelGGL(apply_op_kernel, dim3(grid), dim3(kBlock), lds, s, g, B, transpose, x, out,
                     specws, spec_stride);
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
hipError_t set_solver_lds_limit(size_t bytes) {
  hipError_t e = hipFuncSetAttribute((const void*)sgp_solve_kernel,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
  if (e != hipSuccess) return e;
  e = hipFuncSetAttribute((const void*)apply_op_kernel,
                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
  if (e != hipSuccess) return e;
  return hipFuncSetAttribute((const void*)build_tf_kernel,
                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
}

}  // namespace bsgp
