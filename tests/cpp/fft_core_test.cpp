// Host-side unit test of the FFT core in beta-sgp_amd/csrc/bsgp_fft.hpp.
// Executes each Stockham stage serially (lane loop of width 1), which is the
// same per-stage semantics the per-wave GPU code relies on (stages separated
// by an LDS sync). Checks: 1-D transforms vs a naive long-double DFT for many
// lengths, and the two-real-rows R2C split / C2R gather round trip.
// Build+run: g++ -O2 -std=c++17 -I beta-sgp_amd/csrc tests/cpp/fft_core_test.cpp && ./a.out
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "bsgp_fft.hpp"
using namespace bsgp;

static std::vector<cd> twiddles(int n) {
  std::vector<cd> t(n);
  for (int k = 0; k < n; ++k) {
    long double a = -2.0L * 3.141592653589793238462643383279502884L * k / n;
    t[k] = cmk((double)cosl(a), (double)sinl(a));
  }
  return t;
}

static double check_len(int n, bool inv) {
  FftPlan p;
  p.n = n;
  if (!plan_radices(n, p.radix, &p.ns)) { printf("plan fail %d\n", n); exit(1); }
  std::vector<cd> tw = twiddles(n);
  p.tw = tw.data();
  std::vector<cd> a(n), b(n), x(n);
  srand(n * 7 + inv);
  for (int i = 0; i < n; ++i) x[i] = a[i] = cmk(rand() / (double)RAND_MAX - 0.5, rand() / (double)RAND_MAX - 0.5);
  cd* res = fft_run(a.data(), b.data(), p, inv, 0, 1, [] {});
  double maxerr = 0, maxref = 0;
  for (int k = 0; k < n; ++k) {
    long double sr = 0, si = 0;
    for (int j = 0; j < n; ++j) {
      long double ang = (inv ? 2.0L : -2.0L) * 3.141592653589793238462643383279502884L * (((long long)j * k) % n) / n;
      sr += x[j].x * cosl(ang) - x[j].y * sinl(ang);
      si += x[j].x * sinl(ang) + x[j].y * cosl(ang);
    }
    maxerr = fmax(maxerr, fabs((double)(res[k].x - sr)) + fabs((double)(res[k].y - si)));
    maxref = fmax(maxref, fabs((double)sr) + fabs((double)si));
  }
  return maxerr / maxref;
}

int main() {
  int lens[] = {1, 2, 3, 4, 5, 6, 7, 8, 9, 12, 14, 16, 25, 31, 32, 49, 62, 77, 93, 60, 64, 96, 100, 128, 243, 256, 270, 288, 300, 320, 384, 512};
  int bad = 0;
  for (int n : lens) {
    for (int inv = 0; inv < 2; ++inv) {
      double e = check_len(n, inv);
      if (!(e < 1e-14)) { printf("FAIL n=%d inv=%d relerr=%g\n", n, inv, e); bad++; }
    }
  }
  // two-real-rows split + gather round trip
  for (int Q : {8, 9, 31, 256, 270}) {
    FftPlan p;
    p.n = Q;
    plan_radices(Q, p.radix, &p.ns);
    std::vector<cd> tw = twiddles(Q);
    p.tw = tw.data();
    int Qh = Q / 2 + 1;
    std::vector<double> ra(Q), rb(Q);
    std::vector<cd> z(Q), s(Q), A(Qh), B(Qh);
    for (int j = 0; j < Q; ++j) { ra[j] = rand() / (double)RAND_MAX; rb[j] = rand() / (double)RAND_MAX; z[j] = cmk(ra[j], rb[j]); }
    cd* Z = fft_run(z.data(), s.data(), p, false, 0, 1, [] {});
    for (int k = 0; k < Qh; ++k) r2c_split(Z, Q, k, &A[k], &B[k]);
    // check A against the direct real DFT of ra
    double e1 = 0;
    for (int k = 0; k < Qh; ++k) {
      long double sr = 0, si = 0;
      for (int j = 0; j < Q; ++j) {
        long double ang = -2.0L * 3.141592653589793238462643383279502884L * (((long long)j * k) % Q) / Q;
        sr += rb[j] * cosl(ang); si += rb[j] * sinl(ang);
      }
      e1 = fmax(e1, fabs((double)(B[k].x - sr)) + fabs((double)(B[k].y - si)));
    }
    std::vector<cd> zz(Q), ss(Q);
    for (int k = 0; k < Q; ++k) zz[k] = c2r_gather(A.data(), B.data(), Q, Qh, k);
    cd* zr = fft_run(zz.data(), ss.data(), p, true, 0, 1, [] {});
    double e2 = 0;
    for (int j = 0; j < Q; ++j) e2 = fmax(e2, fabs(zr[j].x / Q - ra[j]) + fabs(zr[j].y / Q - rb[j]));
    if (!(e1 < 1e-12 && e2 < 1e-14)) { printf("FAIL split Q=%d e1=%g e2=%g\n", Q, e1, e2); bad++; }
  }
  // compile-time paths (composite radix-6/9 stages for 270, 8/10/5 for 400,
  // 8/6/10 for 480) vs the naive DFT
  // and vs the runtime plan
  for (int n : {256, 270, 400, 480}) {
    for (int inv = 0; inv < 2; ++inv) {
      FftPlan p;
      p.n = n;
      plan_radices(n, p.radix, &p.ns);
      std::vector<cd> tw = twiddles(n);
      p.tw = tw.data();
      std::vector<cd> a(n), b(n), c(n), d(n), x(n);
      for (int i = 0; i < n; ++i) x[i] = c[i] = a[i] = cmk(rand() / (double)RAND_MAX, rand() / (double)RAND_MAX);
      cd* r1 = fft_run(a.data(), b.data(), p, inv, 0, 1, [] {});
      cd* r2 = fft_any(c.data(), d.data(), p, inv, 0, 1, [] {});
      double maxerr = 0, maxref = 0, maxdiff = 0;
      for (int k = 0; k < n; ++k) {
        long double sr = 0, si = 0;
        for (int j = 0; j < n; ++j) {
          long double ang = (inv ? 2.0L : -2.0L) * 3.141592653589793238462643383279502884L * (((long long)j * k) % n) / n;
          sr += x[j].x * cosl(ang) - x[j].y * sinl(ang);
          si += x[j].x * sinl(ang) + x[j].y * cosl(ang);
        }
        maxerr = fmax(maxerr, fabs((double)(r2[k].x - sr)) + fabs((double)(r2[k].y - si)));
        maxref = fmax(maxref, fabs((double)sr) + fabs((double)si));
        maxdiff = fmax(maxdiff, fabs(r1[k].x - r2[k].x) + fabs(r1[k].y - r2[k].y));
      }
      if (!(maxerr / maxref < 1e-14 && maxdiff / maxref < 1e-14)) {
        printf("FAIL static n=%d inv=%d relerr=%g vs runtime %g\n", n, inv, maxerr / maxref, maxdiff / maxref);
        bad++;
      }
    }
  }
  // workgroup-wide radix-8 plan for 2048 (cooperative passes, 256 lanes run
  // serially here) vs the runtime plan
  for (int inv = 0; inv < 2; ++inv) {
    const int n = 2048;
    FftPlan p;
    p.n = n;
    plan_radices(n, p.radix, &p.ns);
    std::vector<cd> tw = twiddles(n);
    p.tw = tw.data();
    std::vector<cd> a(n), b(n), c(n), d(n);
    for (int i = 0; i < n; ++i) c[i] = a[i] = cmk(rand() / (double)RAND_MAX, rand() / (double)RAND_MAX);
    cd* r1 = fft_run(a.data(), b.data(), p, inv, 0, 1, [] {});
    {
      std::vector<cd> x(c), y(n);
      cd* r2 = fft_wide(x.data(), y.data(), p, inv, 0, 1, [] {});
      double maxdiff = 0, maxref = 0;
      for (int k = 0; k < n; ++k) {
        maxdiff = fmax(maxdiff, fabs(r1[k].x - r2[k].x) + fabs(r1[k].y - r2[k].y));
        maxref = fmax(maxref, fabs(r1[k].x) + fabs(r1[k].y));
      }
      if (!(maxdiff / maxref < 1e-14)) {
        printf("FAIL wide n=2048 inv=%d diff %g\n", inv, maxdiff / maxref);
        bad++;
      }
    }
    {  // the two-level twiddle table (Tw2: w^a * w^(64 b), the device's LDS copy)
      std::vector<cd> t2(64 + n / 64);
      for (int a = 0; a < 64; ++a) t2[a] = tw[a];
      for (int b2 = 0; b2 < n / 64; ++b2) t2[64 + b2] = tw[64 * b2];
      std::vector<cd> x(c), y(n);
      cd* r3 = fft_run_static<2048, true, true>(x.data(), y.data(), Tw2{t2.data(), t2.data() + 64},
                                               inv, 0, 1, [] {});
      double maxdiff = 0, maxref = 0;
      for (int k = 0; k < n; ++k) {
        maxdiff = fmax(maxdiff, fabs(r1[k].x - r3[k].x) + fabs(r1[k].y - r3[k].y));
        maxref = fmax(maxref, fabs(r1[k].x) + fabs(r1[k].y));
      }
      if (!(maxdiff / maxref < 1e-14)) {
        printf("FAIL wide n=2048 two-level twiddles inv=%d diff %g\n", inv, maxdiff / maxref);
        bad++;
      }
    }
  }
  printf(bad ? "FFT core: %d failures\n" : "FFT core: all ok\n", bad);
  return bad ? 1 : 0;
}
