// Host accuracy test of bsgp::fast_log (beta-sgp_amd/csrc/bsgp_math.hpp)
// against long double log: max error in ulp over random normal inputs.
#include <cmath>
#include <cstdio>
#include <random>
#include "bsgp_math.hpp"

int main() {
  std::mt19937_64 rng(7);
  double worst = 0, worst_x = 0;
  auto check = [&](double x) {
    long double ref = logl((long double)x);
    double got = bsgp::fast_log(x);
    double r = (double)ref;
    double ulp = std::fabs(std::nextafter(r, INFINITY) - r);
    if (r == 0) ulp = 4.9e-324;
    double e = std::fabs((long double)got - ref) / ulp;
    if (e > worst) { worst = e; worst_x = x; }
  };
  std::uniform_real_distribution<double> ue(-700, 700), uu(0.5, 2.0);
  for (int i = 0; i < 2000000; ++i) check(std::exp(ue(rng)));
  for (int i = 0; i < 2000000; ++i) check(uu(rng));
  for (int i = 0; i < 200000; ++i) check(1.0 + (uu(rng) - 1.25) * 1e-6);
  check(1.0); check(2.0); check(0.5); check(1e-300); check(1e300);
  printf("fast_log max error %.3f ulp at x=%.17g\n", worst, worst_x);
  bool ok = worst < 1.0 && std::isnan(bsgp::fast_log(-1.0)) && std::isinf(bsgp::fast_log(0.0));
  // fast_exp over the whole finite range and densely near 0 (the beta-1
  // exponents of the line search)
  double wexp = 0, wexp_t = 0;
  auto check_exp = [&](double t) {
    long double ref = expl((long double)t);
    double got = bsgp::fast_exp(t);
    double r = (double)ref;
    double ulp = std::fabs(std::nextafter(r, INFINITY) - r);
    double e = std::fabs((long double)got - ref) / ulp;
    if (e > wexp) { wexp = e; wexp_t = t; }
  };
  std::uniform_real_distribution<double> te(-707.9, 708.9), ts(-2.0, 2.0);
  for (int i = 0; i < 2000000; ++i) check_exp(te(rng));
  for (int i = 0; i < 2000000; ++i) check_exp(ts(rng));
  for (int i = 0; i < 200000; ++i) check_exp((uu(rng) - 1.25) * 1e-8);
  check_exp(0.0); check_exp(1.0); check_exp(-1.0); check_exp(0.34657359027997264);
  printf("fast_exp max error %.3f ulp at t=%.17g\n", wexp, wexp_t);
  ok = ok && wexp < 1.0 && std::isinf(bsgp::fast_exp(1000.0)) && bsgp::fast_exp(-1000.0) == 0.0 &&
       std::isnan(bsgp::fast_exp(NAN));
  // div_rn: the compact-gn decode gn/scaling (bsgp_math.hpp) must equal the
  // IEEE quotient bit for bit for positive f32 numerators over a positive f32
  // scaling (integer counts and general f32 FITS samples)
  long ndiv = 0, bad_div = 0;
  std::uniform_real_distribution<float> uf(1e-3f, 1e5f), us(1.0f, 7e4f);
  std::uniform_int_distribution<int> ui(1, 70000);
  for (int s = 0; s < 2000; ++s) {
    const double sc = (s & 1) ? (double)us(rng) : (double)ui(rng);  // max(gn): f32-exact
    const double r = 1.0 / sc;
    for (int i = 0; i < 2000; ++i) {
      const double a = (i & 1) ? (double)uf(rng) : (double)ui(rng);
      ++ndiv;
      if (bsgp::div_rn(a, sc, r) != a / sc) ++bad_div;
    }
    ++ndiv;
    if (bsgp::div_rn(sc, sc, r) != 1.0) ++bad_div;  // the maximum pixel scales to exactly 1
  }
  printf("div_rn: %ld of %ld quotients differ from a / b\n", bad_div, ndiv);
  ok = ok && bad_div == 0;
  printf(ok ? "math: all ok\n" : "math: FAIL\n");
  return ok ? 0 : 1;
}
