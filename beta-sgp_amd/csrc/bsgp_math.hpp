// bsgp_math.hpp — f64 logarithm for the divergence hot loops (host + device).
//
// The beta-divergence line search evaluates den**(beta-1) = exp((beta-1)*log den)
// and, for KL, gn*log(gn/den) for every pixel and every trial step
// (sgp.py:453-458 via betaDiv, sgp.py:334).  ocml's log is a double-double
// implementation (~103 VALU instructions on gfx950); this one is the classic
// reduction to [sqrt(2)/2, sqrt(2)) with s = f/(2+f) and a degree-7 minimax
// polynomial in s^2 (the fdlibm/Cody-Waite formulation, coefficients from
// that published algorithm), ~35 instructions, error < 1 ulp over normal
// positive inputs (checked against long double in tests/cpp/math_test.cpp).
// Non-normal inputs (<= 0, subnormal, inf, NaN) fall back to the library log.
#pragma once

#include <stdint.h>
#include <string.h>

#include <cmath>

#include "bsgp_fft.hpp"  // BSGP_HD

namespace bsgp {

BSGP_HD uint64_t dbits(double x) {
  uint64_t u;
  memcpy(&u, &x, 8);
  return u;
}
BSGP_HD double bitsd(uint64_t u) {
  double x;
  memcpy(&x, &u, 8);
  return x;
}

BSGP_HD double fast_log(double x) {
  const double ln2_hi = 6.93147180369123816490e-01;
  const double ln2_lo = 1.90821492927058770002e-10;
  const double Lg1 = 6.666666666666735130e-01, Lg2 = 3.999999999940941908e-01,
               Lg3 = 2.857142874366239149e-01, Lg4 = 2.222219843214978396e-01,
               Lg5 = 1.818357216161805012e-01, Lg6 = 1.531383769920937332e-01,
               Lg7 = 1.479819860511658591e-01;
  if (!(x >= 2.2250738585072014e-308 && x <= 1.7976931348623157e308)) return std::log(x);
  const uint64_t u = dbits(x);
  int32_t hx = (int32_t)(u >> 32);
  int k = ((hx >> 20) & 0x7ff) - 1023;
  hx &= 0x000fffff;
  const int32_t i = (hx + 0x95f64) & 0x100000;
  // mantissa (or mantissa/2) in [sqrt(2)/2, sqrt(2))
  const double m = bitsd(((uint64_t)(uint32_t)(hx | (i ^ 0x3ff00000)) << 32) | (u & 0xffffffffu));
  k += (i >> 20);
  const double f = m - 1.0;
  const double s = f / (2.0 + f);
  const double dk = (double)k;
  const double z = s * s;
  const double w = z * z;
  const double t1 = w * (Lg2 + w * (Lg4 + w * Lg6));
  const double t2 = z * (Lg1 + w * (Lg3 + w * (Lg5 + w * Lg7)));
  const double R = t2 + t1;
  const double hfsq = 0.5 * f * f;
  return dk * ln2_hi - ((hfsq - (s * (hfsq + R) + dk * ln2_lo)) - f);
}

// exp(t): t = k*ln2 + r with |r| <= ln2/2 (Cody-Waite, fma, exact), exp(r) by
// its degree-13 Taylor polynomial (truncation < 4e-18 relative), scaled by 2^k
// (v_ldexp_f64).  ~20 VALU instructions instead of ocml's ~42; error < 1 ulp
// (tests/cpp/math_test.cpp).  Arguments that over/underflow, and NaN, go to
// the library exp.
BSGP_HD double fast_exp(double t) {
  if (!(t > -708.0 && t < 709.0)) return std::exp(t);
  const double inv_ln2 = 1.44269504088896338700e+00;
  const double ln2_hi = 6.93147180369123816490e-01;
  const double ln2_lo = 1.90821492927058770002e-10;
  const double kd = std::rint(t * inv_ln2);
  const double r = std::fma(-kd, ln2_lo, std::fma(-kd, ln2_hi, t));
  double p = 1.6059043836821614599e-10;  // 1/13!
  p = std::fma(p, r, 2.0876756987868098979e-09);  // 1/12!
  p = std::fma(p, r, 2.5052108385441718775e-08);  // 1/11!
  p = std::fma(p, r, 2.7557319223985890653e-07);  // 1/10!
  p = std::fma(p, r, 2.7557319223985890653e-06);  // 1/9!
  p = std::fma(p, r, 2.4801587301587301587e-05);  // 1/8!
  p = std::fma(p, r, 1.9841269841269841270e-04);  // 1/7!
  p = std::fma(p, r, 1.3888888888888888889e-03);  // 1/6!
  p = std::fma(p, r, 8.3333333333333333333e-03);  // 1/5!
  p = std::fma(p, r, 4.1666666666666666667e-02);  // 1/4!
  p = std::fma(p, r, 1.6666666666666666667e-01);  // 1/3!
  p = std::fma(p, r, 0.5);
  p = std::fma(p, r * r, r);  // r + r^2 * (1/2 + r/6 + ...)
  return std::ldexp(1.0 + p, (int)kd);
}

// a / b correctly rounded from r = RN(1/b) (Markstein's final correction step,
// the one IA-64 division ends with): q = RN(a*r) is within an ulp of a/b, the
// residual a - b*q is exact by fma, and RN(q + residual*r) is the correctly
// rounded quotient when nothing over/underflows.  For the compact gn decode
// (positive f32 counts over a positive f32 scaling) that always holds; it
// needs 3 fp64 ops and no temporaries of v_div_scale/v_div_fixup.  Checked
// bit for bit against a / b in tests/cpp/math_test.cpp.
BSGP_HD double div_rn(double a, double b, double r) {
  const double q = a * r;
  const double e = std::fma(-q, b, a);
  return std::fma(e, r, q);
}

// x**a for positive x via exp(a*log x); for |a*log x| small (the beta-1
// exponents of this path) the result carries ~1 ulp.
BSGP_HD double fast_pow(double x, double a) { return fast_exp(a * fast_log(x)); }

}  // namespace bsgp
