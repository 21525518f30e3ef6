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

// ---------------------------------------------------------------------------
// numpy 1.x float32 power and log of a float32 image (sgp.py:458, 495).
//
// On a float32 array numpy 1.26 evaluates ``x ** b`` and ``np.log(x)``
// element by element with the C library's powf(x, (float)b) / logf(x) unless
// it dispatches to its own SIMD kernels (AVX-512 SVML / AVX2), which are not
// correctly rounded and differ from one CPU to the next.  The reference
// fixtures of the float32 paths (tests/golden/make_golden.py, ``_libm``) are
// made with those SIMD kernels disabled, so the device evaluates exactly
// what the C library computes: glibc >= 2.28's powf / logf (the published
// table-driven algorithms: a 16-entry log table with a short polynomial in
// double, and for powf a 32-entry exp2 table), as glibc's x86-64 build runs
// them on an FMA CPU (its __powf_fma / __logf_fma variants, compiled with
// contraction: each a*b + c is one fma).  All arithmetic is in double, so
// the result is the same bits on the host and on gfx950; checked bit for bit
// against the host's libm in tests/cpp/libmf_test.cpp.
namespace libmf {
struct InvLog {
  double invc, logc;
};
// logf: c near the centre of subinterval i of [OFF, 2*OFF), logc = log(c)
constexpr InvLog kLogTab[16] = {
    {0x1.661ec79f8f3bep+0, -0x1.57bf7808caadep-2}, {0x1.571ed4aaf883dp+0, -0x1.2bef0a7c06ddbp-2},
    {0x1.49539f0f010bp+0, -0x1.01eae7f513a67p-2},  {0x1.3c995b0b80385p+0, -0x1.b31d8a68224e9p-3},
    {0x1.30d190c8864a5p+0, -0x1.6574f0ac07758p-3}, {0x1.25e227b0b8eap+0, -0x1.1aa2bc79c81p-3},
    {0x1.1bb4a4a1a343fp+0, -0x1.a4e76ce8c0e5ep-4}, {0x1.12358f08ae5bap+0, -0x1.1973c5a611cccp-4},
    {0x1.0953f419900a7p+0, -0x1.252f438e10c1ep-5}, {0x1p+0, 0x0p+0},
    {0x1.e608cfd9a47acp-1, 0x1.aa5aa5df25984p-5},  {0x1.ca4b31f026aap-1, 0x1.c5e53aa362eb4p-4},
    {0x1.b2036576afce6p-1, 0x1.526e57720db08p-3},  {0x1.9c2d163a1aa2dp-1, 0x1.bc2860d22477p-3},
    {0x1.886e6037841edp-1, 0x1.1058bc8a07ee1p-2},  {0x1.767dcf5534862p-1, 0x1.4043057b6ee09p-2}};
constexpr double kLn2 = 0x1.62e42fefa39efp-1;
constexpr double kLogPoly[3] = {-0x1.00ea348b88334p-2, 0x1.5575b0be00b6ap-2,
                                -0x1.ffffef20a4123p-2};
// powf's log2: the same subintervals, logc = log2(c)
constexpr double kLog2c[16] = {
    -0x1.efec65b963019p-2, -0x1.b0b6832d4fca4p-2, -0x1.7418b0a1fb77bp-2, -0x1.39de91a6dcf7bp-2,
    -0x1.01d9bf3f2b631p-2, -0x1.97c1d1b3b7afp-3,  -0x1.2f9e393af3c9fp-3, -0x1.960cbbf788d5cp-4,
    -0x1.a6f9db6475fcep-5, 0x0p+0,                0x1.338ca9f24f53dp-4,  0x1.476a9543891bap-3,
    0x1.e840b4ac4e4d2p-3,  0x1.40645f0c6651cp-2,  0x1.88e9c2c1b9ff8p-2,  0x1.ce0a44eb17bccp-2};
constexpr double kLog2Poly[5] = {0x1.27616c9496e0bp-2, -0x1.71969a075c67ap-2,
                                 0x1.ec70a6ca7baddp-2, -0x1.7154748bef6c8p-1,
                                 0x1.71547652ab82bp+0};
// exp2: tab[i] = bits(2^(i/32)) - (i << 47); x = k/32 + r
constexpr uint64_t kExp2Tab[32] = {
    0x3ff0000000000000, 0x3fefd9b0d3158574, 0x3fefb5586cf9890f, 0x3fef9301d0125b51,
    0x3fef72b83c7d517b, 0x3fef54873168b9aa, 0x3fef387a6e756238, 0x3fef1e9df51fdee1,
    0x3fef06fe0a31b715, 0x3feef1a7373aa9cb, 0x3feedea64c123422, 0x3feece086061892d,
    0x3feebfdad5362a27, 0x3feeb42b569d4f82, 0x3feeab07dd485429, 0x3feea47eb03a5585,
    0x3feea09e667f3bcd, 0x3fee9f75e8ec5f74, 0x3feea11473eb0187, 0x3feea589994cce13,
    0x3feeace5422aa0db, 0x3feeb737b0cdc5e5, 0x3feec49182a3f090, 0x3feed503b23e255d,
    0x3feee89f995ad3ad, 0x3feeff76f2fb5e47, 0x3fef199bdd85529c, 0x3fef3720dcef9069,
    0x3fef5818dcfba487, 0x3fef7c97337b9b5f, 0x3fefa4afa2a490da, 0x3fefd0765b6e4540};
constexpr double kExp2Shift = 0x1.8p+47;
constexpr double kExp2Poly[3] = {0x1.c6af84b912394p-5, 0x1.ebfce50fac4f3p-3,
                                 0x1.62e42ff0c52d6p-1};
constexpr uint32_t kOff = 0x3f330000u;
}  // namespace libmf

BSGP_HD uint32_t fbits(float x) {
  uint32_t u;
  memcpy(&u, &x, 4);
  return u;
}
BSGP_HD float bitsf(uint32_t u) {
  float x;
  memcpy(&x, &u, 4);
  return x;
}

// logf(x) (glibc e_logf.c): log(x) = log1p(z/c - 1) + log(c) + k*ln2
BSGP_HD float libm_logf(float x) {
  using namespace libmf;
  uint32_t ix = fbits(x);
  if (ix == 0x3f800000u) return 0.0f;
  if (ix - 0x00800000u >= 0x7f800000u - 0x00800000u) {
    if (ix * 2 == 0) return -INFINITY;
    if (ix == 0x7f800000u) return x;
    if ((ix & 0x80000000u) || ix * 2 >= 0xff000000u) return NAN;
    ix = fbits(x * 0x1p23f);  // subnormal: normalise
    ix -= 23u << 23;
  }
  const uint32_t tmp = ix - kOff;
  const int i = (int)((tmp >> 19) % 16);
  const int k = (int32_t)tmp >> 23;
  const uint32_t iz = ix - (tmp & (0x1ffu << 23));
  const double z = (double)bitsf(iz);
  const double r = std::fma(z, kLogTab[i].invc, -1.0);
  const double y0 = std::fma((double)k, kLn2, kLogTab[i].logc);
  const double r2 = r * r;
  double y = std::fma(kLogPoly[1], r, kLogPoly[2]);
  y = std::fma(kLogPoly[0], r2, y);
  y = std::fma(y, r2, y0 + r);
  return (float)y;
}

// powf(x, y) (glibc e_powf.c) for x >= 0 and finite y != 0 -- the float32
// image terms gn**beta; other operands return the IEEE special values.
BSGP_HD float libm_powf(float x, float y) {
  using namespace libmf;
  uint32_t ix = fbits(x);
  const uint32_t iy = fbits(y);
  if (2 * iy - 1 >= 2u * 0x7f800000u - 1) return (float)std::pow((double)x, (double)y);
  if (ix - 0x00800000u >= 0x7f800000u - 0x00800000u) {
    if (2 * ix - 1 >= 2u * 0x7f800000u - 1 || (ix & 0x80000000u))
      return (float)std::pow((double)x, (double)y);  // 0, inf, nan, negative
    ix = fbits(x * 0x1p23f) & 0x7fffffffu;          // subnormal: normalise
    ix -= 23u << 23;
  }
  // log2(x) = log1p(z/c - 1)/ln2 + log2(c) + k
  const uint32_t tmp = ix - kOff;
  const int i = (int)((tmp >> 19) % 16);
  const uint32_t top = tmp & 0xff800000u;
  const uint32_t iz = ix - top;
  const int k = (int32_t)top >> 23;
  const double z = (double)bitsf(iz);
  const double r = std::fma(z, kLogTab[i].invc, -1.0);
  const double y0 = kLog2c[i] + (double)k;
  const double r2 = r * r;
  double q1 = std::fma(kLog2Poly[0], r, kLog2Poly[1]);
  const double p = std::fma(kLog2Poly[2], r, kLog2Poly[3]);
  const double r4 = r2 * r2;
  double q = std::fma(kLog2Poly[4], r, y0);
  q = std::fma(p, r2, q);
  const double logx = std::fma(q1, r4, q);
  const double ylogx = (double)y * logx;
  if (((dbits(ylogx) >> 47) & 0xffff) >= (dbits(126.0) >> 47)) {
    if (ylogx > 0x1.fffffffd1d571p+6) return INFINITY;
    if (ylogx <= -150.0) return 0.0f;
  }
  // exp2(ylogx) = 2^(k/32) * 2^r
  double kd = ylogx + kExp2Shift;
  const uint64_t ki = dbits(kd);
  kd -= kExp2Shift;
  const double rr = ylogx - kd;
  const double s = bitsd(kExp2Tab[ki % 32] + (ki << 47));
  const double zz = std::fma(kExp2Poly[0], rr, kExp2Poly[1]);
  const double rr2 = rr * rr;
  double e = std::fma(kExp2Poly[2], rr, 1.0);
  e = std::fma(zz, rr2, e);
  return (float)(e * s);
}

}  // namespace bsgp
