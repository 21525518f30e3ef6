/* TEST INFRASTRUCTURE ONLY (oracle/): the C library's float32 powf / logf over
 * arrays, for sgp_oracle.py's LIBM_F32 mode.
 *
 * numpy 1.26 with its SIMD float32 kernels disabled (NPY_DISABLE_CPU_FEATURES
 * naming AVX2 and the AVX-512 features; tests/golden/make_golden.py) evaluates
 * a float32 array's ``x ** b`` and ``np.log(x)`` element by element with
 * powf(x, (float)b) and logf(x) -- measured bit for bit here on 4e5 values.
 * These are the float32 terms of the reference's betaDiv (sgp.py:458) and
 * betaDivDeriv (sgp.py:495) on a float32 image.  Built by __graft_entry__.build()
 * into oracle/_build/ and loaded with ctypes; nothing else links it. */
#include <math.h>

void bsgp_orc_powf(const float* x, float b, float* out, long n) {
  for (long i = 0; i < n; ++i) out[i] = powf(x[i], b);
}

void bsgp_orc_logf(const float* x, float* out, long n) {
  for (long i = 0; i < n; ++i) out[i] = logf(x[i]);
}
