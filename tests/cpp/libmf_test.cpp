// Host test of bsgp::libm_powf / libm_logf (beta-sgp_amd/csrc/bsgp_math.hpp):
// bit for bit against this host's C library powf / logf, which numpy 1.x
// calls for a float32 array's ``**`` and ``np.log`` when its SIMD kernels are
// off (the reference fixtures with suffix _libm, tests/golden/make_golden.py).
//   logf: every positive float32 (every one with argument "full", else every 29th);
//   powf: x over (0, 1] and a band above 1 at the exponents of the
//         application's five beta seeds and a few more.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include "bsgp_math.hpp"

int main(int argc, char** argv) {
  const bool full = argc > 1 && !strcmp(argv[1], "full");
  const uint32_t step = full ? 1 : 29;
  long nlog = 0, bad_log = 0;
  for (uint64_t u = 0; u < 0x7f800001ull; u += step) {
    const float x = bsgp::bitsf((uint32_t)u);
    const float a = logf(x), b = bsgp::libm_logf(x);
    ++nlog;
    if (bsgp::fbits(a) != bsgp::fbits(b)) {
      if (bad_log < 5) printf("logf(%a): libm %a, ours %a\n", x, a, b);
      ++bad_log;
    }
  }
  printf("logf: %ld of %ld differ\n", bad_log, nlog);
  const float ys[] = {1.0881172613560043f, 0.9979165937393577f, 0.9652434498519898f,
                      0.9904367219749186f, 1.0815024541066357f, 1.05f, 0.95f, 1.0248357f,
                      0.5f, 2.0f, -0.5f, 1.0f / 3.0f};
  long npow = 0, bad_pow = 0;
  const uint32_t pstep = full ? 3 : 211;
  for (float y : ys) {
    for (uint32_t u = 0; u <= 0x40000000u; u += pstep) {  // (0, 2]
      const float x = bsgp::bitsf(u);
      const float a = powf(x, y), b = bsgp::libm_powf(x, y);
      ++npow;
      if (bsgp::fbits(a) != bsgp::fbits(b)) {
        if (bad_pow < 5) printf("powf(%a, %a): libm %a, ours %a\n", x, y, a, b);
        ++bad_pow;
      }
    }
  }
  printf("powf: %ld of %ld differ\n", bad_pow, npow);
  const bool ok = !bad_log && !bad_pow;
  if (ok) printf("all ok\n");
  return ok ? 0 : 1;
}
