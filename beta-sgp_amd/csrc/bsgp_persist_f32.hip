// bsgp_persist_f32.hip — the float32-storage build (BSGP_STORAGE_F32) of the
// persistent task-queue solver (k_persist, bsgp_kernels.hpp).
#include <hip/hip_runtime.h>

#include <vector>

#include "bsgp_kernels.hpp"

namespace bsgp {

hipError_t launch_persist_f32(const SolveArgs& a, int K, size_t lds, hipStream_t s,
                              unsigned* queue, unsigned* done, int grid) {
  return launch_persist_t<float>(a, K, lds, s, queue, done, grid);
}
const void* persist_kernel_f32(int K, int mode, bool adapt, bool scalar_bkg) {
  return persist_kernel<float>(K, mode, adapt, scalar_bkg);
}
void persist_kernels_f32(std::vector<const void*>& f) { persist_kernels<float>(f); }
hipError_t persist_phase_prof_f32(unsigned long long* out, int n, int reset) {
#ifdef BSGP_PHASE_PROF
  hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_phase), n * sizeof(unsigned long long));
  if (e == hipSuccess && reset) {
    unsigned long long z[kPhaseSlots] = {};
    e = hipMemcpyToSymbol(HIP_SYMBOL(g_phase), z, sizeof z);
  }
  return e;
#else
  for (int i = 0; i < n; ++i) out[i] = 0;
  (void)reset;
  return hipSuccess;
#endif
}

}  // namespace bsgp
