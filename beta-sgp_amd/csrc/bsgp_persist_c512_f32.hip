// bsgp_persist_c512_f32.hip — the float32-storage build (BSGP_STORAGE_F32) of
// the cooperative plans' persistent solver (bsgp_persist_c512.hip).
#include <hip/hip_runtime.h>

#include <vector>

#define BSGP_BLOCK 512
#define bsgp bsgp_c512
#include "bsgp_kernels.hpp"

namespace bsgp {

hipError_t launch_persist_coop_f32(const SolveArgs& a, int K, size_t lds, hipStream_t s,
                                   unsigned* queue, unsigned* done, int grid) {
  return launch_persist_t<float, true>(a, K, lds, s, queue, done, grid);
}
const void* persist_kernel_coop_f32(int K, int mode, bool adapt) {
  return persist_kernel<float, true>(K, mode, adapt);
}
void persist_kernels_coop_f32(std::vector<const void*>& f) { persist_kernels<float, true>(f); }

}  // namespace bsgp
