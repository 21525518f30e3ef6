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
const void* persist_kernel_f32(int K, int mode, bool adapt) {
  return persist_kernel<float>(K, mode, adapt);
}
void persist_kernels_f32(std::vector<const void*>& f) { persist_kernels<float>(f); }

}  // namespace bsgp
