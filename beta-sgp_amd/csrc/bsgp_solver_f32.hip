// bsgp_solver_f32.hip — the float32-storage builds (BSGP_STORAGE_F32, SURVEY
// config C4) of the batched beta-SGP phase kernels of bsgp_kernels.hpp: the
// seven iteration vectors in float32, every reduction and scalar in float64.
#include <hip/hip_runtime.h>

#include <vector>

#include "bsgp_kernels.hpp"

namespace bsgp {

hipError_t launch_setup_f32(const SolveArgs& a, size_t lds, hipStream_t s) {
  return a.g.coop ? launch_setup_t<true, float>(a, lds, s) : launch_setup_t<false, float>(a, lds, s);
}
hipError_t launch_iteration_f32(const SolveArgs& a, int K, size_t lds, hipStream_t s,
                                hipEvent_t* ev) {
  return a.g.coop ? launch_iteration_t<true, float>(a, K, lds, s, ev)
                  : launch_iteration_t<false, float>(a, K, lds, s, ev);
}
hipError_t launch_track_f32(const SolveArgs& a, int it, hipStream_t s) {
  return launch_track_t<float>(a, it, s);
}
void solver_kernels_f32(std::vector<const void*>& f, bool coop) {
  if (coop)
    solver_kernels<true, float>(f);
  else
    solver_kernels<false, float>(f);
}

}  // namespace bsgp
