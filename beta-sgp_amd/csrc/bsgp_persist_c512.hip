// bsgp_persist_c512.hip — the persistent task-queue solver (k_persist,
// bsgp_kernels.hpp) for cooperative plans (Geo::coop): the application's
// 375^2 / 450^2 subdivisions on their 400- / 480-point grids and other
// transforms too long for one wave's share of the LDS.  The same task loop as
// the per-wave build (one task = one iteration of one image, slot order or
// ready ring, agent-scope hand-offs), with the cooperative phase code of the
// 512-thread phase kernels (bsgp_solver_c512.hip): thread-group transforms,
// column groups for A's column pass.  Results are bit-identical to those
// phase kernels.  The float64-storage kernels live here, the float32 ones in
// bsgp_persist_c512_f32.hip (parallel compiles).
//
// Reference hot path: restoration/sgp.py:748-882 (one iteration of the main
// loop of sgp_betaDiv; :302-425 for sgp), run for every image of a batch.
#include <hip/hip_runtime.h>

#include <vector>

#define BSGP_BLOCK 512
#define bsgp bsgp_c512
#include "bsgp_kernels.hpp"

namespace bsgp {

hipError_t launch_persist_coop_f32(const SolveArgs& a, int K, size_t lds, hipStream_t s,
                                   unsigned* queue, unsigned* done, int grid);
const void* persist_kernel_coop_f32(int K, int mode, bool adapt);
void persist_kernels_coop_f32(std::vector<const void*>& f);

static int persist_mode_coop(const SolveArgs& a, bool* adapt) {
  const bsgp_params& P = a.prm;
  *adapt = P.adapt_beta && P.variant == BSGP_VARIANT_BETA;
  const bool special = a.in.beta0 ? !P.beta0_general : (P.betaParam == 0.0 || P.betaParam == 1.0);
  return P.variant == BSGP_VARIANT_KL ? 0 : special ? -1 : P.gn_f32 ? 4 : 3;
}

}  // namespace bsgp

extern "C" {

hipError_t bsgp_c512_launch_persist(const void* a, int K, size_t lds, hipStream_t s,
                                    unsigned* queue, unsigned* done, int grid) {
  const bsgp_c512::SolveArgs& A = *static_cast<const bsgp_c512::SolveArgs*>(a);
  if (A.storage == BSGP_STORAGE_F32)
    return bsgp_c512::launch_persist_coop_f32(A, K, lds, s, queue, done, grid);
  return bsgp_c512::launch_persist_t<double, true>(A, K, lds, s, queue, done, grid);
}

// Workgroups of the cooperative persistent kernel a solve would launch that
// one CU holds at once.
hipError_t bsgp_c512_persist_resident(const void* a, int K, size_t lds, int* per_cu) {
  const bsgp_c512::SolveArgs& A = *static_cast<const bsgp_c512::SolveArgs*>(a);
  bool adapt = false;
  const int mode = bsgp_c512::persist_mode_coop(A, &adapt);
  const void* f = A.storage == BSGP_STORAGE_F32
                      ? bsgp_c512::persist_kernel_coop_f32(K, mode, adapt)
                      : bsgp_c512::persist_kernel<double, true>(K, mode, adapt);
  return hipOccupancyMaxActiveBlocksPerMultiprocessor(per_cu, f, bsgp_c512::kBlock, lds);
}

hipError_t bsgp_c512_persist_set_lds_limit(size_t bytes) {
  std::vector<const void*> fns;
  bsgp_c512::persist_kernels<double, true>(fns);
  bsgp_c512::persist_kernels_coop_f32(fns);
  for (const void* f : fns) {
    hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

}  // extern "C"
