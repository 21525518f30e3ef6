// bsgp_persist.hip — the float64-storage build of the persistent task-queue
// solver (k_persist, bsgp_kernels.hpp) and the dispatch of both storage
// builds (bsgp_persist_f32.hip holds the float32 one).  Own translation units:
// every k_persist instantiation inlines a whole SGP iteration.
//
// Reference hot path: restoration/sgp.py:748-882 (one iteration of the main
// loop of sgp_betaDiv; :302-425 for sgp), run for every image of a batch.
#include <hip/hip_runtime.h>

#include <vector>

#ifndef BSGP_LS1_K2
#define BSGP_LS1_K2 1  // (bsgp_kernels.hpp)
#endif
#include "bsgp_kernels.hpp"

namespace bsgp {

hipError_t launch_persist_f32(const SolveArgs& a, int K, size_t lds, hipStream_t s,
                              unsigned* queue, unsigned* done, int grid);
const void* persist_kernel_f32(int K, int mode, bool adapt, bool scalar_bkg);
void persist_kernels_f32(std::vector<const void*>& f);

static int persist_mode(const SolveArgs& a, bool* adapt) {
  const bsgp_params& P = a.prm;
  *adapt = P.adapt_beta && P.variant == BSGP_VARIANT_BETA;
  const bool special = a.in.beta0 ? !P.beta0_general : (P.betaParam == 0.0 || P.betaParam == 1.0);
  return P.variant == BSGP_VARIANT_KL ? 0 : special ? -1 : P.gn_f32 ? 4 : 3;
}

hipError_t launch_persist(const SolveArgs& a, int K, size_t lds, hipStream_t s, unsigned* queue,
                          unsigned* done, int grid) {
  if (a.g.coop) return bsgp_c512_launch_persist(&a, K, lds, s, queue, done, grid);
  if (app_static_plan(a.g, a.storage))
    return bsgp_app_launch_persist(&a, K, lds, s, queue, done, grid);
  if (a.storage == BSGP_STORAGE_F32) return launch_persist_f32(a, K, lds, s, queue, done, grid);
  return launch_persist_t<double>(a, K, lds, s, queue, done, grid);
}

// Workgroups of the persistent kernel a solve would launch that one CU holds.
hipError_t persist_resident_per_cu(const SolveArgs& a, int K, size_t lds, int* per_cu) {
  if (a.g.coop) return bsgp_c512_persist_resident(&a, K, lds, per_cu);
  if (app_static_plan(a.g, a.storage)) return bsgp_app_persist_resident(&a, K, lds, per_cu);
  bool adapt = false;
  const int mode = persist_mode(a, &adapt);
  const bool sb = !a.prm.bkg_is_map;
  const void* f = a.storage == BSGP_STORAGE_F32 ? persist_kernel_f32(K, mode, adapt, sb)
                                                : persist_kernel<double>(K, mode, adapt, sb);
  return hipOccupancyMaxActiveBlocksPerMultiprocessor(per_cu, f, kBlock, lds);
}

// phase-profile counters of this translation unit's kernels (-DBSGP_PHASE_PROF;
// phase_prof in bsgp_solver.hip adds them)
hipError_t persist_phase_prof_f32(unsigned long long* out, int n, int reset);
hipError_t persist_phase_prof(unsigned long long* out, int n, int reset) {
#ifdef BSGP_PHASE_PROF
  hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_phase), n * sizeof(unsigned long long));
  if (e == hipSuccess && reset) {
    unsigned long long z[kPhaseSlots] = {};
    e = hipMemcpyToSymbol(HIP_SYMBOL(g_phase), z, sizeof z);
  }
  if (e == hipSuccess) {
    unsigned long long c[kPhaseSlots] = {};
    e = persist_phase_prof_f32(c, n, reset);
    for (int i = 0; i < n; ++i) out[i] += c[i];
  }
  if (e == hipSuccess) {
    unsigned long long c[kPhaseSlots] = {};
    e = bsgp_app_phase_prof(c, n, reset);
    for (int i = 0; i < n; ++i) out[i] += c[i];
  }
  return e;
#else
  for (int i = 0; i < n; ++i) out[i] = 0;
  (void)reset;
  return hipSuccess;
#endif
}

void persist_kernels_all(std::vector<const void*>& f) {
  persist_kernels<double>(f);
  persist_kernels_f32(f);
}

}  // namespace bsgp
