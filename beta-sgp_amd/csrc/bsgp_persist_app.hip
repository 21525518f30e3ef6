// bsgp_persist_app.hip — the persistent task-queue solver (k_persist,
// bsgp_kernels.hpp; float64 storage, per-wave transforms) built with the
// compile-time 400- / 480-point transforms (BSGP_FFT_STATIC_APP, bsgp_fft.hpp)
// for the application's subdivisions: 375^2 tiles and the 450^2 CROWDED frame
// with the 31x31 DIAPL PSF in linear mode sit on 400- / 480-point grids
// (application_sgp_subdivisions.py:43-50).  A build of its own (namespace
// bsgp_app, like the cooperative build's bsgp_c512) so that the kernels of
// every other plan keep their code: inlined into them the extra stages cost
// C3 0.7 % (A/B), while the 375^2 tiles gain 3.6 % and the 450^2 frames ~9 %.
//
// Reference hot path: restoration/sgp.py:748-882 (one iteration of the main
// loop of sgp_betaDiv; :302-425 for sgp), run for every image of a batch.
#include <hip/hip_runtime.h>

#include <vector>

#define BSGP_FFT_STATIC_APP 1
// These plans run two workgroups per CU (their transform buffers and LDS
// twiddles fill the LDS), so the register budget is that of two waves per
// SIMD, not the three the other per-wave plans get: 375^2 tiles 97.2 k ->
// 99.9 k image-it/s (A/B, profiles/r04/ab_round4.txt).  The host sizes the
// grid from the occupancy the runtime reports, whatever the plan.
#define BSGP_PERSIST_ATTR __attribute__((amdgpu_waves_per_eu(2)))
// With that budget the row passes keep two operand batches in flight (the
// PIPE knobs of bsgp_kernels.hpp): 375^2 +3.1 %, 450^2 +3.8 % (A/B), and
// the inverse passes issue their first batch before the transform (PRE):
// +0.9 % / +0.7 %.
#define BSGP_LS1_PIPE true
#define BSGP_LSACC_PIPE true
#define BSGP_BB_PIPE true
#define BSGP_LS1_PRE true
#define BSGP_BB_PRE true
#define bsgp bsgp_app
#include "bsgp_kernels.hpp"

namespace bsgp {

static int persist_mode_app(const SolveArgs& a, bool* adapt) {
  const bsgp_params& P = a.prm;
  *adapt = P.adapt_beta && P.variant == BSGP_VARIANT_BETA;
  const bool special = a.in.beta0 ? !P.beta0_general : (P.betaParam == 0.0 || P.betaParam == 1.0);
  return P.variant == BSGP_VARIANT_KL ? 0 : special ? -1 : P.gn_f32 ? 4 : 3;
}

}  // namespace bsgp

extern "C" {

size_t bsgp_app_args_size(void) { return sizeof(bsgp_app::SolveArgs); }

hipError_t bsgp_app_launch_persist(const void* a, int K, size_t lds, hipStream_t s,
                                   unsigned* queue, unsigned* done, int grid) {
  const bsgp_app::SolveArgs& A = *static_cast<const bsgp_app::SolveArgs*>(a);
  return bsgp_app::launch_persist_t<double>(A, K, lds, s, queue, done, grid);
}

hipError_t bsgp_app_persist_resident(const void* a, int K, size_t lds, int* per_cu) {
  const bsgp_app::SolveArgs& A = *static_cast<const bsgp_app::SolveArgs*>(a);
  bool adapt = false;
  const int mode = bsgp_app::persist_mode_app(A, &adapt);
  return hipOccupancyMaxActiveBlocksPerMultiprocessor(
      per_cu, bsgp_app::persist_kernel<double>(K, mode, adapt, !A.prm.bkg_is_map),
      bsgp_app::kBlock, lds);
}

hipError_t bsgp_app_persist_set_lds_limit(size_t bytes) {
  std::vector<const void*> fns;
  bsgp_app::persist_kernels<double>(fns);
  for (const void* f : fns) {
    hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

// phase-profile counters of this build (-DBSGP_PHASE_PROF; persist_phase_prof adds them)
hipError_t bsgp_app_phase_prof(unsigned long long* out, int n, int reset) {
#ifdef BSGP_PHASE_PROF
  hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(bsgp_app::g_phase),
                                     n * sizeof(unsigned long long));
  if (e == hipSuccess && reset) {
    unsigned long long z[bsgp_app::kPhaseSlots] = {};
    e = hipMemcpyToSymbol(HIP_SYMBOL(bsgp_app::g_phase), z, sizeof z);
  }
  return e;
#else
  for (int i = 0; i < n; ++i) out[i] = 0;
  (void)reset;
  return hipSuccess;
#endif
}

}  // extern "C"
