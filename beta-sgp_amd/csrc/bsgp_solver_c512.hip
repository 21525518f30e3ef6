// bsgp_solver_c512.hip — the cooperative (long-transform) builds of the phase
// kernels with 512-thread workgroups.
//
// Plans whose rows or columns are too long for one wave's share of the LDS
// (Geo::coop: the 2048^2 field of config C4, the application's 375^2/450^2
// subdivisions on their 400-/480-point grids) run every transform on the
// whole workgroup and hold one or two workgroups per CU (the two FFT buffers
// of a 2048-point transform are 64 KiB).  At 256 threads that is one wave per
// SIMD: the pixel streams and row batches of those kernels have too few loads
// in flight.  This translation unit compiles the same kernels (bsgp_kernels.hpp)
// with kBlock = 512, two waves per SIMD per workgroup, at the same LDS.
// Measured on C4 (2048^2, float32 storage, team of 256): 1539 -> 1657 it/s.
//
// Every kBlock-dependent type and kernel lives in its own namespace
// (bsgp_c512) so the two builds do not collide; the host reaches them through
// the C-linkage launchers below, which take the SolveArgs of bsgp_api.hip
// (same header, same layout: checked at plan creation by bsgp_c512_args_size).
#include <hip/hip_runtime.h>

#include <vector>

#define BSGP_BLOCK 512
#define bsgp bsgp_c512
// the column kernel keeps two 512-thread workgroups per CU (<= 128 VGPRs): its
// LDS (two 2048-point buffers + the two-level twiddles, 67 KiB) holds two, and
// the twiddle products of the LDS table had taken it to 168 VGPRs (one per CU)
#ifndef BSGP_COL_WPE
#define BSGP_COL_WPE 4
#endif
#if BSGP_COL_WPE
#define BSGP_COL_ATTR __attribute__((amdgpu_waves_per_eu(BSGP_COL_WPE)))
#endif
#include "bsgp_kernels.hpp"

namespace bsgp {

static const SolveArgs& args_of(const void* a) { return *static_cast<const SolveArgs*>(a); }

static void kernels_of(std::vector<const void*>& f, int storage) {
  if (storage == BSGP_STORAGE_F32)
    solver_kernels<true, float>(f);
  else
    solver_kernels<true, double>(f);
}

}  // namespace bsgp

extern "C" {

size_t bsgp_c512_args_size(void) { return sizeof(bsgp_c512::SolveArgs); }
int bsgp_c512_block(void) { return bsgp_c512::kBlock; }
int bsgp_c512_waves(void) { return bsgp_c512::kWaves; }

hipError_t bsgp_c512_launch_setup(const void* a, size_t lds, hipStream_t s) {
  const bsgp_c512::SolveArgs& A = bsgp_c512::args_of(a);
  return A.storage == BSGP_STORAGE_F32 ? bsgp_c512::launch_setup_t<true, float>(A, lds, s)
                                       : bsgp_c512::launch_setup_t<true, double>(A, lds, s);
}

hipError_t bsgp_c512_launch_iteration(const void* a, int K, size_t lds, hipStream_t s,
                                      hipEvent_t* ev) {
  const bsgp_c512::SolveArgs& A = bsgp_c512::args_of(a);
  return A.storage == BSGP_STORAGE_F32
             ? bsgp_c512::launch_iteration_t<true, float>(A, K, lds, s, ev)
             : bsgp_c512::launch_iteration_t<true, double>(A, K, lds, s, ev);
}

// Workgroups of every team kernel of the build one CU holds at once.
hipError_t bsgp_c512_team_resident(int storage, size_t lds, int* per_cu) {
  std::vector<const void*> fns;
  bsgp_c512::kernels_of(fns, storage);
  return bsgp_c512::team_resident(fns, lds, per_cu);
}

// phase-profile counters of this build (-DBSGP_PHASE_PROF; bsgp_solver.hip adds them)
hipError_t bsgp_c512_phase_prof(unsigned long long* out, int n, int reset) {
#ifdef BSGP_PHASE_PROF
  hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(bsgp_c512::g_phase),
                                     n * sizeof(unsigned long long));
  if (e == hipSuccess && reset) {
    unsigned long long z[bsgp_c512::kPhaseSlots] = {};
    e = hipMemcpyToSymbol(HIP_SYMBOL(bsgp_c512::g_phase), z, sizeof z);
  }
  return e;
#else
  (void)out;
  (void)n;
  (void)reset;
  return hipSuccess;
#endif
}

hipError_t bsgp_c512_set_lds_limit(size_t bytes) {
  std::vector<const void*> fns = {(const void*)bsgp_c512::k_col<true>};
  bsgp_c512::kernels_of(fns, BSGP_STORAGE_F64);
  bsgp_c512::kernels_of(fns, BSGP_STORAGE_F32);
  for (const void* f : fns) {
    hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

}  // extern "C"
