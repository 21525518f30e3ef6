// bsgp_internal.hpp — structures shared by the kernels (bsgp_solver.hip) and
// the C-ABI host layer (bsgp_api.hip).  Not part of the public interface.
#pragma once

#include <hip/hip_runtime.h>

#include "../../include/bsgp.h"
#include "bsgp_device.hpp"

namespace bsgp {

// Everything one launch of the persistent solver needs (passed by value).
struct SolveArgs {
  Geo g;
  bsgp_params prm;
  bsgp_inputs in;
  bsgp_outputs out;
  int B;
  int* queue;          // image dequeue counter, zeroed before the launch
  double* ws;          // per-workgroup slots
  size_t slot_stride;  // doubles per slot
  size_t vec_stride;   // doubles per image vector (N rounded up to 32)
  size_t lds_fft_bytes;
};

hipError_t launch_solve(const SolveArgs& a, int grid, size_t lds, hipStream_t s);
hipError_t launch_build_tf(const Geo& g, const double* kc, cd* spec, cd* tf, double scale,
                           int conj, size_t lds, hipStream_t s);
hipError_t launch_apply_op(const Geo& g, int B, int transpose, const double* x, double* out,
                           cd* specws, size_t spec_stride, int grid, size_t lds, hipStream_t s);
hipError_t launch_project_df(int n, double b, const double* c, const double* dia, ProjClip clip,
                             double lam0, double dlam0, double tol_lam, int biter, int siter,
                             int max_projs, double* x, double* info, hipStream_t s);
hipError_t launch_beta_div(int n, const double* y, const double* x, double beta, double* out,
                           hipStream_t s);
hipError_t launch_beta_div_deriv(int64_t n, const double* y, const double* x, double beta,
                                 double* out, hipStream_t s);
hipError_t launch_grad_parts(int64_t n, const double* den, const double* gn, double beta,
                             double* pow1, double* w, hipStream_t s);
hipError_t set_solver_lds_limit(size_t bytes);

}  // namespace bsgp
