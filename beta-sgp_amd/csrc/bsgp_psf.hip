// bsgp_psf.hip — PSF stamps from the DIAPL model on the device.
//
// One workgroup per stamp: the local coefficient vector at the stamp's field
// position (init_psf's spatial expansion, psf_calculate.py:140-165) goes to
// LDS, every thread evaluates pixels of the (2hw+1)^2 stamp (calc_psf_pix,
// :52-87, at x = column offset, y = row offset as get_psf_mat, :89-107,
// indexes them), and with `normalize` one lane forms numpy's pairwise sum of
// the stamp and the workgroup divides (normalize_psf_mat, :129-137).  The
// stamps can go straight into bsgp_plan_set_psfs, so a spatially varying PSF
// per subdivision never leaves HBM.  Work per stamp is ~1k pixels x ngauss
// exp(): tiny next to a solve; the point is removing the host round trip.
#include <hip/hip_runtime.h>

#include "bsgp_internal.hpp"
#include "bsgp_psf.hpp"

namespace bsgp {

__global__ void __launch_bounds__(256) psf_stamps_kernel(PsfModel M, const double* xy,
                                                         int spatial, int normalize,
                                                         double* out) {
  __shared__ double loc[kPsfMaxLocal];
  __shared__ double s_sum;
  const int S = 2 * M.hw + 1, S2 = S * S;
  double* st = out + (size_t)blockIdx.x * S2;
  if ((int)threadIdx.x < M.ncomp) {
    loc[threadIdx.x] = spatial ? psf_local_coef(M, threadIdx.x, xy[2 * blockIdx.x],
                                                xy[2 * blockIdx.x + 1])
                               : M.coef[threadIdx.x];
  }
  __syncthreads();
  for (int p = threadIdx.x; p < S2; p += 256) {
    const int i = p / S - M.hw, j = p % S - M.hw;  // row offset i (y), column offset j (x)
    st[p] = psf_pix(M, loc, (double)j, (double)i);
  }
  if (!normalize) return;
  __syncthreads();  // the stamp is in global memory, visible to the workgroup
  if (threadIdx.x == 0) s_sum = np_pairwise_sum(st, S2);
  __syncthreads();
  const double s = s_sum;
  for (int p = threadIdx.x; p < S2; p += 256) st[p] = st[p] / s;
}

hipError_t launch_psf_stamps(const PsfModel& m, const double* xy, int n, int spatial,
                             int normalize, double* out, hipStream_t s) {
  hipLaunchKernelGGL(psf_stamps_kernel, dim3(n), dim3(256), 0, s, m, xy, spatial, normalize,
                     out);
  return hipGetLastError();
}

}  // namespace bsgp
