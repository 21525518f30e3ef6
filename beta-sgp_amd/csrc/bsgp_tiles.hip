// bsgp_tiles.hip — the data paths either side of the solver:
//
//  * subdivision tiles: extraction of overlapping tiles from a field into the
//    [n][th][tw] batch the solver takes (restoration/utils.py:375-386,
//    create_subdivisions / Cutout2D of calculate_slice_bboxes boxes,
//    utils.py:332-372), and the mean co-add of solved tiles back into a
//    mosaic with its footprint (the same-WCS case of reproject_and_coadd,
//    utils.py:389-395, combine_function='mean', without background matching);
//  * FITS data blocks: big-endian BITPIX 8/16/32/64/-32/-64 samples with
//    BSCALE/BZERO to f64 on the device, so raw file bytes go to HBM with one
//    copy and no host-side decode.
//
// All three are HBM-bound byte/element streams: coalesced along image rows,
// one workgroup per (tile, row band) or per pixel block, no LDS beyond the box
// table of the co-add.
#include <hip/hip_runtime.h>

#include "bsgp_internal.hpp"

namespace bsgp {

// ---------------------------------------------------------- tile extraction
// out[t][r][c] = img[(y0_t + r) * W + x0_t + c]; boxes[t] = {x0, y0, x1, y1}
// (xyxy as calculate_slice_bboxes returns them), every box th x tw inside the
// image (checked on the host).  Grid: (n * th) blocks, one tile row each.
__global__ void __launch_bounds__(256) extract_tiles_kernel(const double* img, int W,
                                                            const int* boxes, int th, int tw,
                                                            double* out) {
  const int t = blockIdx.x / th, r = blockIdx.x % th;
  const int x0 = boxes[4 * t], y0 = boxes[4 * t + 1];
  const double* src = img + (size_t)(y0 + r) * W + x0;
  double* dst = out + ((size_t)t * th + r) * tw;
  for (int c = threadIdx.x; c < tw; c += 256) dst[c] = src[c];
}

// ---------------------------------------------------------------- co-add
// mean[y][x] = sum_t tile_t[y - y0_t][x - x0_t] / count, count = number of
// boxes covering (y, x) (the footprint); pixels no box covers get 0 and
// footprint 0.  Tiles are summed in index order, so the mosaic is
// deterministic (bit-identical to the numpy restatement in oracle/).  The box
// table is staged in LDS; each thread owns one output pixel.
__global__ void __launch_bounds__(256) coadd_tiles_kernel(const double* tiles, int n, int th,
                                                          int tw, const int* boxes, int H, int W,
                                                          double* mean, double* footprint) {
  extern __shared__ int sbox[];
  for (int i = threadIdx.x; i < 4 * n; i += 256) sbox[i] = boxes[i];
  __syncthreads();
  const int64_t N = (int64_t)H * W;
  for (int64_t p = blockIdx.x * (int64_t)256 + threadIdx.x; p < N; p += (int64_t)gridDim.x * 256) {
    const int y = (int)(p / W), x = (int)(p % W);
    double s = 0.0;
    int cnt = 0;
    for (int t = 0; t < n; ++t) {
      const int x0 = sbox[4 * t], y0 = sbox[4 * t + 1], x1 = sbox[4 * t + 2], y1 = sbox[4 * t + 3];
      if (x >= x0 && x < x1 && y >= y0 && y < y1) {
        s += tiles[((size_t)t * th + (y - y0)) * tw + (x - x0)];
        ++cnt;
      }
    }
    mean[p] = cnt ? s / cnt : 0.0;
    if (footprint) footprint[p] = (double)cnt;
  }
}

// ------------------------------------------------------------ FITS samples
// Big-endian sample i of a FITS primary data array to f64:
// value = BZERO + BSCALE * raw (FITS standard §5.3); IEEE samples are
// byte-swapped and widened exactly.
template <int BITPIX>
__device__ __forceinline__ double fits_sample(const unsigned char* b, int64_t i) {
  if constexpr (BITPIX == 8) {
    return (double)b[i];
  } else if constexpr (BITPIX == 16) {
    const unsigned short u = (unsigned short)((b[2 * i] << 8) | b[2 * i + 1]);
    return (double)(short)u;
  } else if constexpr (BITPIX == 32 || BITPIX == -32) {
    const unsigned int u = __builtin_bswap32(reinterpret_cast<const unsigned int*>(b)[i]);
    if constexpr (BITPIX == 32) return (double)(int)u;
    return (double)__uint_as_float(u);
  } else {
    const unsigned long long u =
        __builtin_bswap64(reinterpret_cast<const unsigned long long*>(b)[i]);
    if constexpr (BITPIX == 64) return (double)(long long)u;
    return __longlong_as_double((long long)u);
  }
}

template <int BITPIX>
__global__ void __launch_bounds__(256) fits_to_f64_kernel(const unsigned char* raw, int64_t n,
                                                          double bscale, double bzero,
                                                          int scaled, double* out) {
  for (int64_t i = blockIdx.x * (int64_t)256 + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * 256) {
    const double v = fits_sample<BITPIX>(raw, i);
    out[i] = scaled ? bzero + bscale * v : v;
  }
}

hipError_t launch_extract_tiles(const double* img, int W, const int* boxes, int n, int th, int tw,
                                double* out, hipStream_t s) {
  hipLaunchKernelGGL(extract_tiles_kernel, dim3(n * th), dim3(256), 0, s, img, W, boxes, th, tw,
                     out);
  return hipGetLastError();
}

hipError_t launch_coadd_tiles(const double* tiles, int n, int th, int tw, const int* boxes, int H,
                              int W, double* mean, double* footprint, hipStream_t s) {
  const int64_t N = (int64_t)H * W;
  int64_t g = (N + 255) / 256;
  if (g > 8192) g = 8192;
  hipLaunchKernelGGL(coadd_tiles_kernel, dim3((unsigned)g), dim3(256), 4 * n * sizeof(int), s,
                     tiles, n, th, tw, boxes, H, W, mean, footprint);
  return hipGetLastError();
}

hipError_t launch_fits_to_f64(const void* raw, int64_t n, int bitpix, double bscale, double bzero,
                              double* out, hipStream_t s) {
  const unsigned char* b = static_cast<const unsigned char*>(raw);
  int64_t g = (n + 255) / 256;
  if (g > 16384) g = 16384;
  if (g < 1) g = 1;
  const int scaled = (bscale != 1.0 || bzero != 0.0) ? 1 : 0;
  const dim3 grid((unsigned)g), block(256);
  switch (bitpix) {
    case 8: hipLaunchKernelGGL(fits_to_f64_kernel<8>, grid, block, 0, s, b, n, bscale, bzero, scaled, out); break;
    case 16: hipLaunchKernelGGL(fits_to_f64_kernel<16>, grid, block, 0, s, b, n, bscale, bzero, scaled, out); break;
    case 32: hipLaunchKernelGGL(fits_to_f64_kernel<32>, grid, block, 0, s, b, n, bscale, bzero, scaled, out); break;
    case 64: hipLaunchKernelGGL(fits_to_f64_kernel<64>, grid, block, 0, s, b, n, bscale, bzero, scaled, out); break;
    case -32: hipLaunchKernelGGL(fits_to_f64_kernel<-32>, grid, block, 0, s, b, n, bscale, bzero, scaled, out); break;
    default: hipLaunchKernelGGL(fits_to_f64_kernel<-64>, grid, block, 0, s, b, n, bscale, bzero, scaled, out); break;
  }
  return hipGetLastError();
}

}  // namespace bsgp
