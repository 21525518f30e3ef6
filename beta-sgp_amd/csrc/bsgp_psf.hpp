// bsgp_psf.hpp — DIAPL PSF model evaluation (host + device), SURVEY §8f row 4.
//
// The reference turns DIAPL PSF coefficient files into 31x31 stamps with
// psf/psf_calculate.py: a sum of ngauss Gaussians, each times a local
// polynomial of degree ldeg in the pixel offsets (calc_psf_pix, :52-87), whose
// coefficients are themselves polynomials of degree sdeg in the field position
// (init_psf, :140-165: the spatial expansion about (x_orig, y_orig)).  The
// stamp is normalised by its numpy sum (normalize_psf_mat, :129-137).
//
// Everything here follows the reference's operation order (no FMA contraction
// in the build), and the normalising sum is numpy's pairwise summation, so a
// stamp differs from the reference's only by the exp() implementation.
#pragma once

#include <cmath>

#include "bsgp_fft.hpp"  // BSGP_HD

namespace bsgp {

constexpr int kPsfMaxCoef = 384;  // coefficients carried in the kernel arguments
constexpr int kPsfMaxLocal = 128; // ngauss * (ldeg+1)(ldeg+2)/2

struct PsfModel {
  double cosv, sinv, ax, ay;  // rotation and Gaussian widths (file values 5-8)
  double sig2;                // sigma_inc * sigma_inc (psf_calculate.py:87)
  double x_orig, y_orig;      // spatial expansion origin (values 12-13)
  int ngauss, ldeg, sdeg, hw;
  int ncomp;                  // ngauss * (ldeg+1)(ldeg+2)/2 local coefficients
  int ncoef;                  // coefficients supplied
  double coef[kPsfMaxCoef];
};

// Local coefficient vector at field position (x, y): init_psf (:154-165) —
// local[icomp] = sum over spatial terms (m, n) of coef[itot] * dx^m * dy^n,
// itot running over (term, icomp) with icomp fastest.
BSGP_HD double psf_local_coef(const PsfModel& M, int icomp, double x, double y) {
  double v = 0.0;
  int term = 0;
  double a1 = 1.0;
  for (int m = 0; m <= M.sdeg; ++m) {
    double a2 = 1.0;
    for (int n = 0; n <= M.sdeg - m; ++n) {
      v += M.coef[term * M.ncomp + icomp] * a1 * a2;
      ++term;
      a2 *= y - M.y_orig;
    }
    a1 *= x - M.x_orig;
  }
  return v;
}

// calc_psf_pix (:52-87) at pixel offset (x, y) with local coefficients `loc`.
template <class Coef>
BSGP_HD double psf_pix(const PsfModel& M, const Coef& loc, double x, double y) {
  const double x1 = M.cosv * x - M.sinv * y;
  const double y1 = M.sinv * x + M.cosv * y;
  double rr = M.ax * x1 * x1 + M.ay * y1 * y1;
  double pix = 0.0;
  int icomp = 0;
  for (int g = 0; g < M.ngauss; ++g) {
    const double f = exp(rr);
    double a1 = 1.0;
    for (int m = 0; m <= M.ldeg; ++m) {
      double a2 = 1.0;
      for (int n = 0; n <= M.ldeg - m; ++n) {
        pix += loc[icomp] * f * a1 * a2;
        ++icomp;
        a2 *= y;
      }
      a1 *= x;
    }
    rr *= M.sig2;
  }
  return pix;
}

// numpy's pairwise summation of a contiguous double array (what np.sum does
// for the 31x31 stamp): blocks of <= 128 with 8 accumulators, halves split at
// a multiple of 8, evaluated left half first.  Iterative (explicit stack).
BSGP_HD double np_pairwise_block(const double* a, int n) {
  if (n < 8) {
    double r = 0.0;
    for (int i = 0; i < n; ++i) r += a[i];
    return r;
  }
  double r[8];
  for (int j = 0; j < 8; ++j) r[j] = a[j];
  int i = 8;
  for (; i < n - (n % 8); i += 8)
    for (int j = 0; j < 8; ++j) r[j] += a[i + j];
  double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
  for (; i < n; ++i) res += a[i];
  return res;
}

BSGP_HD double np_pairwise_sum(const double* a, int n) {
  int off[40], len[40], stage[40];
  double left[40];
  int sp = 0;
  off[0] = 0;
  len[0] = n;
  stage[0] = 0;
  double ret = 0.0;
  for (;;) {
    if (len[sp] > 128 && stage[sp] == 0) {  // descend into the left half
      int n2 = len[sp] / 2;
      n2 -= n2 % 8;
      stage[sp] = 1;
      off[sp + 1] = off[sp];
      len[sp + 1] = n2;
      stage[sp + 1] = 0;
      ++sp;
      continue;
    }
    ret = np_pairwise_block(a + off[sp], len[sp]);
    for (;;) {  // hand `ret` up the stack
      if (sp == 0) return ret;
      --sp;
      if (stage[sp] == 1) {  // left half done: evaluate the right half
        left[sp] = ret;
        stage[sp] = 2;
        int n2 = len[sp] / 2;
        n2 -= n2 % 8;
        off[sp + 1] = off[sp] + n2;
        len[sp + 1] = len[sp] - n2;
        stage[sp + 1] = 0;
        ++sp;
        break;
      }
      ret = left[sp] + ret;
    }
  }
}

}  // namespace bsgp
