// Covariance kernels and their derivatives on the reference's transformed scale,
// shared by host and device code.
//   C(r)       : cov_fcts.h:1681-1745 (CovarianceMaternShape0_5 / 1_5 / 2_5, CovarianceGaussian)
//   dC/dlog phi: cov_fcts.h:1750-1786 (DetermineConstantsForGradient, transf_scale=true)
//                and :2116-2143 (GradientRangeMaternShape*, GradientRangeGaussian)
//   parameters : var = sigma1^2 / sigma2, phi = range transform (cov_fcts.h:438-460)
#pragma once

#include <hip/hip_runtime.h>

namespace gpb_amd {

enum CovType : int { kMatern05 = 0, kMatern15 = 1, kMatern25 = 2, kGaussian = 3 };

template <int COV>
__host__ __device__ __forceinline__ void cov_dcov(double r, double var, double phi, double& c, double& dc) {
  if constexpr (COV == kMatern05) {
    const double e = exp(-phi * r);
    c = var * e;
    dc = -phi * r * c;
  } else if constexpr (COV == kMatern15) {
    const double x = phi * r;
    const double e = exp(-x);
    c = var * (1. + x) * e;
    dc = -var * x * x * e;
  } else if constexpr (COV == kMatern25) {
    const double x = phi * r;
    const double e = exp(-x);
    c = var * (1. + x + x * x / 3.) * e;
    dc = -var * x * x / 3. * (1. + x) * e;
  } else {
    const double e = exp(-phi * r * r);
    c = var * e;
    dc = -phi * r * r * c;
  }
}

// ---- device forms for the row kernels: the same operation sequences as the ROCm device library's
// sqrt and exp (so the same bits on their common range), minus the range handling these arguments
// never need. sqrt: no denormal rescaling (squared distances are 0 or far above 2^-767; 0 gives 0
// exactly: the rsq seed is taken of max(s, 1e-300) and every refinement uses s itself). exp: the
// argument is <= 0 (no overflow branch); it is clamped at -1075, below which the result is 0 either
// way (2^-1551 after the final ldexp), replacing the underflow compare-and-selects.
__device__ __forceinline__ double sqrt_nonneg(double s) {
  const double y0 = __builtin_amdgcn_rsq(fmax(s, 1e-300));
  double g = s * y0;
  double h = y0 * 0.5;
  const double r = fma(-h, g, 0.5);
  g = fma(g, r, g);
  double e = fma(-g, g, s);
  h = fma(h, r, h);
  g = fma(e, h, g);
  e = fma(-g, g, s);
  return fma(e, h, g);
}

__device__ __forceinline__ double exp_nonpos(double x) {
  x = fmax(x, -1075.);
  const double n = __builtin_rint(x * 0x1.71547652b82fep+0);
  double t = fma(-0x1.62e42fefa39efp-1, n, x);
  t = fma(-0x1.abc9e3b39803fp-56, n, t);
  double p = fma(0x1.ade156a5dcb37p-26, t, 0x1.28af3fca7ab0cp-22);
  p = fma(t, p, 0x1.71dee623fde64p-19);
  p = fma(t, p, 0x1.a01997c89e6b0p-16);
  p = fma(t, p, 0x1.a01a014761f6ep-13);
  p = fma(t, p, 0x1.6c16c1852b7b0p-10);
  p = fma(t, p, 0x1.1111111122322p-7);
  p = fma(t, p, 0x1.55555555502a1p-5);
  p = fma(t, p, 0x1.5555555555511p-3);
  p = fma(t, p, 0x1.000000000000bp-1);
  p = fma(t, p, 1.);
  p = fma(t, p, 1.);
  return __builtin_amdgcn_ldexp(p, (int)n);
}

// cov_dcov on the squared distance with the device forms above (identical formulas)
template <int COV>
__device__ __forceinline__ void cov_dcov_sq(double s, double var, double phi, double& c, double& dc) {
  const double r = sqrt_nonneg(s);
  if constexpr (COV == kMatern05) {
    const double e = exp_nonpos(-phi * r);
    c = var * e;
    dc = -phi * r * c;
  } else if constexpr (COV == kMatern15) {
    const double x = phi * r;
    const double e = exp_nonpos(-x);
    c = var * (1. + x) * e;
    dc = -var * x * x * e;
  } else if constexpr (COV == kMatern25) {
    const double x = phi * r;
    const double e = exp_nonpos(-x);
    c = var * (1. + x + x * x / 3.) * e;
    dc = -var * x * x / 3. * (1. + x) * e;
  } else {
    const double e = exp_nonpos(-phi * r * r);
    c = var * e;
    dc = -phi * r * r * c;
  }
}

}  // namespace gpb_amd
