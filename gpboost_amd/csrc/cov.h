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

}  // namespace gpb_amd
