// Per-sample log-likelihood, its first derivative, the information (negative second derivative) and
// the information's derivative wrt the location parameter, for the latent (Laplace) likelihoods.
//   gaussian        likelihoods.h :8795, 9263, 9937 (aux = error variance)
//   bernoulli_logit likelihoods.h :8724, 9226, 9896, 10187; sigmoid_stable / softplus DF_utils.h:37-60
// Shared by the Vecchia (sparse_kernels.hip) and FITC (fitc_laplace.hip) Laplace paths.
#pragma once

#include <hip/hip_runtime.h>

#include "latent_kernels.h"

namespace gpb_amd {

__device__ __forceinline__ double sigmoid_stable(double x) {
  if (x >= 0.) {
    const double e = exp(-x);
    return 1. / (1. + e);
  }
  const double e = exp(x);
  return e / (1. + e);
}
__device__ __forceinline__ double softplus(double x) { return log1p(exp(-fabs(x))) + fmax(x, 0.); }

__device__ __forceinline__ double lik_loglik(int lik, double aux, double y, double l) {
  if (lik == kLikGaussian) {
    const double r = y - l;
    return -r * r / 2. / aux - 0.91893853320467274178 - 0.5 * log(aux);   // M_LOGSQRT2PI
  }
  return y * l - softplus(l);
}
__device__ __forceinline__ double lik_d1(int lik, double aux, double y, double l) {
  return lik == kLikGaussian ? (y - l) / aux : y - sigmoid_stable(l);
}
__device__ __forceinline__ double lik_info(int lik, double aux, double l) {
  if (lik == kLikGaussian) return 1. / aux;
  const double p = sigmoid_stable(l);
  return p * (1. - p);
}
__device__ __forceinline__ double lik_dinfo(int lik, double l) {
  if (lik == kLikGaussian) return 0.;
  const double p = sigmoid_stable(l);
  return -p * (1. - p) * (2. * p - 1.);
}

}  // namespace gpb_amd
