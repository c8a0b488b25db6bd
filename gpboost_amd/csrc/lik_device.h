// Per-sample log-likelihood, its first derivative, the information (negative second derivative) and
// the information's derivative wrt the location parameter, for the latent (Laplace) likelihoods.
//   gaussian        likelihoods.h :8795, 9263, 9937 (aux = error variance)
//   bernoulli_logit likelihoods.h :8724, 9226, 9896, 10187; sigmoid_stable / softplus DF_utils.h:37-60
//   bernoulli_probit :8708, 9208, 9871, 10171;  poisson :8730, 9230, 9904, 10200
//   gamma           :8740, 9234, 9908, 10228 (aux = shape; log link, the normalizing constant on the host)
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

// DF_utils.h:62-104: normal log-CDF with its tails, inverse Mills ratios phi / Phi and phi / (1 - Phi)
__device__ __forceinline__ double normal_log_pdf(double x) { return -x * x / 2. - 0.91893853320467274178; }
__device__ __forceinline__ double normal_log_cdf(double x) {
  if (x < 0.) {
    const double e = erfc(-x * 0.70710678118654752440);
    if (e > 0.) return -0.69314718055994530942 + log(e);
    const double u = -x, u2 = u * u;   // extreme left tail: asymptotic series
    const double series = 1. - 1. / u2 + 3. / (u2 * u2);
    return -0.5 * u2 - log(u) - 0.5 * log(2. * 3.14159265358979323846) + log(series);
  }
  const double Q = 0.5 * erfc(x * 0.70710678118654752440);
  if (Q == 0.) return 0.;
  return log1p(-Q);
}
__device__ __forceinline__ double mills_phi(double x) { return exp(normal_log_pdf(x) - normal_log_cdf(x)); }
__device__ __forceinline__ double mills_one_minus_phi(double x) { return exp(normal_log_pdf(x) - normal_log_cdf(-x)); }

// log-likelihood without the normalizing constant (the Poisson -log y! is added on the host)
__device__ __forceinline__ double lik_loglik(int lik, double aux, double y, double l) {
  if (lik == kLikGaussian) {
    const double r = y - l;
    return -r * r / 2. / aux - 0.91893853320467274178 - 0.5 * log(aux);   // M_LOGSQRT2PI
  }
  if (lik == kLikBernoulliProbit) return y == 0. ? normal_log_cdf(-l) : normal_log_cdf(l);   // :8708-8715
  if (lik == kLikPoisson) return y * l - exp(l);                                              // :8730-8737
  if (lik == kLikGamma) return -aux * (l + y * exp(-l));                                      // :8740-8748
  return y * l - softplus(l);
}
__device__ __forceinline__ double lik_d1(int lik, double aux, double y, double l) {
  if (lik == kLikGaussian) return (y - l) / aux;
  if (lik == kLikBernoulliProbit) return y == 0. ? -mills_one_minus_phi(l) : mills_phi(l);    // :9208-9215
  if (lik == kLikPoisson) return y - exp(l);                                                  // :9230-9232
  if (lik == kLikGamma) return aux * (y * exp(-l) - 1.);                                      // :9234-9236
  return y - sigmoid_stable(l);
}
// information (negative second derivative), likelihoods.h:9871-9906
__device__ __forceinline__ double lik_info(int lik, double aux, double y, double l) {
  if (lik == kLikGaussian) return 1. / aux;
  if (lik == kLikBernoulliProbit) {
    if (y == 0.) {
      const double r = mills_one_minus_phi(l);
      return -r * (l - r);
    }
    const double r = mills_phi(l);
    return r * (l + r);
  }
  if (lik == kLikPoisson) return exp(l);
  if (lik == kLikGamma) return aux * y * exp(-l);   // :9908-9910
  const double p = sigmoid_stable(l);
  return p * (1. - p);
}
// derivative of the information wrt the location parameter, likelihoods.h:10165-10195
__device__ __forceinline__ double lik_dinfo(int lik, double aux, double y, double l) {
  if (lik == kLikGaussian) return 0.;
  if (lik == kLikGamma) return -aux * y * exp(-l);   // :10228-10233
  if (lik == kLikBernoulliProbit) {
    const double x2 = l * l;
    if (y == 0.) {
      const double r = mills_one_minus_phi(l);
      return -r * (1. - x2 + r * (3. * l - 2. * r));
    }
    const double r = mills_phi(l);
    return -r * (x2 - 1. + r * (3. * l + 2. * r));
  }
  if (lik == kLikPoisson) return exp(l);
  const double p = sigmoid_stable(l);
  return -p * (1. - p) * (2. * p - 1.);
}

}  // namespace gpb_amd
