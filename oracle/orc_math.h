// ORACLE TEST INFRASTRUCTURE — NOT PART OF THE PRODUCT.
// Scalar helpers shared by the oracle's restatements (covariance kernels, small dense
// Cholesky). Internal linkage; included by gp_oracle.cpp and gp_oracle_iter.cpp.
#pragma once

#include <cmath>
#include <vector>

#include "gp_oracle.h"

namespace {

// cov_fcts.h:1681-1745 (CovarianceMaternShape0_5/1_5/2_5, CovarianceGaussian)
double cov(int t, double r, double var, double phi) {
  switch (t) {
    case ORC_MATERN05: return var * std::exp(-phi * r);
    case ORC_MATERN15: { double x = phi * r; return var * (1. + x) * std::exp(-x); }
    case ORC_MATERN25: { double x = phi * r; return var * (1. + x + x * x / 3.) * std::exp(-x); }
    case ORC_GAUSSIAN: return var * std::exp(-phi * r * r);
  }
  return 0.;
}

// d cov / d log(phi) on the transformed scale: cov_fcts.h:1750-1786 (cm constants with
// transf_scale=true) and :2116-2143 (GradientRange*).
double dcov_dlogphi(int t, double r, double var, double phi) {
  switch (t) {
    case ORC_MATERN05: return -phi * r * cov(t, r, var, phi);
    case ORC_MATERN15: return -var * phi * phi * r * r * std::exp(-phi * r);
    case ORC_MATERN25: { double x = phi * r; return -var * phi * phi / 3. * r * r * (1. + x) * std::exp(-x); }
    case ORC_GAUSSIAN: return -phi * r * r * cov(t, r, var, phi);
  }
  return 0.;
}

double dist(const double* a, const double* b, int d) {
  double s = 0.;
  for (int k = 0; k < d; ++k) { double t = a[k] - b[k]; s += t * t; }
  return std::sqrt(s);
}

// In-place lower Cholesky of a k x k row-major SPD matrix (Eigen::LLT equivalent math).
bool chol(std::vector<double>& a, int k) {
  for (int j = 0; j < k; ++j) {
    double s = a[j * k + j];
    for (int p = 0; p < j; ++p) s -= a[j * k + p] * a[j * k + p];
    if (!(s > 0.)) return false;
    double ljj = std::sqrt(s);
    a[j * k + j] = ljj;
    for (int i = j + 1; i < k; ++i) {
      double t = a[i * k + j];
      for (int p = 0; p < j; ++p) t -= a[i * k + p] * a[j * k + p];
      a[i * k + j] = t / ljj;
    }
  }
  return true;
}

// Solve (L L^T) x = b in place.
void chol_solve(const std::vector<double>& l, int k, double* b) {
  for (int i = 0; i < k; ++i) {
    double t = b[i];
    for (int p = 0; p < i; ++p) t -= l[i * k + p] * b[p];
    b[i] = t / l[i * k + i];
  }
  for (int i = k - 1; i >= 0; --i) {
    double t = b[i];
    for (int p = i + 1; p < k; ++p) t -= l[p * k + i] * b[p];
    b[i] = t / l[i * k + i];
  }
}

}  // namespace
