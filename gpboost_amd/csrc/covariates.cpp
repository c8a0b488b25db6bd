// Host side of the GLS coefficient update: O(p^3) small dense algebra on the Gram matrix that the
// device kernels reduce (covariate_kernels.hip, DenseSolver::Gram).
#include "covariates.h"

#include <cmath>

#include "common.h"

namespace gpb_amd {

namespace {

// In-place lower Cholesky of the leading p x p block of the row-major ld x ld matrix A.
void cholesky(std::vector<double>& L, int p, int ld) {
  for (int j = 0; j < p; ++j) {
    double d = L[(size_t)j * ld + j];
    for (int k = 0; k < j; ++k) d -= L[(size_t)j * ld + k] * L[(size_t)j * ld + k];
    if (!(d > 0.) || !std::isfinite(d))
      Fatal("the matrix X^T Psi^-1 X of the covariates is not positive definite (collinear covariates?)");
    const double ljj = std::sqrt(d);
    L[(size_t)j * ld + j] = ljj;
    for (int i = j + 1; i < p; ++i) {
      double s = L[(size_t)i * ld + j];
      for (int k = 0; k < j; ++k) s -= L[(size_t)i * ld + k] * L[(size_t)j * ld + k];
      L[(size_t)i * ld + j] = s / ljj;
    }
  }
}

// x = (L L^T)^-1 b
void chol_solve(const std::vector<double>& L, int p, int ld, std::vector<double>& x) {
  for (int i = 0; i < p; ++i) {
    double s = x[i];
    for (int k = 0; k < i; ++k) s -= L[(size_t)i * ld + k] * x[k];
    x[i] = s / L[(size_t)i * ld + i];
  }
  for (int i = p - 1; i >= 0; --i) {
    double s = x[i];
    for (int k = i + 1; k < p; ++k) s -= L[(size_t)k * ld + i] * x[k];
    x[i] = s / L[(size_t)i * ld + i];
  }
}

}  // namespace

std::vector<double> unpack_gram(const double* packed, int c) {
  std::vector<double> G((size_t)c * c);
  int k = 0;
  for (int a = 0; a < c; ++a)
    for (int b = a; b < c; ++b) {
      G[(size_t)a * c + b] = packed[k];
      G[(size_t)b * c + a] = packed[k];
      ++k;
    }
  return G;
}

std::vector<double> gls_coef(const std::vector<double>& G, int p) {
  const int c = p + 1;
  std::vector<double> L = G;
  cholesky(L, p, c);
  std::vector<double> beta(p);
  for (int a = 0; a < p; ++a) beta[a] = G[(size_t)a * c + p];   // X^T Psi^-1 y
  chol_solve(L, p, c, beta);
  return beta;
}

std::vector<double> gls_coef_std_dev(const std::vector<double>& G, int p, double sigma2) {
  const int c = p + 1;
  std::vector<double> L = G;
  cholesky(L, p, c);
  std::vector<double> sd(p), e(p);
  for (int a = 0; a < p; ++a) {   // column a of (G_XX)^-1, sigma2 (G_XX)^-1 = (G_XX / sigma2)^-1
    for (int b = 0; b < p; ++b) e[b] = a == b ? 1. : 0.;
    chol_solve(L, p, c, e);
    sd[a] = std::sqrt(sigma2 * e[a]);
  }
  return sd;
}

}  // namespace gpb_amd
