// Linear regression covariates (GLS, re_model_template.h:9125-9132) and training-data random-effect
// predictions (PredictTrainingDataRandomEffects) for the Gaussian likelihood: device launchers
// (covariate_kernels.hip) and host helpers (covariates.cpp).
#pragma once

#include <hip/hip_runtime.h>

#include <vector>

namespace gpb_amd {

constexpr int kCovMaxCols = 32;   // covariates + the response column

// Blocks used by launch_vecchia_gram (its `partial` needs blocks * c (c + 1) / 2 doubles).
int vecchia_gram_blocks(int n);
// out[pair(a, b), a <= b, row-major upper triangle] = sum_i D^-1_i (B Z)_ia (B Z)_ib for the n x c
// row-major matrix Z (Vecchia order); B, D^-1 from the row kernel's factor mode.
void launch_vecchia_gram(int n, int m, int c, const int* nbr, const double* B, const double* Dinv, const double* Z,
                         double* partial, double* out, hipStream_t s);
// yaux = B^T D^-1 B y (= Psi^-1 y) and diag = diag(B^T D^-1 B); u: n scratch. tptr / trow / tslot:
// the transposed neighbour lists (rows ascending).
void launch_vecchia_psi_inv_diag(int n, int m, const int* nbr, const int* tptr, const int* trow, const int* tslot,
                                 const double* B, const double* Dinv, const double* y, double* u, double* yaux,
                                 double* diag, hipStream_t s);

// Host: unpack the packed upper triangle of a c x c Gram matrix into a full row-major matrix.
std::vector<double> unpack_gram(const double* packed, int c);
// Host: beta = G_XX^-1 G_Xy by Cholesky (Eigen's llt().solve, re_model_template.h:9131), where
// G is the full (p + 1) x (p + 1) Gram of [X | y]. Fails on a non-positive-definite G_XX.
std::vector<double> gls_coef(const std::vector<double>& G, int p);
// Host: sqrt(diag((G_XX / sigma2)^-1)) (CalcStdDevCoef, re_model_template.h:9797-9814).
std::vector<double> gls_coef_std_dev(const std::vector<double>& G, int p, double sigma2);

}  // namespace gpb_amd
