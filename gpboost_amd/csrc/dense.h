// Dense Gaussian-process likelihood on the GPU (gp_approx = "none"):
// Psi = Sigma/sigma2 + I built in HBM, blocked fp64 Cholesky with MFMA trailing updates,
// Psi^-1 for the gradient traces. Reference: re_model_template.h:5902-5904 (CalcChol),
// :5987-6007 (CalcPsiInv), :1798-1818 (dense gradient), :2875-2880 (nll).
#pragma once

#include <hip/hip_runtime.h>

#include "common.h"

namespace gpb_amd {

class DenseSolver {
 public:
  DenseSolver(int n, int d, const double* d_X, hipStream_t stream);
  ~DenseSolver();
  // sums = [logdet, q, s1_var, s1_range, s2_var, s2_range] (same contract as the Vecchia rows):
  // s1_k = -1/2 y_aux^T dPsi_k y_aux, s2_k = tr(dPsi_k Psi^-1).
  // kernel_ms[0] = Cholesky time, kernel_ms[1] = whole device evaluation.
  void Eval(int cov_type, double var, double phi, const double* d_y, bool want_grad, double* sums, double* kernel_ms);
  // Traces of the Fisher information on the original scale (standard errors): with P = Psi^-1,
  // D1 = correlation matrix, D2 = dscale * dcorr/dlog(phi) and G_k = P D_k, sums6 =
  // [sum P^2, sum P o G1, sum P o G2, tr(G1 G1), tr(G1 G2), tr(G2 G2)].
  void Fisher(int cov_type, double var, double phi, double dscale, double* sums6);
  // Gram matrix of the covariates: G (host, c x c) = Z^T Psi^-1 Z for the host column-major n x c
  // matrix Z = [X | y] (CalcXTPsiInvX, re_model_template.h:9125-9132).
  void Gram(int cov_type, double var, double phi, const double* Z, int c, double* G);
  // Psi^-1 y and diag(Psi^-1) (host, n each) for the training-data random-effect predictions.
  void PsiInvDiag(int cov_type, double var, double phi, const double* d_y, double* yaux, double* diag);
  // Predictions at np new points (host row-major Xp): mean, latent variances (nullable) and the latent
  // covariance (column-major np x np, nullable) on the transformed scale (before sigma^2 / nugget)
  void Predict(int cov_type, double var, double phi, const double* d_y, const double* Xp, int np, bool want_var,
               bool want_cov, double* mean, double* pvar, double* pcov);
  // Combined GP + grouped random effects (gp_approx = "none"; re_model_template.h:8430-8441 CalcZSigmaZt sums the
  // components): Psi gains sum_k tau_k [lev_k(i) == lev_k(j)] (d_lev: device K x n level indices, K <= 8)
  // in every build; K = 0 switches it off. Predictions then take the prediction points' levels (SetGroupedPred:
  // device K x np, -1 - id for a label not in the training data, equal ids for equal new labels).
  void SetGrouped(int K, const int* d_lev, const double* tau);
  void SetGroupedPred(int np, const int* d_plev);
  // After Eval(want_grad = true): tr(Psi^-1 dPsi / dlog tau_k) = tau_k sum_{lev_k(i) == lev_k(j)} (Psi^-1)_ij
  // (K values) and y_aux = Psi^-1 y (host, n) for the quadratic terms.
  void GroupedTraces(double* s2, double* yaux);

 private:
  void Potrf();
  void PotrfLookahead();
  void Trtri(int a, int b);
  void Factor(int cov_type, double var, double phi);   // Psi, L (POTRF) and W = L^-1 (TRTRI)
  void CheckInfo();                                    // synchronises; fails if POTRF failed

  int n_, d_, ld_;
  const double* d_X_;
  hipStream_t stream_;
  DevBuf<double> A_, W_, T_, vec_, red_;
  void AddGrouped();   // Psi += the grouped term (lower triangle), after a build
  int gK_ = 0, gnp_ = 0;
  const int* g_lev_ = nullptr;
  const int* g_plev_ = nullptr;
  double g_tau_[8] = {0., 0., 0., 0., 0., 0., 0., 0.};
  DevBuf<double> g_part_;
  DevBuf<int> info_;
  double* h_red_ = nullptr;
  hipEvent_t ev_[3] = {nullptr, nullptr, nullptr};
  // lookahead POTRF: panel chain on a high-priority stream, the rest of each trailing update on a
  // second stream (created on first use)
  hipStream_t s_chain_ = nullptr, s_rest_ = nullptr;
  hipEvent_t ev_la_[3] = {nullptr, nullptr, nullptr};
};

// C[M x N] = alpha op(A) op(B) + beta C, column-major fp64, MFMA tiles (dense_kernels.hip).
// Masks: lower_out skips output tiles above the diagonal; a_lower / a_upper: op(A)[i][k] == 0
// for k > i / k < i; b_lower: op(B)[k][j] == 0 for k < j (structural zeros are skipped).
void gemm_f64(hipStream_t s, int M, int N, int K, double alpha, const double* A, int lda, int transA, const double* B,
              int ldb, int transB, double beta, double* C, int ldc, int lower_out = 0, int a_lower = 0,
              int a_upper = 0, int b_lower = 0);

// Split-K product: chunk z of K (a multiple of 16 long, as many chunks as give ~target_blocks
// workgroups, at most max_chunks) writes op(A) op(B) over its K range to C + z * cstride (M x N, ldc). Returns the
// number of chunks (the caller sums the partial products in chunk order). No triangle masks.
int gemm_f64_splitk(hipStream_t s, int M, int N, int K, const double* A, int lda, int transA, const double* B, int ldb,
                    int transB, double* C, int ldc, long cstride, int target_blocks, int max_chunks);

// In-place two-level Cholesky of the lower triangle of the n x n matrix A (leading dimension ld, a
// multiple of 64): L overwrites A's lower triangle, the inverses of its 64 x 64 diagonal blocks go to
// W's diagonal blocks; info counts non-positive pivots (DenseSolver's factorization, also FITC's).
void chol_lower(hipStream_t s, double* A, double* W, int n, int ld, int* info);
// W[a:b, a:b] = L[a:b, a:b]^-1 (lower) from chol_lower's diagonal-block inverses; X: scratch of
// >= ld x (ld / 2 + 64) doubles.
void trtri_lower(hipStream_t s, const double* L, double* W, double* X, int a, int b, int ld);
// out[0] = 2 sum_i log L_ii (one block, fixed order)
void launch_logdet_chol(hipStream_t s, const double* L, int ld, int n, double* out);

// Dense SPD system of order n on the GPU (host column-major A): x = A^-1 b (b, x nullable),
// diag(A^-1) (nullable), the full A^-1 column-major (nullable). Fails if A is not positive definite.
void spd_solve_inverse(hipStream_t s, int n, const double* A, const double* b, double* x, double* diag, double* inv);

// Gaussian prediction through a dense Vecchia approximation of the latent process over N points
// (observed first: n, then np = N - n prediction points): B (host column-major N x N, unit lower),
// D (N) -> Sigma = B^-1 diag(D) B^-T; mean = Sigma_po (Sigma_oo + I)^-1 y, cov = Sigma_pp -
// Sigma_po (Sigma_oo + I)^-1 Sigma_op (variances its diagonal). Transformed scale (nugget 1).
void vecchia_latent_dense_pred(hipStream_t s, int N, int n, const double* B, const double* D, const double* y,
                               bool want_var, bool want_cov, double* mean, double* var, double* cov);

// Latent-model predictive moments from nsim simulation draws (PredictLaplaceApproxVecchia,
// likelihoods.h:6713-6749): d_V (device np x nsim column-major) = Bpo z per draw; Bp (host dense np x np
// unit lower, nullable = identity for cond_obs_only): U = Bp^-1 V, var = rowsum(U^2) / nsim +
// diag(Bp^-1 diag(Dp) Bp^-T), cov = U U^T / nsim + Bp^-1 diag(Dp) Bp^-T (column-major).
void latent_pred_moments(hipStream_t s, int np, const double* Bp, const double* Dp, const double* d_V, int nsim,
                         bool want_var, bool want_cov, double* var, double* cov);

// host helper shared by all paths (re_model.cpp)
void combine_partials(const double* s, int n, double sigma2_in, int profile, double* nll, double* grad,
                      double* sigma2_out);

}  // namespace gpb_amd
