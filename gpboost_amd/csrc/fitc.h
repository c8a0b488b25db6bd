// FITC (fully independent training conditional) approximation for the Gaussian likelihood,
// gp_approx = "fitc": the reference's low-rank-plus-diagonal covariance
//   Psi = K_nm K_mm,s^-1 K_mn + diag(d),   d_i = 1 + sigma1^2 (1 + 1e-6) - [K_nm K_mm,s^-1 K_mn]_ii
// (transformed scale: nugget 1, K = sigma1^2 / sigma^2 rho), K_mm,s = K_mm with its diagonal times
// JITTER_MULT_IP_FITC_FSA (utils.h:39), the m inducing points chosen once by kmeans++ / random.
//
// Reference path replaced:
//   inducing points       re_model_template.h:6931-7073 (CreateREComponentsFITC_FSA), GP_utils.cpp:203-295
//                         (random_plusplus, calculate_means, kmeans_plusplus), utils.h:323-337
//                         (SampleIntNoReplaceSort)
//   Sigma components      re_model_template.h:7341-7378 (CalcSigmaComps, fitc_resid_diag_)
//   Woodbury factor       re_model_template.h:8823-8863 (CalcCovFactorFITC_FSA, cholesky)
//   y_aux = Psi^-1 y      re_model_template.h:8898-8908 (CalcYAux)
//   log det Psi           re_model_template.h:2698-2714
//   gradient              re_model_template.h:1985-2232 (CalcGradPars_FITC_FSA_GaussLikelihood_Cluster_i)
// The reference offloads its DGEMM / DTRSM to cuBLAS here (cuda_kernel.cu:613-941); this build
// runs every m x n product on the fp64 MFMA tile GEMM of dense_kernels.hip, the m x m Cholesky /
// inverse on the dense path's POTRF / TRTRI, and the O(n m) reductions in fused column kernels.
//
// HBM layout: every m x n matrix column-major with leading dimension ldm = round_up(m, 64), i.e.
// observation i's m entries contiguous (one wave per observation in the column kernels).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <random>
#include <string>
#include <vector>

#include "common.h"

namespace gpb_amd {

// Inducing points (host, row-major m x d) of the reference's selection methods on the coordinates
// (host row-major n x d, original order; must be unique locations). kmeans++ runs its Lloyd
// iterations on the GPU (stream s) with the reference's exact distance / mean arithmetic.
std::vector<double> fitc_inducing_points(const std::vector<double>& coords, int n, int d, int m,
                                         const std::string& method, std::mt19937& rng, hipStream_t s);

// Building blocks shared with the Laplace approximation (fitc_kernels.hip): out = S x (S symmetric
// m x m, ld ldm); W = sum of `chunks` split-K partials + K_mm,s; the six m x m terms of the gradient
// [sum Kinv o Kmm, sum Winv o Kmm, sum Kinv o dK, sum Winv o dK, a^T Kmm a, a^T dK a] (part: 6 (m + 3) / 4
// doubles of scratch); K_mn (m x n, ld ldm) of the coordinates X (row-major n x d) and inducing points Z.
void fitc_symv(hipStream_t s, const double* S, const double* x, int m, int ldm, double* out);
// out = S^-1 x = Li^T (Li x) from the inverse Li of S's Cholesky factor (lower triangle read only) and its
// transpose LiT (fitc_lower_t; tmp: m doubles). Two triangular products instead of one product with the
// explicit S^-1: the Cholesky-solve accuracy (error ~ cond(L) eps rather than cond(S) eps), which the
// Laplace Newton iteration needs when K_mm,s or the Woodbury matrix is ill-conditioned.
void fitc_chol_solve(hipStream_t s, const double* Li, const double* LiT, const double* x, int m, int ldm, double* tmp,
                     double* out);
// LT = transpose of the lower triangle of L (zeros above the diagonal)
void fitc_lower_t(hipStream_t s, const double* L, int m, int ldm, double* LT);
// out = S^-1 K_mn (m x n, ld ldm) with the explicit Sinv (one full MFMA GEMM), or Li^T (Li K_mn) through tmp
// (two triangle-masked GEMMs) when GPBOOST_AMD_FITC_G=tri (A/B: same gradients, slower; fitc_kernels.hip)
void fitc_solve_kmn(hipStream_t s, const double* Li, const double* Sinv, const double* Kmn, int m, int n, int ldm,
                    double* tmp, double* out);
void fitc_wsum(hipStream_t s, const double* P, int chunks, long stride, int m, int ldm, const double* Ks, double* W);
void fitc_mm_terms(hipStream_t s, const double* Kinv, const double* Winv, const double* Kmm, const double* dK,
                   const double* a, int m, int ldm, double* part, double* out6);
void fitc_kmn(hipStream_t s, int cov_type, const double* X, const double* Z, int n, int m, int d, int ldm, double var,
              double phi, double* Kmn);

class FitcSolver {
 public:
  // d_X: device row-major n x d coordinates; Z: host row-major m x d inducing points.
  FitcSolver(int n, int d, const double* d_X, const std::vector<double>& Z, hipStream_t stream);
  int num_ind_points() const { return m_; }
  const std::vector<double>& inducing_points() const { return Z_; }
  // sums = [logdet, q, s1_var, s1_range, s2_var, s2_range] (DenseSolver::Eval's contract):
  // s1_k = -1/2 y_aux^T dPsi_k y_aux, s2_k = tr(Psi^-1 dPsi_k) with the reference's dPsi_k (the
  // un-jittered dK_mm in the derivative). A non-positive-definite K_mm,s or Woodbury matrix gives
  // NaN sums. kernel_ms[0] = factor part, kernel_ms[1] = whole device evaluation.
  void Eval(int cov_type, double var, double phi, const double* d_y, bool want_grad, double* sums, double* kernel_ms);
  // Psi^-1 y (host, n) at the last Eval's parameters (the y_aux of the last Eval)
  void YAux(double* out);
  // Predictions at np new points (CalcPredFITC_FSA, re_model_template.h:10600-10828, Gaussian,
  // transformed scale: variances and covariance before the sigma^2 factor). Xp host row-major
  // np x d; match[i] = the training point with the same coordinates as prediction point i (the FITC
  // diagonal correction, :10643-10691) or -1. mean (np) always; var (np) when want_var; cov (np x np,
  // column-major) when want_cov; response adds the nugget 1.
  void Predict(int cov_type, double var, double phi, const double* d_y, const double* Xp, int np,
               const std::vector<int>& match, bool want_var, bool want_cov, bool response, double* mean,
               double* pvar, double* pcov);
  // Fisher information of the covariance parameters (3 x 3 row-major, [sigma^2, sigma1^2, rho]) at the
  // original-scale orig (trafo: the same transformed), Hutchinson estimates over t probes from (seed,
  // run_id): CalcFisherInformation_FITC_FSA (re_model_template.h:9363-9548; fitc_fisher.hip).
  void Fisher(int cov_type, const double* orig, const double* trafo, int t, int seed, uint64_t run_id, double* FI);

 private:
  friend class FitcLaplace;   // the Laplace approximation (fitc_laplace.h) works on these buffers
  friend class VifSolver;     // the full-scale Vecchia approximation (vif.h) reuses the low-rank part
  friend class VifLaplace;    // and its Laplace approximation (vif_laplace.h)
  // K_mn, K_mm, K_mm,s, dK_mm, L = chol(K_mm,s) (red[0] = 2 sum log L_ii), L^-1 (Li_), V = L^-1 K_mn,
  // K_mm,s^-1 (Kinv_): the part of the factorization that does not depend on the likelihood
  void Prior(int cov_type, double var, double phi, double* red);
  void Factor(int cov_type, double var, double phi, const double* d_y, double* red);

  int n_, d_, m_, ldm_;
  const double* d_X_;
  std::vector<double> Z_;
  hipStream_t stream_;
  int max_chunks_ = 1;
  DevBuf<double> dZ_;
  DevBuf<double> Kmn_, V_, Kd_, A_;        // m x n (ldm)
  DevBuf<double> Kmm_, Ks_, Li_, W_, Wi_, Kinv_, Winv_, dKmm_, T_;   // m x m (ldm)
  DevBuf<double> LiT_, WiT_;                                         // transposed inverse factors
  DevBuf<double> part_, vec_, red_;
  DevBuf<int> info_;
  double* h_red_ = nullptr;
  hipEvent_t ev_[3] = {nullptr, nullptr, nullptr};
};

}  // namespace gpb_amd
