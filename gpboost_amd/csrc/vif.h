// Full-scale Vecchia approximation ("VIF", gp_approx = "full_scale_vecchia" / "vif") for the Gaussian
// likelihood: the reference's predictive-process-plus-Vecchia-residual covariance
//   Psi = K_nm K_mm,s^-1 K_mn + B^-1 D B^-T
// on the transformed scale (nugget 1 in the residual part), where B (unit lower, the Vecchia neighbours
// of each point in the model order) and D come from the RESIDUAL covariances
//   C_res(a, b) = k(a, b) + [a == b] - V_a . V_b,   V = L^-1 K_mn,  L = chol(K_mm,s)
// among each point and its neighbours, and K_mm,s = K_mm with its diagonal times (1 + 1e-6).
//
// Reference path replaced:
//   ordering + inducing points  re_model_template.h:348-357 (shuffle with rng_, then CreateREComponentsFITC_FSA
//                               on the shuffled coordinates with the same generator)
//   neighbours                  Vecchia_utils.cpp:732-1058 (Euclidean kNN among earlier points; the GPU search)
//   Sigma components            re_model_template.h:7341-7378 (CalcSigmaComps)
//   residual factor + gradient  Vecchia_utils.cpp:1388-1617 (CalcCovFactorGradientVecchia, full_scale_vecchia)
//   Woodbury factor             re_model_template.h:8770-8880 (CalcCovFactorFITC_FSA, cholesky)
//   y_aux, log det              re_model_template.h:8898-8935, 2698-2714
//   gradient                    re_model_template.h:1985-2232 (CalcGradPars_FITC_FSA_GaussLikelihood_Cluster_i)
// The reference runs these with Eigen sparse products, cuBLAS / cuSPARSE offloads (cuda_kernel.cu:613-941).
// This build: one wave per row for the residual factor with the neighbour set's Gram blocks V_S^T [V P_0
// P_1]_S on the fp64 MFMA (operands loaded straight from the m x n matrices; sets of up to 32 points, the
// reference's default 30 neighbours; larger sets: a 256-thread LDS-staged register-tile form), the small
// Cholesky and solves in LDS / registers of that wave; sparse B / B^T products over contiguous m-vectors
// (one wave per point; B^T vectors from the factor values gathered into column order); every m x n /
// m x m product on the fp64 MFMA GEMM (split-K for the m x m Woodbury Gram).
//
// HBM layout: every m x n matrix column-major with leading dimension ldm = round_up(m, 64) (point i's m
// entries contiguous), the B / D factor and its derivatives as n x nn value rows beside the neighbour lists.
#pragma once

#include <hip/hip_runtime.h>

#include <memory>
#include <vector>

#include "common.h"
#include "fitc.h"

namespace gpb_amd {

class VifSolver {
 public:
  // d_X: device row-major n x d coordinates in the model order; Z: host row-major m x d inducing points;
  // nbr: host n x nn neighbour lists (row i holds its min(i, nn) neighbours, the rest -1).
  VifSolver(int n, int d, const double* d_X, const std::vector<double>& Z, const std::vector<int>& nbr, int nn,
            hipStream_t stream);
  ~VifSolver();
  const std::vector<double>& inducing_points() const { return F_->inducing_points(); }
  // sums = [logdet, q, s1_var, s1_range, s2_var, s2_range] (combine_partials): s1_k = -1/2 y_aux^T dPsi_k
  // y_aux, s2_k = tr(Psi^-1 dPsi_k) with the reference's dPsi_k (un-jittered dK_mm, B_grad, D_grad). A
  // non-positive-definite factor gives NaN sums. kernel_ms[0] = factor part, [1] = whole evaluation.
  void Eval(int cov_type, double var, double phi, const double* d_y, bool want_grad, double* sums, double* kernel_ms);
  // D (n) and B's values (n x nn, 0 past a row's neighbours) of the last Eval (host)
  void GetFactor(double* D, double* Bv) const;
  // Predictions for the Gaussian likelihood (CalcPredVecchiaObservedFirstOrder, full_scale_vecchia branches,
  // Vecchia_utils.cpp:1686-1707, 1826-1840, 1872-1873, 1901-1980) at (var, phi) on the transformed scale,
  // nugget 1 included: Xp host row-major np x d prediction points (after the n observed points); nbr host
  // np x mp neighbour indices (< n: observed points; >= n: earlier prediction points, cond_all). mean (np);
  // pvar (np, nullable); pcov (np x np column-major, nullable). Runs Eval(want_grad = false) first.
  void Predict(int cov_type, double var, double phi, const double* d_y, const double* Xp, int np, const int* nbr,
               int mp, bool cond_all, double* mean, double* pvar, double* pcov);

 private:
  friend class VifLaplace;   // the Laplace approximation for non-Gaussian likelihoods (vif_laplace.h)
  // the likelihood-independent part of an evaluation: the low-rank part (K_mn, K_mm,s, L, V), with grad the
  // derivative blocks (dK, A, P_0, P_1), the residual factor (+ column-order values) and the Woodbury
  // matrix M = K_mm,s + BK^T D^-1 BK factored in place (F_->W_ = L_M, Wi_ = L_M^-1, WiT_); red[0] = log det
  // K_mm,s, red[1] = log det M; M_copy (nullable, ldm x ldm): M before its factorization
  void Prepare(int cov_type, double var, double phi, bool grad, double* red, double* M_copy = nullptr);
  void Rows(int cov_type, double var, double phi, bool grad);
  // the prediction points' residual rows (Xp host np x d after the n observed points, nbr host np x mp):
  // KP = K_mp (m x np), Va = [V | L^-1 K_mp], Bvp (np x mp), Dp (np), dnb the neighbour lists on the device
  void PredRows(int cov_type, double var, double phi, const double* Xp, int np, const int* nbr, int mp,
                DevBuf<double>& KP, DevBuf<double>& Va, DevBuf<double>& Bvp, DevBuf<double>& Dp, DevBuf<int>& dnb);
  // mo_p = sum over observed neighbours of B(p, j) r_j, Qt[:, p] = sum of B(p, j) M[:, j] (M m x n; Qt m x np)
  void PredBpo(int np, int mp, const int* dnb, const double* Bvp, const double* r, const double* M, double* mo,
               double* Qt);
  // out_i = M[:, i] . w (w != nullptr) or M[:, i] . M2[:, i] for `cols` columns
  void ColDotN(const double* M, const double* w, const double* M2, int cols, double* out);
  // out = B in (self = 1) or dB in (self = 0) over m-vector columns; div: then times D^-1; out_div
  // (nullable): the same columns times D^-1 as a second output
  void BRow(const double* in, const double* coef, double self, bool div, double* out, double* out_div = nullptr);
  // out = B^T in (self = 1) or dB^T in (self = 0) over m-vector columns
  void BCol(const double* in, const double* coefT, double self, double* out);   // coefT: values in column order
  void BVec(const double* x, const double* coef, double self, double* out);
  // out = B^T x (self = 1) or dB^T x (self = 0), coefT: the factor's values in column order (BvT_ ...)
  void BtVec(const double* x, const double* coefT, double self, double* out);
  void Gemv(const double* M, const double* x, double* out);   // out (m) = M x, M m x n
  void ColDot(const double* M, const double* w, const double* M2, double* out);   // out_i = M_i . (w | M2_i)

  std::unique_ptr<FitcSolver> F_;
  int n_, d_, m_, ldm_, nn_;
  bool latent_ = false;   // residual rows of the latent form (no nugget; JITTER_MULT_VECCHIA on the neighbour diagonal)
  hipStream_t s_;
  const double* d_X_;
  DevBuf<int> nbr_, tptr_, trow_, tslot_;
  DevBuf<int> ord_;   // the points in spatial (Morton) order: processing order of the row / B-product kernels
  DevBuf<double> dK_, P0_, P1_, BK_;                 // m x n (ldm)
  DevBuf<double> Bv_, dBv0_, dBv1_;                   // n x nn
  DevBuf<double> BvT_, dBvT0_, dBvT1_;                // the same values in column (B^T) order
  int nnz_ = 0;
  DevBuf<double> D_, dD0_, dD1_;                      // n
  DevBuf<double> vec_;                                // n-vectors (scratch)
  DevBuf<double> mvec_;                               // m-vectors (scratch)
  DevBuf<double> part_, red_;
  double* h_red_ = nullptr;
  size_t lds_bytes_ = 0;
  hipEvent_t ev_[3] = {nullptr, nullptr, nullptr};
};

}  // namespace gpb_amd
