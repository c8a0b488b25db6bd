// FitcLaplace: the Laplace approximation for non-Gaussian likelihoods with the FITC approximation
// (gp_approx = "fitc", matrix_inversion_method = "cholesky"), on top of FitcSolver's buffers.
//
// Prior covariance of the latent process (no nugget): Sigma = K_nm K_mm,s^-1 K_mn + diag(d),
// d_i = sigma1^2 jitter - [K_nm K_mm,s^-1 K_mn]_ii (CalcSigmaComps, re_model_template.h:7341-7378).
// Reference path replaced:
//   mode finding + approximate marginal likelihood
//                FindModePostRandEffCalcMLLFITC      likelihoods.h:3090-3235 (Newton, Woodbury
//                                                    M = K_mm,s + K_mn diag(W (DW + I)^-1) K_nm, Armijo)
//   gradient     CalcGradNegMargLikelihoodLaplaceApproxFITC  likelihoods.h:5397-5593 (explicit traces,
//                implicit derivative through the mode; fixed-effect gradient for the booster)
//   call sites   re_model_template.h:8496-8500 (CalcModePostRandEffCalcMLL), :7789 (CalcGradFLaplace),
//                :1882 (CalcGradPars)
// Every m x n product runs on the fp64 MFMA GEMM (split-K for the m x m Woodbury Gram of each Newton
// step), the m x m factorizations on the dense path's POTRF / TRTRI, every O(n m) matrix-vector pass and
// elementwise step in HIP kernels (fitc_laplace.hip); the host runs the Newton / Armijo logic and reads
// one or two reduced scalars per step.
#pragma once

#include <hip/hip_runtime.h>

#include <vector>

#include "common.h"
#include "fitc.h"
#include "latent.h"

namespace gpb_amd {

class FitcLaplace : public LatentSolverBase {
 public:
  FitcLaplace(FitcSolver* fitc, hipStream_t stream);
  ~FitcLaplace() override;

  void SetY(const double* y) override;
  void SetOffset(const double* off) override;
  void GetMode(double* mode) override;
  // trafo = (sigma1^2, phi); aux: the shape of likelihood 'gamma' (want_aux_grad: its gradient appended to grad).
  // grad = [d/dlog sigma1^2, d/dlog phi] of the negative approximate marginal log-likelihood;
  // grad_f (nullable, host n): the gradient wrt the fixed effects F (booster).
  LatentResult Eval(int cov_type, int lik, const double* trafo, double aux, const IterativeConfig& cfg,
                    bool want_grad, bool want_aux_grad, double* grad_f = nullptr,
                    ModeStart start = ModeStart::kZero) override;
  void ResetModeToPrevious() override;
  void ClearModePrevious() override { prev_valid_ = false; }

  // Latent predictions at np points (PredictLaplaceApproxFITC, likelihoods.h:7157-7232, with the
  // unconditional FITC part of CalcPredFITC_FSA, re_model_template.h:10735-10778) from the state of the
  // last Eval (want_grad = false) at (var, phi): mean = K_pm K_mm,s^-1 K_mn d1 (+ the coincident-point
  // correction), var = sigma1^2 - |L^-1 K_mp|^2 + |Lm^-1 (K_mp - K_mn (d + W^-1)^-1 corr^T)|^2 - corr
  // terms (Lm = chol(M)); cov (np x np, column-major) analogously. Xp host row-major np x d; match[p] =
  // the training point with the same coordinates or -1.
  void Predict(int cov_type, double var, double phi, const double* Xp, int np, const std::vector<int>& match,
               bool want_var, bool want_cov, double* mean, double* pvar, double* pcov);


 private:
  // out_j = sum_i M[j, i] x_v[i] for nv <= 4 vectors (m x n matrix, ld ldm), fixed-order partials
  void Gemv(const double* M, int nv, const double* const* x, double* const* out);
  // Sigma x = K_nm K_mm,s^-1 K_mn x + d o x (into out)
  void SigmaApply(const double* x, double* out);
  // Woodbury matrix K_mm,s + K_mn diag(s) K_nm: Cholesky into W_, logdet, the factor's inverse into Wi_
  // and (full_inverse) M^-1 into Winv_; a non-positive pivot is counted in F_->info_
  void Woodbury(const double* s, double* logdet_dev, bool full_inverse);

  FitcSolver* F_;
  hipStream_t s_;
  int n_, m_, ldm_;
  bool y_set_ = false, has_off_ = false, prev_valid_ = false, evaluated_ = false;
  double cached_obj_ = 0.;     // -1/2 a^T mode + log p(y | mode + F) at the current mode
  double aux_ = 1.;            // the likelihood's auxiliary parameter (gamma: shape)
  DevBuf<double> y_, off_, mode_, a_, mode_prev_, a_prev_, mode_upd_, a_upd_, d1_, w_, wdw_, dw_, rhs_, sig_, c_, z_;
  DevBuf<double> sgv_, sgr_, dmll_, sdiag_, auxrec_;
  double sum_log_y_ = 0.;
  DevBuf<double> mv_;          // m-vectors: 18 x ldm (fitc_laplace.hip kMv)
  DevBuf<double> part_, red_;  // partials and reduced scalars
  double* h_red_ = nullptr;    // pinned
};

}  // namespace gpb_amd
