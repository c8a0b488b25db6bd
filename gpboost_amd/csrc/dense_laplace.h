// DenseLaplace: the Laplace approximation for non-Gaussian likelihoods without an approximation of the GP
// (gp_approx = "none"), the numerically stable form of Rasmussen and Williams (2006) that the reference uses
// for dense covariance matrices. Sigma = sigma1^2 corr(phi) (n x n, no nugget), W = the likelihood's
// information at the mode, B = I + W^1/2 Sigma W^1/2 = L L^T.
// Reference path replaced:
//   mode finding + approximate marginal likelihood
//                FindModePostRandEffCalcMLLStable              likelihoods.h:1843-1960 (Newton on
//                a = Sigma^-1 mode with B's Cholesky factor, Armijo backtracking, mll = obj - sum log L_ii)
//   gradient     CalcGradNegMargLikelihoodLaplaceApproxStable  likelihoods.h:3261-3413 (explicit
//                -1/2 a^T dSigma a + 1/2 tr((W^-1 + Sigma)^-1 dSigma), implicit through the mode with
//                diag((Sigma^-1 + W)^-1) = diag(Sigma) - colnorms(L^-1 W^1/2 Sigma)^2; fixed-effect gradient)
//   predictions  PredictLaplaceApproxStable                    likelihoods.h:5610-5676 (mean Sigma_po d1,
//                (co)variances Sigma_pp - (L^-1 W^1/2 Sigma_op)^T (L^-1 W^1/2 Sigma_op))
//   call sites   re_model_template.h:8496-8518 (CalcModePostRandEffCalcMLL), :1882 (CalcGradPars)
// Every n x n step runs on the dense path's MFMA kernels (dense.h: chol_lower, trtri_lower, gemm_f64):
// one Cholesky and one triangular inverse of B per Newton step, every matrix-vector product as an MFMA
// GEMM with one column, (W^-1 + Sigma)^-1 = Q^T Q and L^-1 W^1/2 Sigma = Q Sigma (Q = L^-1 W^1/2) for the
// gradient; the host runs the Newton / Armijo logic on reduced scalars.
#pragma once

#include <hip/hip_runtime.h>

#include "common.h"
#include "latent.h"

namespace gpb_amd {

class DenseLaplace : public LatentSolverBase {
 public:
  // d_X: device coordinates, row-major n x d (distinct points), owned by the caller
  DenseLaplace(int n, int d, const double* d_X, hipStream_t stream);
  ~DenseLaplace() override;

  void SetY(const double* y) override;
  void SetOffset(const double* off) override;
  void GetMode(double* mode) override;
  // trafo = (sigma1^2, phi); grad = [d/dlog sigma1^2, d/dlog phi] of the negative approximate marginal
  // log-likelihood (+ d/dlog shape for likelihood 'gamma' with want_aux_grad: CalcGradNegLogLikAuxPars +
  // 1/2 sum dW/dlog shape o diag((Sigma^-1 + W)^-1) + the implicit term, likelihoods.h:3379-3411, 10508-10524,
  // 10856-10869); aux: the gamma shape; grad_f (nullable, host n): the gradient wrt the fixed effects F (booster).
  LatentResult Eval(int cov_type, int lik, const double* trafo, double aux, const IterativeConfig& cfg,
                    bool want_grad, bool want_aux_grad, double* grad_f = nullptr,
                    ModeStart start = ModeStart::kZero) override;
  void ResetModeToPrevious() override;
  void ClearModePrevious() override { prev_valid_ = false; }
  // Latent predictions at np points (Xp host row-major np x d) from the state of the last Eval at (var, phi):
  // mean = Sigma_po d1, var / cov (column-major np x np) as PredictLaplaceApproxStable.
  void Predict(int cov_type, double var, double phi, const double* Xp, int np, bool want_var, bool want_cov,
               double* mean, double* pvar, double* pcov);

 private:
  void BuildSigma(int cov_type, double var, double phi);
  // B = I + W^1/2 Sigma W^1/2 (lower) from ws_, its Cholesky factor in place (B_), 2 sum log L_ii -> *logdet_dev;
  // with_inverse: L^-1 into Li_
  void FactorB(double* logdet_dev, bool with_inverse);
  // y = op(M) x for an n x n matrix (ld), lower: M is lower triangular, trans: M^T
  void Gemv(const double* M, bool lower, bool trans, const double* x, double* y);
  bool InfoFailed();

  int n_, d_, ld_;
  const double* d_X_;
  hipStream_t s_;
  bool y_set_ = false, has_off_ = false, prev_valid_ = false, evaluated_ = false;
  double cached_obj_ = 0.;
  double aux_ = 1.;   // the likelihood's auxiliary parameter (gamma: shape)
  double sum_log_y_ = 0.;
  int cov_type_ = 0;
  double var_ = 0., phi_ = 0.;
  DevBuf<double> Sig_, B_, Li_, X_, R_, C_;   // n x n (ld); X_: trtri scratch
  DevBuf<double> y_, off_, mode_, a_, mode_prev_, a_prev_, mode_upd_, a_upd_, d1_, w_, ws_, rhs_, t1_, t2_, t3_, t4_;
  DevBuf<double> dmll_, dg_, uv_, ur_, rec_, cols_, red_;
  DevBuf<int> info_;
  double* h_red_ = nullptr;
  hipEvent_t ev_[2] = {nullptr, nullptr};
};

}  // namespace gpb_amd
