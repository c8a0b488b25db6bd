// VifLaplace: the Laplace approximation for non-Gaussian likelihoods with the full-scale Vecchia
// approximation (gp_approx = "full_scale_vecchia" / "vif", matrix_inversion_method = "cholesky"; the
// reference's "FSVA" path), on top of VifSolver's low-rank part and residual Vecchia factor and the GPU
// sparse Cholesky (sparse_chol.h).
//
// Prior precision (latent form, no nugget):
//   Sigma^-1 = R - C M^-1 C^T,  R = B^T D^-1 B,  C = R K_nm,  M = K_mm,s + K_mn R K_nm
// with B, D the Vecchia factor of the residual covariance k(a, b) - V_a . V_b (its neighbour matrices'
// diagonal times JITTER_MULT_VECCHIA, Vecchia_utils.cpp:1546-1548).
// Reference path replaced:
//   mode finding + approximate marginal likelihood
//                FindModePostRandEffCalcMLLFSVA, Cholesky branch   likelihoods.h:2316-2742 (per Newton step
//                A = R + W factored (sparse), M2 = M - C^T A^-1 C, update A^-1 rhs + A^-1 C M2^-1 C^T A^-1 rhs,
//                Armijo; log det: -sum log L_A + 1/2 sum log D^-1 + sum log L_{K_mm,s} - sum log L_{M2})
//   gradient     CalcGradNegMargLikelihoodLaplaceApproxFSVA, Cholesky branch   likelihoods.h:4716-4925
//                (explicit traces tr(S' A^-1) from the selected inverse of A, the m x m Woodbury traces as
//                Frobenius products of n x m matrices, the implicit term through (Sigma^-1 + W)^-1 d_mll)
//   call sites   re_model_template.h:8487 (CalcModePostRandEffCalcMLL), :7795 (CalcGradFLaplace),
//                :1889 (CalcGradPars)
// Every n x m product runs on the MFMA GEMM / the VIF column kernels, the sparse solves with n x m
// right-hand sides on the supernodal solve schedule, m x m factorizations on the dense path's POTRF /
// TRTRI; the host runs the Newton / Armijo logic and reads reduced scalars.
#pragma once

#include <hip/hip_runtime.h>

#include <memory>
#include <vector>

#include "common.h"
#include "latent.h"
#include "sparse_chol.h"
#include "vif.h"

namespace gpb_amd {

class VifLaplace : public LatentSolverBase {
 public:
  // nbr: host n x nn neighbour lists of the VIF model (model order), X: host row-major n x d coordinates.
  VifLaplace(VifSolver* vif, const std::vector<int>& nbr, const std::vector<double>& X, hipStream_t stream);
  ~VifLaplace() override;

  void SetY(const double* y) override;
  void SetOffset(const double* off) override;
  // The fixed effects as the caller passed them (data order, NULL: none). The reference's covariance
  // gradient (CalcGradPars, re_model_template.h:1859) hands them to CalcGradNegMargLikelihoodLaplaceApproxFSVA
  // without the model-order permutation of FSVA's random ordering (its mode finding, :8487, and CalcGradFLaplace,
  // :7768, permute them), so there the information derivative and the gamma-shape terms are evaluated at
  // mode_i + F[i]. The covariance / aux gradient of Eval(grad_f = NULL) follows that; the F-gradient uses the
  // model-order offsets. GPBOOST_AMD_VIF_OFFSET_CONSISTENT=1: the model-order offsets everywhere.
  void SetGradOffset(const double* off_data_order);
  void GetMode(double* mode) override;
  // trafo = (sigma1^2, phi); aux: the shape of likelihood 'gamma' (want_aux_grad: its gradient appended).
  LatentResult Eval(int cov_type, int lik, const double* trafo, double aux, const IterativeConfig& cfg,
                    bool want_grad, bool want_aux_grad, double* grad_f = nullptr,
                    ModeStart start = ModeStart::kZero) override;
  void ResetModeToPrevious() override;
  void ClearModePrevious() override { prev_valid_ = false; }
  const CholPlan& plan() const { return chol_->plan(); }
  float last_factor_ms() { return chol_->last_factor_ms(); }

  // Latent predictions (PredictLaplaceApproxFSVA, Cholesky branch, likelihoods.h:6060-6130, 6478-6548) from the
  // state of the last Eval at (var, phi): Xp host row-major np x d, nbr host np x mp (< n: observed points,
  // >= n: earlier prediction points, cond_all). mean (np); pvar (np, nullable); pcov (np x np column-major,
  // nullable).
  void Predict(int cov_type, double var, double phi, const double* Xp, int np, const int* nbr, int mp, bool cond_all,
               double* mean, double* pvar, double* pcov);

 private:
  // objective -1/2 m^T Sigma^-1 m + log p(y | m + F) at m = trial (written by the trial kernel)
  double Objective(int lik, const double* mode, const double* upd, double lam, bool first, bool cap, double* trial);
  // M2 = M - C^T A^-1 C from the current factor of A: CL = L^-1 P C (n x m), the split-K Gram, its
  // Cholesky (M2_ -> L, M2i_ = L^-1, M2iT_) and log det (red slot)
  void Woodbury2(double* logdet_dev);
  // out = (Sigma^-1 + W)^-1 r = A^-1 r + A^-1 C M2^-1 C^T A^-1 r (x: n scratch)
  void SolveSW(const double* r, double* out, double* x);
  // out = R x (R = B^T D^-1 B) and out = S'_1 x (range derivative of R); t: n scratch
  void RVec(const double* x, double* out, double* t);
  void SpVec(const double* x, double* out, double* t, double* t2);
  // out (m x n, ldm) = R X and S'_1 X for m x n column sets (t, t2: m x n scratch)
  void RMat(const double* X, double* out, double* t);
  void SpMat(const double* X, double* out, double* t, double* t2);
  void ToNM(const double* mn, double* nm);   // m x n (ldm) -> n x m (ld n)
  void ToMN(const double* nm, double* mn);   // and back
  double MDot(const double* a, const double* b);   // m-vector dot (synchronises)

  VifSolver* V_;
  hipStream_t s_;
  int n_, m_, ldm_;
  std::unique_ptr<SparseChol> chol_;
  bool y_set_ = false, has_off_ = false, prev_valid_ = false, evaluated_ = false;
  double cached_obj_ = 0.;
  double aux_ = 1.;
  int lik_ = -1;
  double sum_log_y_ = 0.;
  DevBuf<double> y_, off_, mode_, mode_prev_, upd_, trial_, d1_, w_, dw_, rhs_, dinv_, diagS_, dmll_, vS_;
  DevBuf<double> goff_, gd1_, gw_;       // data-order offsets; d1, W at mode + them (the reference's gradient)
  bool has_goff_ = false;
  DevBuf<double> vec_;                   // n-vector scratch
  DevBuf<double> mv_;                    // m-vector scratch
  DevBuf<double> M_, M2_, M2i_, M2iT_, M2inv_;   // m x m (ldm)
  DevBuf<double> C_, Cnm_, CL_, AiC_, Y_, G_, T1_, T2_, T3_;   // n x m sets (C_, AiC_, Y_, G_, T*: m x n ldm)
  DevBuf<double> part_, red_;
  DevBuf<int> info_;          // non-positive pivots of the M2 factorization
  double* h_red_ = nullptr;   // pinned
  hipEvent_t ev_[2] = {nullptr, nullptr};
};

}  // namespace gpb_amd
