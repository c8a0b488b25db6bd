// LatentVecchia with matrix_inversion_method = "cholesky": the reference's exact Laplace-Vecchia path
// on the GPU sparse Cholesky of Sigma^-1 + W (sparse_chol.h).
//   mode finding      FindModePostRandEffCalcMLLVecchia, Cholesky branch (likelihoods.h:2935-2955, 2957-2995):
//                     per Newton step W from the likelihood, A = B^T D^-1 B + W factored, the update
//                     (Sigma^-1 + W)^-1 (W mode + d1) by the two triangular sweeps, Armijo backtracking
//   log-determinant   :3052-3070: refactor at the mode, -sum log L_ii + 0.5 sum log D^-1_ii
//   gradient          CalcGradNegMargLikelihoodLaplaceApproxVecchia, Cholesky branch (:5207-5336): the exact
//                     traces tr(SigmaI_deriv (Sigma^-1 + W)^-1) from the selected inverse on the pattern of L
//                     (the reference's CalcLtLGivenSparsityPattern over L^-1), d_mll_d_mode = 0.5 diag(S) dW,
//                     the implicit term through one more solve, the aux / F gradients (:5281-5336, 5337-5369)
//   predictions       PredictLaplaceApproxVecchia, Cholesky branch (:6751-6811): Maux = L \ (Bpo^T [Bp^-T])
// Reused from the iterative path: the latent factor kernel, the Newton record (newton_prep), the row
// scalars (quadratic forms, log-likelihood, implicit terms) and the A operator for the Armijo slope.
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>

#include "kernels.h"
#include "latent.h"
#include "sparse_chol.h"

namespace gpb_amd {

namespace {
constexpr double kJitterMultVecchiaC = 1. + 1e-10;   // JITTER_MULT_VECCHIA (utils.h)
constexpr double kCArmijoC = 1e-4;                   // c_armijo_ (likelihoods.h:12737)
}  // namespace

void LatentVecchia::SetCholesky(bool on) { use_chol_ = on; }

void LatentVecchia::EnsureChol() {
  if (chol_) return;
  std::vector<int> nbr((size_t)n_ * m_);
  std::vector<double> X((size_t)n_ * d_);
  HIP_CHECK(hipMemcpyAsync(nbr.data(), d_nbr_.get(), sizeof(int) * nbr.size(), hipMemcpyDeviceToHost, s_));
  HIP_CHECK(hipMemcpyAsync(X.data(), d_Xp_.get(), sizeof(double) * X.size(), hipMemcpyDeviceToHost, s_));
  HIP_CHECK(hipStreamSynchronize(s_));
  chol_.reset(new SparseChol(n_, m_, nbr.data(), d_, X.data(), s_));
  d_diagS_.alloc(n_);
}

const CholPlan* LatentVecchia::CholPlanInfo() {
  if (!use_chol_) return nullptr;
  EnsureChol();
  return &chol_->plan();
}

LatentResult LatentVecchia::EvalChol(int cov_type, int lik, const double* trafo, double aux, const IterativeConfig& cfg,
                                     bool want_grad, bool want_aux_grad, double* grad_f_vo, ModeStart start) {
  if (!y_set_) Fatal("response variable y has not been set");
  if (!(trafo[0] > 0. && trafo[1] > 0.)) Fatal("covariance parameters must be > 0");
  if (lik == kLikGaussian && !(aux > 0.)) Fatal("the error variance (aux_pars) must be > 0");
  if (lik == kLikGamma && want_grad && want_aux_grad && has_obs_)
    Fatal("estimating the shape of likelihood 'gamma' with gp_approx = 'vecchia' and repeated coordinates is not "
          "supported by gpboost_amd (set estimate_aux_pars = false)");
  if (world_ > 1) Fatal("matrix_inversion_method = 'cholesky' for latent Vecchia models runs on one rank");
  EnsureChol();
  const int n = n_;
  const bool gauss = lik == kLikGaussian;
  LatentResult res;
  HIP_CHECK(hipEventRecord(ev0_, s_));
  Block& b1 = GetBlock(0, 1, 1);   // G scratch of the A operator (Armijo slope); the reduction buffers

  // ---- 1. latent Vecchia factor (+ range derivatives), A's entries
  LatentFactorArgs fa{};
  fa.X = d_Xp_.get();
  fa.nbr = d_nbr_.get();
  fa.n = n; fa.d = d_; fa.m = m_;
  fa.var = trafo[0];
  fa.phi = trafo[1];
  fa.jitter = kJitterMultVecchiaC;
  fa.Bv = d_Bv_.get();
  fa.dBv = want_grad ? d_dBv_.get() : nullptr;
  fa.Dinv = d_Dinv_.get();
  fa.dD = want_grad ? d_dD_.get() : nullptr;
  launch_latent_factor(cov_type, fa, s_);
  launch_gather(tnnz_, d_tslot_.get(), d_Bv_.get(), d_tval_.get(), s_);   // B^T operator values (Armijo slope)
  if (seg2_n_ > 0) launch_gather(seg2_n_, d_seg_slot2_.get(), d_Bv_.get(), d_seg_val2_.get(), s_);
  sp_.tval_of = d_Bv_.get();
  launch_gather(n * m_, d_ell_slot_.get(), d_Bv_.get(), d_ell_val_.get(), s_);
  sp_.vals_of = d_Bv_.get();
  factor_ready_ = true;
  chol_->SetB(d_Bv_.get(), d_Dinv_.get(), want_grad ? d_dBv_.get() : nullptr, want_grad ? d_dD_.get() : nullptr);

  ScalarArgs sa{};
  sa.n = n; sa.m = m_; sa.lik = lik; sa.aux = aux;
  sa.nbr = d_nbr_.get(); sa.Bv = d_Bv_.get(); sa.Dinv = d_Dinv_.get(); sa.y = d_y_.get();
  sa.offset = has_off_ && !has_obs_ ? d_off_.get() : nullptr;
  sa.obs = Obs();
  auto newton_prep = [&](int W_update, bool with_rhs) {
    NewtonPrepArgs np{};
    np.n = n; np.lik = lik; np.aux = aux; np.y = d_y_.get(); np.loc = d_mode_.get(); np.mode = d_mode_.get();
    np.offset = has_off_ && !has_obs_ ? d_off_.get() : nullptr;
    np.obs = Obs();
    np.Dinv = d_Dinv_.get(); np.d1 = d_d1_.get(); np.W = d_W_.get(); np.W_update = W_update;
    np.rhs = with_rhs ? d_rhs_.get() : nullptr;
    np.dw = d_dw_.get();
    launch_newton_prep(np, s_);
  };
  auto factor = [&]() {
    chol_->Factor(d_W_.get());
    if (chol_->Info() > 0)
      throw LatentNan("NaN or Inf occurred in the mode finding algorithm for the Laplace approximation "
                      "(Sigma^-1 + W not positive definite)");
    ++res.cg_its;   // factorizations of this evaluation (reported in the iteration info)
  };

  // ---- 2. mode finding (likelihoods.h:2780-3001)
  if (start == ModeStart::kZero) {
    HIP_CHECK(hipMemsetAsync(d_mode_.get(), 0, sizeof(double) * n, s_));
  } else if (start == ModeStart::kWarm) {
    d_mode_prev_.alloc(n);
    launch_copy(n, d_mode_.get(), d_mode_prev_.get(), s_);
    mode_prev_valid_ = true;
  }
  double sc[kLatentScalars];
  sa.mode = d_mode_.get();
  Scalars(sa, sc);
  if (std::isnan(sc[kSqLogDinv]) || std::isinf(sc[kSqLogDinv]))   // Vecchia_utils.cpp:1619-1630
    Fatal("The matrix D in the Vecchia approximation contains negative or zero values. "
          "This likely results from numerical instabilities ");
  double mll = sc[kSqLogLik] - 0.5 * sc[kSqQuad];
  const bool info_changes = !gauss;              // information_changes_during/after_mode_finding_
  const int maxit = gauss ? 1 : 1000;            // maxit_mode_newton_ (likelihoods.h:255, 12721)
  const int max_shrink = gauss ? 1 : 20;         // max_number_lr_shrinkage_steps_newton_ (:256, 12725)
  auto line_search_and_check = [&](int it, double gdd) -> bool {   // likelihoods.h:2967-2995, 11820-11870
    double lr = 1., mll_new = mll;
    for (int ih = 0; ih < max_shrink; ++ih) {
      if (ih == 0) launch_copy(n, d_mode_upd_.get(), d_mode_new_.get(), s_);
      else launch_axpby(n, 1. - lr, d_mode_.get(), lr, d_mode_upd_.get(), d_mode_new_.get(), s_);
      if (lik == kLikPoisson || lik == kLikGamma) launch_cap_mode_change(n, d_mode_.get(), d_mode_new_.get(), s_);
      sa.mode = d_mode_new_.get();
      Scalars(sa, sc);
      mll_new = sc[kSqLogLik] - 0.5 * sc[kSqQuad];
      if (mll_new < mll + kCArmijoC * lr * gdd || std::isnan(mll_new) || std::isinf(mll_new)) lr *= 0.5;
      else break;
    }
    std::swap(d_mode_, d_mode_new_);
    res.newton_its = it + 1;
    if (std::isnan(mll_new) || std::isinf(mll_new))
      throw LatentNan("NaN or Inf occurred in the mode finding algorithm for the Laplace approximation");
    const double dc = cfg.delta_conv_mode_finding;
    const bool term = (it == 0) ? std::fabs(mll_new - mll) < dc * std::fabs(mll) : (mll_new - mll) < dc * std::fabs(mll);
    mll = mll_new;
    return term;
  };
  const int newton_its = start == ModeStart::kKeep ? 0 : maxit;   // kKeep: the mode as it stands
  for (int it = 0; it < newton_its; ++it) {
    // rhs = W mode + d1 (:2920-2924); W changes with the mode for non-Gaussian likelihoods
    newton_prep(1, true);
    if (it == 0 || info_changes) factor();
    chol_->Solve(d_rhs_.get(), d_mode_upd_.get());
    double gdd = 0.;
    if (!gauss) {   // Armijo slope (:2957-2966): direction^T (Sigma^-1 + W) direction
      launch_axpby(n, 1., d_mode_upd_.get(), -1., d_mode_.get(), d_dir_.get(), s_);
      ApplyA(d_dir_.get(), d_Adir_.get(), b1.G.get(), 1);
      gdd = Dot1(d_dir_.get(), d_Adir_.get());
    }
    if (line_search_and_check(it, gdd)) break;
  }
  // derivatives / information at the mode, refactor when the information changed (:3008-3011, 3052-3066)
  newton_prep(1, false);
  if (info_changes || newton_its == 0) factor();
  const double two_sum_log_l = chol_->LogDet();
  sa.mode = d_mode_.get();
  sa.dw = nullptr;
  Scalars(sa, sc);
  // approx_marginal_ll = mll - sum log L_ii + 0.5 sum log D^-1 (:3067-3070); log|Sigma W + I| reported as
  // log|Sigma^-1 + W| + log|D|
  res.logdet = two_sum_log_l - sc[kSqLogDinv];
  res.nll = -(mll - 0.5 * res.logdet);

  if (want_grad) {
    // ---- 3. gradient (likelihoods.h:5207-5336): S = (Sigma^-1 + W)^-1 on the pattern of L
    double tr_bdb = 0., tr_da = 0.;
    chol_->SelectedInverse(&tr_bdb, &tr_da, d_diagS_.get());
    if (!gauss) {   // d_mll_d_mode = 0.5 diag(S) dW; (Sigma^-1 + W)^-1 d_mll_d_mode (:5244-5262)
      launch_chol_dmll(n, lik, aux, has_obs_ ? nullptr : d_y_.get(), d_mode_.get(),
                       has_off_ && !has_obs_ ? d_off_.get() : nullptr, Obs(), d_diagS_.get(), d_dmll_.get(), s_);
      chol_->Solve(d_dmll_.get(), d_vS_.get());
    }
    ScalarArgs sg = sa;
    sg.dBv = d_dBv_.get();
    sg.dD = d_dD_.get();
    sg.vS = gauss ? nullptr : d_vS_.get();
    Scalars(sg, sc);
    // marginal variance: SigmaI_deriv = -Sigma^-1, explicit += n / 2 (:5224-5226, 5265-5269)
    {
      double g = 0.5 * (-sc[kSqQuad] - tr_bdb) + 0.5 * n;
      if (!gauss) g += sc[kSqImpVar];   // - vS^T (-Sigma^-1 m)
      res.grad.push_back(g);
    }
    // range: SigmaI_deriv = dB^T D^-1 B + B^T D^-1 dB - B^T D^-1 dD D^-1 B (:5227-5231), explicit
    // += 0.5 sum D^-1 dD (:5270-5272)
    {
      double g = 0.5 * (2. * sc[kSqDQuadRng] - sc[kSqDDQuad] + tr_da) + 0.5 * sc[kSqDinvDD];
      if (!gauss) g -= sc[kSqImpRng];
      res.grad.push_back(g);
    }
    if (grad_f_vo != nullptr && has_obs_)
      Fatal("the gradient wrt the fixed effects of a latent model with repeated coordinates is not supported by "
            "gpboost_amd");
    if (grad_f_vo != nullptr) {   // wrt the fixed effects F (:5337-5369)
      d_gradf_.alloc(n);
      launch_grad_f(n, d_d1_.get(), gauss ? nullptr : d_dmll_.get(), d_W_.get(), gauss ? nullptr : d_vS_.get(),
                    d_gradf_.get(), s_);
      std::vector<double> gp(n);
      HIP_CHECK(hipMemcpyAsync(gp.data(), d_gradf_.get(), sizeof(double) * n, hipMemcpyDeviceToHost, s_));
      HIP_CHECK(hipStreamSynchronize(s_));
      for (int p = 0; p < n; ++p) grad_f_vo[vo_[p]] = gp[p];
    }
    // gamma shape on the log scale (:5304-5335, 10508-10524, 10856-10869)
    if (lik == kLikGamma && want_aux_grad) {
      DevBuf<double> rec((size_t)3 * n), red(3);
      launch_gamma_aux_rec(n, aux, d_y_.get(), has_off_ ? d_off_.get() : nullptr, d_mode_.get(), d_W_.get(),
                           d_dmll_.get(), d_d1_.get(), d_vS_.get(), rec.get(), s_);
      launch_sum_blocks(rec.get(), n, 3, red.get(), s_);
      double h[3];
      HIP_CHECK(hipMemcpyAsync(h, red.get(), sizeof(h), hipMemcpyDeviceToHost, s_));
      HIP_CHECK(hipStreamSynchronize(s_));
      const double neg = aux * (h[0] - n * (std::log(aux) + 1. - digamma_asa103(aux)) - sum_log_y_);
      res.grad.push_back(neg + 0.5 * h[1] + h[2]);
    }
    // gaussian error variance on the log scale: dW / dlog aux = -W, d_detmll = sum dW_i S_ii (:5304-5335)
    if (gauss && want_aux_grad) {
      std::vector<double> dS(n);
      HIP_CHECK(hipMemcpyAsync(dS.data(), d_diagS_.get(), sizeof(double) * n, hipMemcpyDeviceToHost, s_));
      HIP_CHECK(hipStreamSynchronize(s_));
      double tr = 0.;
      for (int p = 0; p < n; ++p) tr += (has_obs_ ? (double)obs_cnt_[p] : 1.) * dS[p];
      res.grad.push_back(sc[kSqRss] * (-0.5 / aux) + 0.5 * (has_obs_ ? n_obs_ : n) + 0.5 * (-1. / aux) * tr);
    }
  }
  HIP_CHECK(hipEventRecord(ev1_, s_));
  HIP_CHECK(hipEventSynchronize(ev1_));
  float ms = 0.f;
  HIP_CHECK(hipEventElapsedTime(&ms, ev0_, ev1_));
  res.ms_total = ms;
  if (std::getenv("GPBOOST_AMD_TIMING") != nullptr)
    std::fprintf(stderr, "[latent cholesky] %.2f ms: %d Newton steps, %d factorizations (last %.2f ms)\n", ms,
                 res.newton_its, res.cg_its, chol_->last_factor_ms());
  return res;
}

// Predictive (co)variance terms of PredictLaplaceApproxVecchia, Cholesky branch (likelihoods.h:6751-6811):
// Maux = L^-1 P Bpo^T (n x n_pred); d_V (n_pred x n, column-major) = sqrt(n) Maux^T, so that the moments of
// latent_pred_moments with nsim = n give Bpo (Sigma^-1 + W)^-1 Bpo^T exactly (V V^T / n = Maux^T Maux).
void LatentVecchia::PredVarChol(int n_pred, int mp, const int* nbr_vo, const double* d_Bpo, double* d_V) {
  if (!use_chol_ || !chol_) Fatal("PredVarChol: no Cholesky factor (evaluate the model first)");
  std::vector<int> nb_st((size_t)n_pred * mp);
  for (size_t e = 0; e < nb_st.size(); ++e) nb_st[e] = nbr_vo[e] >= 0 && nbr_vo[e] < n_ ? lab_[nbr_vo[e]] : -1;
  DevBuf<int> dnb(nb_st.size());
  HIP_CHECK(hipMemcpyAsync(dnb.get(), nb_st.data(), sizeof(int) * nb_st.size(), hipMemcpyHostToDevice, s_));
  const int chunk = std::max(1, std::min(n_pred, 256));
  DevBuf<double> cols((size_t)n_ * chunk), M((size_t)n_ * chunk);
  for (int p0 = 0; p0 < n_pred; p0 += chunk) {
    const int c = std::min(chunk, n_pred - p0);
    launch_chol_pred_cols(n_, c, mp, dnb.get() + (size_t)p0 * mp, d_Bpo + (size_t)p0 * mp, cols.get(), s_);
    chol_->ForwardCols(cols.get(), M.get(), c);
    launch_chol_transpose_scale(n_, c, M.get(), std::sqrt((double)n_), d_V + p0, n_pred, s_);
  }
  HIP_CHECK(hipStreamSynchronize(s_));
}

}  // namespace gpb_amd
