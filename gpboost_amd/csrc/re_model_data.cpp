// REModelAMD: linear regression covariates (GLS), stored data accessors, likelihood switching
// and the training-data random-effect predictions.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <limits>
#include <numeric>

#include "cov.h"
#include "covariates.h"
#include "kernels.h"
#include "re_model.h"
#include "vecchia_host.h"

namespace gpb_amd {

void REModelAMD::SetResponse(const double* y, const double* fixed_effects) {
  const int n = cfg_.n;
  y_raw_.assign(y, y + n);
  if (fixed_effects == nullptr) {
    SetY(y);
    return;
  }
  std::vector<double> r(n);
  for (int i = 0; i < n; ++i) r[i] = y[i] - fixed_effects[i];
  SetY(r.data());
}

void REModelAMD::SetLatentOffset(const double* fe) {
  if (fe == nullptr) {
    has_offset_ = false;
    offset_vo_.clear();
  } else {
    const int n = cfg_.n;
    offset_vo_.resize(n);
    for (int i = 0; i < n; ++i) offset_vo_[i] = fe[perm_[i]];
    has_offset_ = true;
  }
  if (lat()) lat()->SetOffset(has_offset_ ? offset_vo_.data() : nullptr);
  if (vif_lap_) vif_lap_->SetGradOffset(fe);   // data order: the reference's covariance gradient (vif_laplace.h)
}

void REModelAMD::SetResponseAndOffset(const double* y, const double* fixed_effects) {
  if (cfg_.latent) {
    if (y != nullptr) SetResponse(y, nullptr);
    SetLatentOffset(fixed_effects);
    return;
  }
  if (y == nullptr) {
    if (fixed_effects != nullptr) Fatal("'y_data' cannot be NULL when 'fixed_effects' is provided");
    return;
  }
  SetResponse(y, fixed_effects);
}

void REModelAMD::CalcGradientF(double* y, const double* fixed_effects, bool calc_cov_factor) {
  // re_model_template.h:3021-3043. Gaussian: the factor is recomputed at the current parameters
  // (deterministic, so equal to the existing one). Latent: calc_cov_factor re-runs the mode finding
  // from the current mode (CalcModePostRandEffCalcMLL, no InitializeModeAvec); without it the mode
  // of the last evaluation (e.g. OptimCovPar's last objective call) is used as it stands.
  UseDevice();
  if (world_ > 1) Fatal("CalcGradientF is only available on single-rank models");
  if (y == nullptr) Fatal("the output array 'y' is NULL");
  const int n = cfg_.n;
  if (!cov_pars_initialized_) {   // InitializeCovParsIfNotDefined (re_model.cpp:1142-1164)
    if (cfg_.latent && !y_set_) Fatal("Response variable data has not been set");
    InitCovParsIfNotDefined(cfg_.latent ? nullptr : y, nullptr);
  }
  if (cfg_.latent) {
    if (has_dup())
      Fatal("the gradient wrt the fixed effects of a latent model with repeated coordinates is not supported by "
            "gpboost_amd");
    SetLatentOffset(fixed_effects);
    if (!y_set_) Fatal("Response variable data has not been set");
    EnsureStructure();
    const double trafo[2] = {cov_pars_orig_[0], range_trafo(cfg_.cov_type, cov_pars_orig_[1])};
    const double aux = aux_pars_.empty() ? 1. : aux_pars_[0];
    std::vector<double> gvo(n);
    const auto start = (!calc_cov_factor && latent_evaluated_) ? LatentVecchia::ModeStart::kKeep
                                                               : LatentVecchia::ModeStart::kWarm;
    lat()->Eval(cfg_.cov_type, cfg_.lik, trafo, aux, iter, true, false, gvo.data(), start);
    latent_evaluated_ = true;
    for (int i = 0; i < n; ++i) y[perm_[i]] = gvo[i];
    return;
  }
  // Gaussian: SetY(y); CalcYAux(sigma2) -> Psi^-1 y / sigma2 (re_model_template.h:3036-3039)
  SetY(y);
  double trafo[3];
  TransformCovPars(cov_pars_orig_.data(), trafo);
  std::vector<double> yaux(n), dg(n);
  if (vif_) Fatal("the gradient wrt the fixed effects with gp_approx = 'full_scale_vecchia' is not supported by gpboost_amd");
  if (fitc_) {   // Woodbury y_aux of the FITC factor (CalcYAux, re_model_template.h:8898-8908)
    double sums[kVecchiaSums];
    UseDevice();
    fitc_->Eval(cfg_.cov_type, trafo[1], trafo[2], d_y_.get(), false, sums, last_kernel_ms_);
    if (!std::isfinite(sums[0])) Fatal("the FITC covariance is not positive definite (Cholesky failed)");
    fitc_->YAux(yaux.data());
    for (int i = 0; i < n; ++i) y[i] = yaux[i] / trafo[0];
    return;
  }
  if (!vecchia_) {
    dense_->PsiInvDiag(cfg_.cov_type, trafo[1], trafo[2], d_y_.get(), yaux.data(), dg.data());
    for (int i = 0; i < n; ++i) y[i] = yaux[i] / trafo[0];
    return;
  }
  PsiInvVecchia(trafo, yaux.data(), dg.data());
  for (int i = 0; i < n; ++i) y[perm_[i]] = yaux[i] / trafo[0];
}

std::vector<double> REModelAMD::ResidualResponse(const double* y, const double* fixed_effects) const {
  const int n = cfg_.n, p = num_covariates_;
  const double* yy = y != nullptr ? y : y_raw_.data();
  if (yy == nullptr || (y == nullptr && y_raw_.empty())) Fatal("Response variable data has not been set");
  const double* fe = fixed_effects != nullptr ? fixed_effects : (has_fixed_effects_ ? fixed_effects_.data() : nullptr);
  std::vector<double> r(yy, yy + n);
  if (fe != nullptr)
    for (int i = 0; i < n; ++i) r[i] -= fe[i];
  if (has_covariates_)   // UpdateFixedEffects (y_ = y - X beta - offset)
    for (int a = 0; a < p; ++a)
      for (int i = 0; i < n; ++i) r[i] -= X_cov_[(size_t)a * n + i] * coef_[a];
  return r;
}

void REModelAMD::AddLinearPredictor(const double* X_pred, int n_pred, double* mu) const {
  if (!has_covariates_) Fatal("the model has no linear regression covariates ('X_pred' must be NULL)");
  if (X_pred == nullptr) Fatal("covariate data for prediction ('X_pred') is missing for a model with covariates");
  for (int a = 0; a < num_covariates_; ++a)
    for (int p = 0; p < n_pred; ++p) mu[p] += X_pred[(size_t)a * n_pred + p] * coef_[a];
}

// [X | y - offset] in the layout of the model's solver: Vecchia order row-major on the device
// (Vecchia models), original order column-major on the host (dense, passed to DenseSolver::Gram).
void REModelAMD::UploadCovariates() {
  if (!vecchia_) return;
  const int n = cfg_.n, p = num_covariates_, c = p + 1;
  const double* fe = has_fixed_effects_ ? fixed_effects_.data() : nullptr;
  std::vector<double> Z((size_t)n * c);
  for (int i = 0; i < n; ++i) {
    const int o = perm_[i];
    for (int a = 0; a < p; ++a) Z[(size_t)i * c + a] = X_cov_[(size_t)a * n + o];
    Z[(size_t)i * c + p] = y_raw_[o] - (fe ? fe[o] : 0.);
  }
  d_Zcov_.alloc(Z.size());
  HIP_CHECK(hipMemcpyAsync(d_Zcov_.get(), Z.data(), sizeof(double) * Z.size(), hipMemcpyHostToDevice, stream_));
  HIP_CHECK(hipStreamSynchronize(stream_));
}

std::vector<double> REModelAMD::Gram(const double* trafo) {
  const int n = cfg_.n, p = num_covariates_, c = p + 1;
  if (fitc_ || vif_)
    Fatal("linear regression covariates with gp_approx = '%s' are not supported by gpboost_amd", cfg_.gp_approx.c_str());
  if (!vecchia_) {
    std::vector<double> Z((size_t)n * c), G((size_t)c * c);
    const double* fe = has_fixed_effects_ ? fixed_effects_.data() : nullptr;
    std::copy(X_cov_.begin(), X_cov_.end(), Z.begin());
    for (int i = 0; i < n; ++i) Z[(size_t)p * n + i] = y_raw_[i] - (fe ? fe[i] : 0.);
    dense_->Gram(cfg_.cov_type, trafo[1], trafo[2], Z.data(), c, G.data());
    return G;
  }
  if (world_ > 1) Fatal("linear regression covariates are only supported on single-rank models");
  EnsureStructure();
  const int m = cfg_.num_neighbors;
  d_Bf_.alloc((size_t)n * m);
  d_Df_.alloc(n);
  VecchiaRowsArgs a{};
  a.X = d_X_.get();
  a.Y = nullptr;   // factor mode: B rows and D^-1 to HBM
  a.nbr = d_nbr_.get();
  a.n = n; a.d = cfg_.d; a.m = m; a.r0 = 0; a.r1 = n;
  a.var = trafo[1]; a.phi = trafo[2];
  a.diag_mult = 1.; a.diag_add = 1.; a.d_nugget = 1.;
  a.Dinv_out = d_Df_.get();
  a.B_out = d_Bf_.get();
  launch_vecchia_rows(cfg_.cov_type, a, stream_);
  const int npairs = c * (c + 1) / 2;
  d_gram_part_.alloc((size_t)vecchia_gram_blocks(n) * npairs);
  d_gram_out_.alloc(npairs);
  launch_vecchia_gram(n, m, c, d_nbr_.get(), d_Bf_.get(), d_Df_.get(), d_Zcov_.get(), d_gram_part_.get(),
                      d_gram_out_.get(), stream_);
  std::vector<double> packed(npairs);
  HIP_CHECK(hipMemcpyAsync(packed.data(), d_gram_out_.get(), sizeof(double) * npairs, hipMemcpyDeviceToHost, stream_));
  HIP_CHECK(hipStreamSynchronize(stream_));
  return unpack_gram(packed.data(), c);
}

EvalResult REModelAMD::EvalTrafoWls(const double* trafo, bool want_grad, bool fatal_on_nan,
                                    std::vector<double>* beta_out) {
  // optim_utils.h:297-313: CalcCovFactorOrModeAndNegLL, ProfileOutCoef (beta by GLS, y_ = residuals),
  // EvalNegLogLikelihoodOnlyUpdateFixedEffects, ProfileOutSigma2; the gradient on the residuals
  UseDevice();
  const std::vector<double> G = Gram(trafo);
  for (double v : G)
    if (!std::isfinite(v)) {
      if (fatal_on_nan) Fatal("NaN or Inf occurred in X^T Psi^-1 X");
      EvalResult bad;
      bad.nll = std::numeric_limits<double>::quiet_NaN();
      bad.grad.assign(2, 0.);
      return bad;
    }
  coef_ = gls_coef(G, num_covariates_);
  coef_std_dev_valid_ = false;
  if (beta_out) *beta_out = coef_;
  const std::vector<double> r = ResidualResponse(y_raw_.data(), nullptr);
  SetY(r.data());
  return EvalTrafo(trafo, want_grad, 1, fatal_on_nan);
}

void REModelAMD::GetCoef(double* out, bool calc_std_dev) {
  if (!has_covariates_ || (int)coef_.size() != num_covariates_)
    Fatal("Regresion coefficients have not been estimated or correctly set ");
  const int p = num_covariates_;
  std::copy(coef_.begin(), coef_.end(), out);
  if (!calc_std_dev) return;
  if (!coef_std_dev_valid_) {
    if (p >= cfg_.n) {   // re_model_template.h:9801-9806
      Warning("Sample size too small to calculate standard deviations for coefficients");
      coef_std_dev_.assign(p, std::numeric_limits<double>::quiet_NaN());
    } else {
      double trafo[3];
      TransformCovPars(cov_pars_orig_.data(), trafo);
      const std::vector<double> G = Gram(trafo);
      coef_std_dev_ = gls_coef_std_dev(G, p, cov_pars_orig_[0]);
    }
    coef_std_dev_valid_ = true;
  }
  std::copy(coef_std_dev_.begin(), coef_std_dev_.end(), out + p);
}

void REModelAMD::EnsureTransposedLists() {
  if (d_tptr_.get() != nullptr) return;
  const int n = cfg_.n, m = cfg_.num_neighbors;
  std::vector<int> tptr(n + 1, 0);
  for (int i = 0; i < n; ++i) {
    const int k = std::min(i, m);
    for (int r = 0; r < k; ++r) ++tptr[nbr_[(size_t)i * m + r] + 1];
  }
  for (int j = 0; j < n; ++j) tptr[j + 1] += tptr[j];
  const int nnz = tptr[n];
  std::vector<int> trow(std::max(nnz, 1)), tslot(std::max(nnz, 1)), fill(tptr.begin(), tptr.end() - 1);
  for (int i = 0; i < n; ++i) {   // rows ascending within every column
    const int k = std::min(i, m);
    for (int r = 0; r < k; ++r) {
      const int j = nbr_[(size_t)i * m + r];
      trow[fill[j]] = i;
      tslot[fill[j]] = i * m + r;
      ++fill[j];
    }
  }
  d_tptr_.alloc(n + 1);
  d_trow_.alloc(trow.size());
  d_tslot_.alloc(tslot.size());
  HIP_CHECK(hipMemcpyAsync(d_tptr_.get(), tptr.data(), sizeof(int) * (n + 1), hipMemcpyHostToDevice, stream_));
  HIP_CHECK(hipMemcpyAsync(d_trow_.get(), trow.data(), sizeof(int) * trow.size(), hipMemcpyHostToDevice, stream_));
  HIP_CHECK(hipMemcpyAsync(d_tslot_.get(), tslot.data(), sizeof(int) * tslot.size(), hipMemcpyHostToDevice, stream_));
  HIP_CHECK(hipStreamSynchronize(stream_));
}

void REModelAMD::PredictTrainingDataRandomEffects(const double* cov_pars, const double* y, double* out,
                                                  const double* fixed_effects, bool calc_var) {
  // re_model.cpp PredictTrainingDataRandomEffects: cov_pars on the original scale (NULL: the
  // estimated / last ones); y NULL: the response set before
  UseDevice();
  if (world_ > 1) Fatal("PredictTrainingDataRandomEffects is only available on single-rank models");
  const int n = cfg_.n;
  std::vector<double> cp;
  if (cov_pars != nullptr) cp.assign(cov_pars, cov_pars + num_cov_pars());
  else if (!last_cov_pars_.empty()) cp = last_cov_pars_;
  else Fatal("Covariance parameters have not been estimated or are not given.");
  if (cfg_.latent) {
    if (calc_var)
      Fatal("PredictTrainingDataRandomEffects: predictive variances of latent (Laplace) models are not supported by "
            "gpboost_amd");
    if (y != nullptr) SetResponse(y, nullptr);
    if (!y_set_) Fatal("Response variable data is not provided and has not been set before");
    SetLatentOffset(ResolveOffset(fixed_effects));   // re_model_template.h:4032-4039
    EvalLatent(cp.data(), false);   // the posterior mode at cov_pars
    std::vector<double> mvo(nu_);
    lat()->GetMode(mvo.data());
    for (int i = 0; i < n; ++i) out[perm_[i]] = mvo[has_dup() ? obs_row_[i] : i];   // Z mode
    return;
  }
  const std::vector<double> r = ResidualResponse(y, fixed_effects);
  SetY(r.data());
  double trafo[3];
  TransformCovPars(cp.data(), trafo);
  std::vector<double> yaux(n), dg(n);
  if (fitc_ || vif_)
    Fatal("training-data random-effect predictions with gp_approx = '%s' are not supported by gpboost_amd",
          cfg_.gp_approx.c_str());
  if (!vecchia_) {
    dense_->PsiInvDiag(cfg_.cov_type, trafo[1], trafo[2], d_y_.get(), yaux.data(), dg.data());
    for (int i = 0; i < n; ++i) {
      out[i] = r[i] - yaux[i];
      if (calc_var) out[n + i] = trafo[0] * (1. - dg[i]);
    }
    return;
  }
  PsiInvVecchia(trafo, yaux.data(), dg.data());
  for (int i = 0; i < n; ++i) {   // Vecchia order -> original (data_indices_per_cluster_)
    const int o = perm_[i];
    out[o] = r[o] - yaux[i];
    if (calc_var) out[n + o] = trafo[0] * (1. - dg[i]);
  }
}

// Exact Vecchia: Psi^-1 y (the device response) and diag(Psi^-1), Vecchia order, via the row
// kernel's factor mode and the transposed lists.
void REModelAMD::PsiInvVecchia(const double* trafo, double* yaux, double* diag) {
  const int n = cfg_.n;
  EnsureStructure();
  EnsureTransposedLists();
  const int m = cfg_.num_neighbors;
  d_Bf_.alloc((size_t)n * m);
  d_Df_.alloc(n);
  VecchiaRowsArgs a{};
  a.X = d_X_.get();
  a.Y = nullptr;
  a.nbr = d_nbr_.get();
  a.n = n; a.d = cfg_.d; a.m = m; a.r0 = 0; a.r1 = n;
  a.var = trafo[1]; a.phi = trafo[2];
  a.diag_mult = 1.; a.diag_add = 1.; a.d_nugget = 1.;
  a.Dinv_out = d_Df_.get();
  a.B_out = d_Bf_.get();
  launch_vecchia_rows(cfg_.cov_type, a, stream_);
  DevBuf<double> u(n), ya(n), dd(n);
  launch_vecchia_psi_inv_diag(n, m, d_nbr_.get(), d_tptr_.get(), d_trow_.get(), d_tslot_.get(), d_Bf_.get(),
                              d_Df_.get(), d_y_.get(), u.get(), ya.get(), dd.get(), stream_);
  HIP_CHECK(hipMemcpyAsync(yaux, ya.get(), sizeof(double) * n, hipMemcpyDeviceToHost, stream_));
  HIP_CHECK(hipMemcpyAsync(diag, dd.get(), sizeof(double) * n, hipMemcpyDeviceToHost, stream_));
  HIP_CHECK(hipStreamSynchronize(stream_));
}

void REModelAMD::SetLikelihood(const std::string& likelihood) {
  if (likelihood == cfg_.likelihood) return;
  if (cov_pars_initialized_ && num_it_ > 0)   // re_model.cpp:142-147
    Fatal("Cannot change likelihood after a model has been estimated ");
  ModelConfig c = cfg_;
  c.likelihood = likelihood;
  const int lik = parse_likelihood(likelihood);
  const bool dense = c.gp_approx == "none";
  const bool latent = c.gp_approx == "vecchia_latent" || ((vecchia_ || fitc_ || vif_ || dense) && lik != kLikGaussian);
  if (vif_) {   // full-scale Vecchia: the Laplace solver on the same inducing points and neighbours (Cholesky)
    if (latent && !vif_lap_) {
      if (c.ind_points_selection == "random")
        Fatal("Method 'random' is not supported for finding inducing points in the full-scale-vecchia approximation "
              "for non-Gaussian data");
      vif_lap_.reset(new VifLaplace(vif_.get(), vif_nbr_, coords_vo_, stream_));
    } else if (!latent) {
      vif_lap_.reset();
    }
    c.matrix_inversion_method = "cholesky";
  } else if (dense) {   // gp_approx = "none": DenseLaplace (Cholesky) for the Laplace likelihoods, DenseSolver for gaussian
    if (latent && !dense_lap_) {
      std::vector<int> uniq, idx;
      unique_locations(coords_.data(), cfg_.n, cfg_.d, uniq, idx);
      if ((int)uniq.size() < cfg_.n)
        Fatal("gp_approx = 'none' with likelihood '%s' and duplicate coordinates is not supported by gpboost_amd",
              likelihood.c_str());
      dense_.reset();
      dense_lap_.reset(new DenseLaplace(cfg_.n, cfg_.d, d_X_.get(), stream_));
      perm_.resize(cfg_.n);
      std::iota(perm_.begin(), perm_.end(), 0);
    } else if (!latent) {
      dense_lap_.reset();
      if (!dense_) dense_.reset(new DenseSolver(cfg_.n, cfg_.d, d_X_.get(), stream_));
    }
    c.matrix_inversion_method = "cholesky";
  } else if (fitc_) {   // FITC: the Laplace solver on the same inducing points (Cholesky either way)
    if (latent && !fitc_lap_) {
      fitc_lap_.reset(new FitcLaplace(fitc_.get(), stream_));
      perm_.resize(cfg_.n);
      std::iota(perm_.begin(), perm_.end(), 0);
    } else if (!latent) {
      fitc_lap_.reset();
    }
  } else if (latent && !cfg_.latent) {   // exact -> latent: distinct coordinates, iterative solver (re_model_template.h:568-571)
    std::vector<int> ord(cfg_.n);
    for (int i = 0; i < cfg_.n; ++i) ord[i] = i;
    const int d = cfg_.d;
    auto row = [&](int i) { return coords_.data() + (size_t)i * d; };
    std::sort(ord.begin(), ord.end(), [&](int a, int b) { return std::lexicographical_compare(row(a), row(a) + d, row(b), row(b) + d); });
    for (int k = 1; k < cfg_.n; ++k)
      if (std::equal(row(ord[k - 1]), row(ord[k - 1]) + d, row(ord[k])))
        Fatal("Cannot change the likelihood to '%s' from 'gaussian' when gp_approx = '%s' and having duplicate coordinates ",
              likelihood.c_str(), cfg_.gp_approx.c_str());
    c.matrix_inversion_method = "iterative";
  } else if (!latent && cfg_.latent) {
    c.matrix_inversion_method = "cholesky";
    if (has_dup()) {   // back to all points (the exact Gaussian Vecchia path keeps every observation)
      const int n = cfg_.n, d = cfg_.d;
      coords_vo_.resize((size_t)n * d);
      for (int i = 0; i < n; ++i)
        for (int q = 0; q < d; ++q) coords_vo_[(size_t)i * d + q] = coords_[(size_t)perm_[i] * d + q];
      obs_row_.clear();
      nu_ = n;
      row_end_ = n;
      d_X_.alloc((size_t)n * d);
      HIP_CHECK(hipMemcpyAsync(d_X_.get(), coords_vo_.data(), sizeof(double) * n * d, hipMemcpyHostToDevice, stream_));
      HIP_CHECK(hipStreamSynchronize(stream_));
    }
  }
  c.lik = lik;
  c.latent = latent;
  cfg_ = c;
  aux_pars_.clear();
  if (cfg_.latent && (cfg_.lik == kLikGaussian || cfg_.lik == kLikGamma)) aux_pars_ = {1.};
  latent_.reset();
  structure_built_ = false;
  y_set_ = false;
  last_cov_pars_.clear();
  cov_pars_initialized_ = !init_cov_pars_.empty() && (int)init_cov_pars_.size() == num_cov_pars();
  if (!cov_pars_initialized_) { init_cov_pars_.clear(); cov_pars_orig_.clear(); init_used_.clear(); }
}

void REModelAMD::GetResponseData(double* y) const {
  if (y_raw_.empty()) Fatal("Respone variable data has not been set");
  std::copy(y_raw_.begin(), y_raw_.end(), y);
}

void REModelAMD::GetCovariateData(double* X) const {
  if (!has_covariates_) Fatal("Model does not have covariates for a linear predictor");
  std::copy(X_cov_.begin(), X_cov_.end(), X);
}

void REModelAMD::GetOffsetData(double* fe) const {
  if (!has_fixed_effects_) Fatal("Model does not have an offset term ");
  std::copy(fixed_effects_.begin(), fixed_effects_.end(), fe);
}

void REModelAMD::SetOffsetData(const double* fe) {
  if (fe == nullptr) Fatal("fixed_effects is NULL");
  fixed_effects_.assign(fe, fe + cfg_.n);
  has_fixed_effects_ = true;
}

void REModelAMD::SetInitAuxPars(const double* aux) {
  SetAuxPars(aux);
  aux_pars_set_ = true;
  init_aux_pars_.assign(aux, aux + aux_pars_.size());
}

void REModelAMD::GetInitAuxPars(double* out) const {
  for (int k = 0; k < num_aux_pars(); ++k) out[k] = init_aux_pars_.empty() ? -1. : init_aux_pars_[k];
}

void REModelAMD::SetOptimizerNames(const char* optimizer_cov, const char* optimizer_coef, const char* preconditioner) {
  if (optimizer_cov != nullptr && optimizer_cov[0] != '\0') optimizer_cov_ = optimizer_cov;
  if (optimizer_coef != nullptr && optimizer_coef[0] != '\0') {
    const std::string o(optimizer_coef);
    if (o != "wls" && o != "lbfgs")
      Fatal("Optimizer option '%s' is not supported for linear regression coefficients by gpboost_amd (supported: wls)",
            o.c_str());
    optimizer_coef_ = o;
  }
  if (preconditioner != nullptr && preconditioner[0] != '\0') cg_preconditioner_type_ = "vadu";
}

std::string REModelAMD::cg_preconditioner_type() const {
  // InitializeDefaultSettings (re_model_template.h:6501-6514): "vadu" for latent Vecchia models
  if (!cg_preconditioner_type_.empty()) return cg_preconditioner_type_;
  return cfg_.latent ? "vadu" : "";
}

}  // namespace gpb_amd
