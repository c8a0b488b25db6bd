// GroupedModel implementation: configuration, response handling, the combination of GroupedRE's
// device sums into the negative log-likelihood and its gradient, and the L-BFGS fit.
#include "grouped_model.h"

#include <cmath>
#include <cstdlib>
#include <limits>
#include <unordered_map>

namespace gpb_amd {

std::vector<std::vector<int>> parse_group_levels(int n, int K, const char* re_group_data,
                                                 std::vector<std::unordered_map<std::string, int>>* label_index) {
  if (re_group_data == nullptr) Fatal("re_group_data is NULL");
  std::vector<std::vector<int>> levels(K, std::vector<int>(n));
  if (label_index) label_index->assign(K, {});
  const char* p = re_group_data;
  for (int k = 0; k < K; ++k) {
    std::unordered_map<std::string, int> local;
    std::unordered_map<std::string, int>& index = label_index ? (*label_index)[k] : local;
    index.reserve(1024);
    for (int i = 0; i < n; ++i) {
      std::string label(p);
      p += label.size() + 1;
      auto it = index.find(label);
      if (it == index.end()) it = index.emplace(std::move(label), (int)index.size()).first;
      levels[k][i] = it->second;
    }
  }
  return levels;
}

GroupedModel::GroupedModel(int n, const std::vector<std::vector<int>>& levels, const std::string& mim, int seed,
                           std::vector<std::unordered_map<std::string, int>> label_index)
    : n_(n), mim_(mim), levels_(levels), label_index_(std::move(label_index)) {
  (void)seed;   // grouped models draw no random numbers at construction (probes use seed_rand_vec_trace)
  if (n <= 0) Fatal("num_data must be > 0");
  const int K = (int)levels.size();
  if (K < 1) Fatal("num_re_group must be > 0");
  if (mim_ == "default") mim_ = K > 1 ? "iterative" : "cholesky";
  if (mim_ != "iterative" && mim_ != "cholesky")
    Fatal("Matrix inversion method '%s' is not supported.", mim_.c_str());
  if (mim_ == "iterative" && K == 1)   // CheckCompatibilitySpecialOptions (re_model_template.h:6698-6702)
    Fatal("Cannot use matrix_inversion_method = 'iterative' if there is only a single-level grouped random effects. "
          "Use matrix_inversion_method = 'cholesky' instead (this is very fast). Iterative methods are for multiple "
          "grouped random effects ");
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
    Fatal("no HIP device visible: gpboost_amd has no CPU fallback");
  if (const char* dev = std::getenv("GPBOOST_AMD_DEVICE")) {
    device_ = std::atoi(dev);
    if (device_ < 0 || device_ >= ndev) Fatal("GPBOOST_AMD_DEVICE=%d but %d device(s) visible", device_, ndev);
  } else {
    HIP_CHECK(hipGetDevice(&device_));
  }
  UseDevice();
  HIP_CHECK(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));
  re_.reset(new GroupedRE(n, levels, stream_));
}

GroupedModel::~GroupedModel() {
  re_.reset();
  if (stream_) (void)hipStreamDestroy(stream_);
}

void GroupedModel::UseDevice() const { HIP_CHECK(hipSetDevice(device_)); }

void GroupedModel::AttachGP(int d, const double* coords_colmajor, int cov_type, int seed) {
  if (d < 1 || d > 3) Fatal("dim_gp_coords = %d is not supported by gpboost_amd's dense path (1..3)", d);
  if (coords_colmajor == nullptr) Fatal("gp_coords_data is NULL");
  if (re_->K() > 8) Fatal("GP + grouped random effects: at most 8 grouped effects are supported by gpboost_amd");
  if (iterative())
    Fatal("matrix_inversion_method = 'iterative' is not supported for GP + grouped random effects models by "
          "gpboost_amd (use 'cholesky')");
  UseDevice();
  gp_d_ = d;
  cov_type_ = cov_type;
  seed_ = seed;
  coords_.resize((size_t)n_ * d);
  for (int i = 0; i < n_; ++i)
    for (int q = 0; q < d; ++q) coords_[(size_t)i * d + q] = coords_colmajor[(size_t)q * n_ + i];
  const int K = re_->K();
  std::vector<int> lev((size_t)K * n_);
  for (int k = 0; k < K; ++k)
    for (int i = 0; i < n_; ++i) lev[(size_t)k * n_ + i] = levels_[k][i];
  d_X_.alloc(coords_.size());
  d_lev_.alloc(lev.size());
  d_y_.alloc(n_);
  HIP_CHECK(hipMemcpyAsync(d_X_.get(), coords_.data(), sizeof(double) * coords_.size(), hipMemcpyHostToDevice, stream_));
  HIP_CHECK(hipMemcpyAsync(d_lev_.get(), lev.data(), sizeof(int) * lev.size(), hipMemcpyHostToDevice, stream_));
  HIP_CHECK(hipStreamSynchronize(stream_));
  dense_.reset(new DenseSolver(n_, d, d_X_.get(), stream_));
}

void GroupedModel::ToTrafo(const double* orig, double* trafo) const {
  const int K = re_->K();
  trafo[0] = orig[0];
  for (int k = 0; k < K; ++k) trafo[1 + k] = orig[1 + k] / orig[0];
  if (has_gp()) {
    trafo[1 + K] = orig[1 + K] / orig[0];
    trafo[2 + K] = range_trafo(cov_type_, orig[2 + K]);
  }
}

void GroupedModel::ToOrig(const double* trafo, double sigma2, double* orig) const {
  const int K = re_->K();
  orig[0] = sigma2;
  for (int k = 0; k < K; ++k) orig[1 + k] = trafo[1 + k] * sigma2;
  if (has_gp()) {
    orig[1 + K] = trafo[1 + K] * sigma2;
    orig[2 + K] = range_back(cov_type_, trafo[2 + K]);
  }
}

void GroupedModel::SetResponseAndOffset(const double* y, const double* fixed_effects) {
  if (y == nullptr && fixed_effects == nullptr) {
    if (!y_set_) Fatal("response variable y has not been set");
    return;
  }
  if (y != nullptr) y_raw_.assign(y, y + n_);
  if (y_raw_.empty()) Fatal("response variable y has not been set");
  y_ = y_raw_;
  if (fixed_effects != nullptr)
    for (int i = 0; i < n_; ++i) y_[i] -= fixed_effects[i];
  for (int i = 0; i < n_; ++i)
    if (std::isnan(y_[i]) || std::isinf(y_[i])) Fatal("NaN or Inf in response variable / label ");
  UseDevice();
  re_->SetY(y_.data());
  if (has_gp()) {
    HIP_CHECK(hipMemcpyAsync(d_y_.get(), y_.data(), sizeof(double) * n_, hipMemcpyHostToDevice, stream_));
    HIP_CHECK(hipStreamSynchronize(stream_));
  }
  y_set_ = true;
}

void GroupedModel::GetResponseData(double* y) const {
  if (y_raw_.empty()) Fatal("response variable y has not been set");
  std::copy(y_raw_.begin(), y_raw_.end(), y);
}

EvalResult GroupedModel::Eval(const double* cov_pars_orig, bool want_grad, int profile) {
  const int P = num_cov_pars();
  for (int k = 0; k < P; ++k)
    if (!(cov_pars_orig[k] > 0.)) Fatal("covariance parameters must be > 0");
  std::vector<double> trafo(P);   // TransformCovPars (re_comp.h: sigma_k^2 / sigma^2; the GP range transform)
  ToTrafo(cov_pars_orig, trafo.data());
  EvalResult r = EvalTrafo(trafo.data(), want_grad, profile);
  last_cov_pars_.assign(cov_pars_orig, cov_pars_orig + P);
  if (profile) ToOrig(trafo.data(), r.sigma2, last_cov_pars_.data());
  return r;
}

EvalResult GroupedModel::EvalTrafo(const double* trafo, bool want_grad, int profile, bool fatal_on_nan) {
  if (!y_set_) Fatal("response variable y has not been set");
  UseDevice();
  if (has_gp()) return EvalDense(trafo, want_grad, profile, fatal_on_nan);
  const int K = re_->K();
  GroupedParts parts;
  re_->Eval(trafo + 1, want_grad, iterative(), num_iter_ > 0, iter, parts);
  last_cg_its_ = parts.cg_its;
  last_lanczos_ = parts.lanczos_steps;
  const double q = parts.yTPsiInvy;
  const double sigma2 = profile ? q / n_ : trafo[0];   // ProfileOutSigma2 (re_model_template.h:2407)
  EvalResult res;
  res.sigma2 = sigma2;
  // CalcNegLogLikelihood (Gaussian, re_model_template.h:2880-2890)
  res.nll = q / 2. / sigma2 + parts.logdet / 2. + n_ / 2. * (std::log(sigma2) + std::log(2. * M_PI));
  if (!std::isfinite(res.nll)) {
    if (fatal_on_nan) Fatal("NaN or Inf occurred in the negative log-likelihood");
    res.nll = std::numeric_limits<double>::quiet_NaN();
  }
  if (want_grad) {   // CalcGradPars_Only_Grouped_REs_Woodbury_GaussLikelihood_Cluster_i (:2242-2391)
    int off = 0;
    res.grad.assign(profile ? K : K + 1, 0.);
    if (!profile) {
      res.grad[0] = -q / sigma2 / 2. + n_ / 2.;
      off = 1;
    }
    for (int k = 0; k < K; ++k) res.grad[off + k] = -parts.quad[k] / sigma2 / 2. + parts.trace[k] / 2.;
  }
  last_nll_ = res.nll;
  return res;
}

EvalResult GroupedModel::EvalDense(const double* trafo, bool want_grad, int profile, bool fatal_on_nan) {
  // Psi = sum_k tau_k Z_k Z_k^T + v K(phi) + I on the dense path; gradient wrt the log of the transformed
  // parameters [nugget], tau_1 .. tau_K, v, phi (CalcGradPars dense, re_model_template.h:1798-1818, with the
  // grouped components' dPsi / dlog tau_k = tau_k Z_k Z_k^T)
  const int K = re_->K();
  for (int k = 1; k < K + 3; ++k)
    if (!(trafo[k] > 0.)) Fatal("covariance parameters must be > 0");
  dense_->SetGrouped(K, d_lev_.get(), trafo + 1);
  double sums[6], kms[2];
  dense_->Eval(cov_type_, trafo[1 + K], trafo[2 + K], d_y_.get(), want_grad, sums, kms);
  const double q = sums[1];
  const double sigma2 = profile ? q / n_ : trafo[0];
  EvalResult res;
  res.sigma2 = sigma2;
  res.nll = q / 2. / sigma2 + sums[0] / 2. + n_ / 2. * (std::log(sigma2) + std::log(2. * M_PI));
  if (!std::isfinite(res.nll)) {
    if (fatal_on_nan) Fatal("NaN or Inf occurred in the negative log-likelihood");
    res.nll = std::numeric_limits<double>::quiet_NaN();
  }
  if (want_grad) {
    std::vector<double> s2(K), yaux(n_);
    dense_->GroupedTraces(s2.data(), yaux.data());
    const int off = profile ? 0 : 1;
    res.grad.assign(off + K + 2, 0.);
    if (!profile) res.grad[0] = -q / sigma2 / 2. + n_ / 2.;
    for (int k = 0; k < K; ++k) {   // y_aux^T dPsi_k y_aux = tau_k sum over levels of (sum of y_aux)^2
      std::vector<double> lsum(re_->levels_per_effect()[k], 0.);
      for (int i = 0; i < n_; ++i) lsum[levels_[k][i]] += yaux[i];
      double quad = 0.;
      for (double v : lsum) quad += v * v;
      quad *= trafo[1 + k];
      res.grad[off + k] = -quad / sigma2 / 2. + s2[k] / 2.;
    }
    res.grad[off + K] = sums[2] / sigma2 + sums[4] / 2.;
    res.grad[off + K + 1] = sums[3] / sigma2 + sums[5] / 2.;
  }
  last_nll_ = res.nll;
  return res;
}

void GroupedModel::SetOptimSettings(const double* init_cov_pars, double lr, int max_iter, double delta_rel_conv,
                                    const char* optimizer, int m_lbfgs) {
  if (optimizer != nullptr && optimizer[0] != '\0') {
    const std::string o(optimizer);
    if (o != "lbfgs" && o != "nelder_mead" && !is_internal_optimizer(o))
      Fatal("Optimizer option '%s' is not supported for covariance parameters by gpboost_amd (supported: lbfgs, "
            "gradient_descent, fisher_scoring, nelder_mead)", optimizer);
    isettings_.optimizer = o == "lbfgs" ? "" : o;
    optimizer_name_ = o;
  }
  isettings_.lr = lr;
  isettings_.max_iter = max_iter;
  isettings_.delta = delta_rel_conv < 0. ? (isettings_.optimizer == "nelder_mead" ? 1e-8 : 1e-6) : delta_rel_conv;
  if (init_cov_pars != nullptr) {
    init_cov_pars_.assign(init_cov_pars, init_cov_pars + num_cov_pars());
    for (double v : init_cov_pars_)
      if (!(v > 0.)) Fatal("init_cov_pars must be > 0");
    cov_pars_orig_ = init_cov_pars_;
    cov_pars_initialized_ = true;
  }
  optim_.initial_step_factor = lr < 0. ? 1. : lr;
  optim_.max_iterations = max_iter;
  optim_.delta = delta_rel_conv < 0. ? 1e-6 : delta_rel_conv;
  if (m_lbfgs > 0) optim_.m = m_lbfgs;
}

void GroupedModel::SetPreconditioner(const char* preconditioner) {
  if (preconditioner == nullptr || preconditioner[0] == '\0') return;
  const std::string p(preconditioner);
  if (p != "ssor")   // SUPPORTED_PRECONDITIONERS_GROUPED_RE_ (re_model_template.h:5410) minus the ones not built
    Fatal("cg_preconditioner_type '%s' is not supported for grouped random effects by gpboost_amd (supported: ssor)",
          p.c_str());
}

void GroupedModel::FindInitCovPar(const double* y, double* trafo) const {
  // re_model_template.h:4388-4485 (Gaussian): sigma^2 = sample variance / 2, every component's marginal
  // variance 1 / num_comps on the transformed scale; the GP range from the median distance (cov_fcts.h
  // FindInitCovPar, draws from the model's mt19937(seed) when n > 1000)
  double mean = 0., var = 0.;
  for (int i = 0; i < n_; ++i) mean += y[i];
  mean /= n_;
  for (int i = 0; i < n_; ++i) var += (y[i] - mean) * (y[i] - mean);
  var /= (n_ - 1);
  const int K = re_->K(), comps = K + (has_gp() ? 1 : 0);
  trafo[0] = var / 2.;
  for (int k = 0; k < K; ++k) trafo[1 + k] = 1. / comps;
  if (has_gp()) {
    trafo[1 + K] = 1. / comps;
    std::mt19937 rng((std::mt19937::result_type)seed_);
    trafo[2 + K] = init_range_trafo(coords_, gp_d_, cov_type_, rng);
  }
}

void GroupedModel::GetInitCovPar(double* out) const {
  const std::vector<double>& v = !init_cov_pars_.empty() ? init_cov_pars_ : init_used_;
  for (int k = 0; k < num_cov_pars(); ++k) out[k] = v.empty() ? -1. : v[k];
}

namespace {

// EvalLLforLBFGSpp with the error variance profiled out (optim_utils.h:269-313): x = log tau. The
// value and gradient come from one device evaluation, as the reference's gradient call reuses the
// state of the preceding likelihood evaluation at the same point.
class GroupedProfiledObjective : public LbfgsObjective {
 public:
  explicit GroupedProfiledObjective(GroupedModel* m) : m_(m) {}
  double Eval(const std::vector<double>& x, std::vector<double>& grad, bool eval_ll, bool calc_grad,
              bool) override {
    if (eval_ll || !(has_ && x == x_)) {
      std::vector<double> trafo(1 + x.size());
      trafo[0] = 1.;
      for (size_t k = 0; k < x.size(); ++k) trafo[1 + k] = std::exp(x[k]);
      EvalResult r = m_->EvalTrafo(trafo.data(), true, 1, /*fatal_on_nan=*/false);
      x_ = x;
      nll_ = r.nll;
      sigma2_ = r.sigma2;
      grad_ = r.grad;
      has_ = true;
    }
    if (calc_grad) grad = grad_;
    return nll_;
  }
  void SetLag1ProfiledOutVariables() override { sigma2_lag1_ = sigma2_; }
  void ResetProfiledOutVariablesToLag1() override { sigma2_ = sigma2_lag1_; }
  void SetNumIter(int it) override { m_->SetNumIter(it); }
  double sigma2() const { return sigma2_; }

 private:
  GroupedModel* m_;
  std::vector<double> x_, grad_;
  double nll_ = 0., sigma2_ = 1., sigma2_lag1_ = 1.;
  bool has_ = false;
};

class GroupedInternalAdapter : public InternalObjective {
 public:
  explicit GroupedInternalAdapter(GroupedModel* m) : m_(m) {}
  double Nll(const std::vector<double>& t) override { return m_->EvalTrafo(t.data(), false, 0, false).nll; }
  std::vector<double> Grad(const std::vector<double>& t, bool profile, double* sigma2) override {
    EvalResult r = m_->EvalTrafo(t.data(), true, profile ? 1 : 0, false);
    if (sigma2) *sigma2 = r.sigma2;
    return r.grad;
  }
  std::vector<double> FisherTrafo(const std::vector<double>& t) override { return m_->FisherTrafo(t.data()); }

 private:
  GroupedModel* m_;
};

}  // namespace

std::vector<double> GroupedModel::FisherTrafo(const double* trafo) {
  // CalcFisherInformation_Only_Grouped_REs_Woodbury with transf_scale = true (re_model_template.h:9579-9586,
  // 9638-9647): FI_00 = n / 2, FI_0j = tau_j tr(Z_j^T Psi^-1 Z_j) / 2 = (m_j - t_j) / 2,
  // FI_jk = tau_j tau_k ||Z_j^T Psi^-1 Z_k||^2 / 2 = (F_jk + delta_jk (m_j - 2 t_j)) / 2 (grouped.h)
  UseDevice();
  const int K = re_->K(), P = 1 + K;
  std::vector<double> F, tr;
  re_->FisherParts(trafo + 1, F, tr);
  std::vector<double> FI((size_t)P * P, 0.);
  FI[0] = n_ / 2.;
  for (int j = 0; j < K; ++j) {
    const double mj = re_->levels_per_effect()[j];
    FI[j + 1] = FI[(size_t)(j + 1) * P] = (mj - tr[j]) / 2.;
    for (int k = 0; k < K; ++k)
      FI[(size_t)(j + 1) * P + k + 1] = (F[(size_t)j * K + k] + (j == k ? mj - 2. * tr[j] : 0.)) / 2.;
  }
  return FI;
}

void GroupedModel::OptimCovPar(const double* y, const double* fixed_effects) {
  UseDevice();
  if (y == nullptr && y_raw_.empty()) Fatal("response variable y has not been set");
  SetResponseAndOffset(y != nullptr ? y : y_raw_.data(), fixed_effects);
  const int P = num_cov_pars();
  num_iter_ = 0;   // re_model_template.h:974
  std::vector<double> trafo(P);
  if (cov_pars_initialized_) ToTrafo(cov_pars_orig_.data(), trafo.data());
  else FindInitCovPar(y_.data(), trafo.data());
  std::vector<double> start_orig(P);
  ToOrig(trafo.data(), trafo[0], start_orig.data());
  if (!cov_pars_initialized_) init_used_ = start_orig;
  if (optim_.max_iterations <= 0) {
    num_it_ = 0;
    cov_pars_orig_ = start_orig;
    cov_pars_initialized_ = true;
    last_cov_pars_ = cov_pars_orig_;
    return;
  }
  if (isettings_.optimizer == "nelder_mead") {   // OptimExternal "nelder_mead" with the nugget profiled out
    if (iterative())
      Fatal("optimizer_cov = 'nelder_mead' is supported by gpboost_amd for grouped random effects with "
            "matrix_inversion_method = 'cholesky' only (use 'lbfgs')");
    const double tol_obj = isettings_.crit_params ? 1e-20 : isettings_.delta;
    const double tol_sol = isettings_.crit_params ? isettings_.delta : 1e-20;
    std::vector<double> x(P - 1);
    for (int k = 0; k < P - 1; ++k) x[k] = std::log(trafo[1 + k]);
    double s2 = 1., fx = 0.;
    auto fn = [&](const std::vector<double>& v) {
      std::vector<double> t(P, 1.);
      for (int k = 0; k < P - 1; ++k) t[1 + k] = std::exp(v[k]);
      EvalResult r = EvalTrafo(t.data(), false, 1, /*fatal_on_nan=*/false);
      s2 = r.sigma2;
      return r.nll;
    };
    num_it_ = nelder_mead(fn, x, isettings_.max_iter, tol_obj, tol_sol, &fx);
    fn(x);   // the profiled sigma^2 at the solution (optim_utils.h:683-686)
    for (int k = 0; k < P - 1; ++k) trafo[1 + k] = std::exp(x[k]);
    cov_pars_orig_.assign(P, 0.);
    ToOrig(trafo.data(), s2, cov_pars_orig_.data());
    cov_pars_initialized_ = true;
    last_nll_ = fx;
    last_cov_pars_ = cov_pars_orig_;
    return;
  }
  if (!isettings_.optimizer.empty()) {   // "gradient_descent" / "fisher_scoring" (re_model_template.h:1287-1549)
    if (isettings_.optimizer == "fisher_scoring" && (has_gp() || iterative()))
      Fatal("optimizer_cov = 'fisher_scoring' is supported by gpboost_amd for grouped random effects with "
            "matrix_inversion_method = 'cholesky' only (use 'lbfgs')");
    GroupedInternalAdapter obj(this);
    double fx = 0.;
    num_it_ = internal_optimize(obj, trafo, isettings_, &fx);
    cov_pars_orig_.assign(P, 0.);
    ToOrig(trafo.data(), trafo[0], cov_pars_orig_.data());
    cov_pars_initialized_ = true;
    last_nll_ = fx;
    last_cov_pars_ = cov_pars_orig_;
    return;
  }
  std::vector<double> x(P - 1);   // log of the transformed parameters, sigma^2 profiled out
  for (int k = 0; k < P - 1; ++k) x[k] = std::log(trafo[1 + k]);
  double fx = 0.;
  GroupedProfiledObjective obj(this);
  num_it_ = lbfgs_minimize(obj, x, fx, optim_);
  for (double v : x)
    if (std::isnan(v) || std::isinf(v))
      Fatal("NaN or Inf occurred in covariance parameter optimization using 'lbfgs' (the reference's nelder_mead "
            "restart is not supported by gpboost_amd)");
  for (int k = 0; k < P - 1; ++k) trafo[1 + k] = std::exp(x[k]);
  cov_pars_orig_.assign(P, 0.);
  ToOrig(trafo.data(), obj.sigma2(), cov_pars_orig_.data());
  cov_pars_initialized_ = true;
  last_nll_ = fx;
  last_cov_pars_ = cov_pars_orig_;
}

std::vector<double> GroupedModel::Blup(const double* cov_pars, const double* y, const double* fixed_effects,
                                       std::vector<double>* var) {
  UseDevice();
  const int K = re_->K();
  std::vector<double> cp;
  if (cov_pars != nullptr) cp.assign(cov_pars, cov_pars + 1 + K);
  else if (!last_cov_pars_.empty()) cp = last_cov_pars_;
  else Fatal("Covariance parameters have not been estimated or correctly set ");
  for (double v : cp)
    if (!(v > 0.)) Fatal("covariance parameters must be > 0");
  if (y != nullptr || fixed_effects != nullptr) SetResponseAndOffset(y, fixed_effects);
  if (!y_set_) Fatal("Response variable data is not provided and has not been set before");
  std::vector<double> tau(K);
  for (int k = 0; k < K; ++k) tau[k] = cp[1 + k] / cp[0];
  std::vector<double> b(re_->M());
  if (var) var->assign(re_->M(), 0.);
  re_->Blup(tau.data(), iterative(), num_iter_ > 0, iter, b.data(), var ? var->data() : nullptr);
  if (var)
    for (double& v : *var) v *= cp[0];   // transformed -> original scale (cov_pars[0] x ..., :4095)
  return b;
}

void GroupedModel::PredictTrainingDataRandomEffects(const double* cov_pars, const double* y, double* out,
                                                    const double* fixed_effects, bool calc_var) {
  const int K = re_->K();
  if (has_gp())
    Fatal("PredictTrainingDataRandomEffects() for GP + grouped random effects models is not supported by "
          "gpboost_amd (call predict())");
  if (calc_var && iterative())
    Fatal("PredictTrainingDataRandomEffects() is currently not implemented for matrix_inversion_method_ == '%s' and "
          "likelihood == 'Gaussian'. Call the predict() function instead.", mim_.c_str());
  std::vector<double> var;
  const std::vector<double> b = Blup(cov_pars, y, fixed_effects, calc_var ? &var : nullptr);
  const std::vector<int>& cum_m = re_->levels_per_effect();
  int off = 0;
  for (int k = 0; k < K; ++k) {
    for (int i = 0; i < n_; ++i) {
      out[(size_t)k * n_ + i] = b[off + levels_[k][i]];
      if (calc_var) out[(size_t)K * n_ + (size_t)k * n_ + i] = var[off + levels_[k][i]];
    }
    off += cum_m[k];
  }
}

void GroupedModel::Predict(const double* y, int n_pred, const char* re_group_data_pred, const double* gp_coords_pred,
                           const double* cov_pars, bool predict_cov_mat, bool predict_var, bool predict_response,
                           const double* fixed_effects, const double* fixed_effects_pred, double* out) {
  if (has_gp()) {
    PredictCombined(y, n_pred, re_group_data_pred, gp_coords_pred, cov_pars, predict_cov_mat, predict_var,
                    predict_response, fixed_effects, fixed_effects_pred, out);
    return;
  }
  if (gp_coords_pred != nullptr) Fatal("gp_coords_pred given for a model without a Gaussian process");
  if ((predict_cov_mat || predict_var) && iterative())
    Fatal("predictive (co)variances for grouped random effects with matrix_inversion_method = 'iterative' (the "
          "reference's simulation-based estimate) are not supported by gpboost_amd (use 'cholesky')");
  if (n_pred <= 0) Fatal("num_data_pred must be > 0");
  if (re_group_data_pred == nullptr) Fatal("re_group_data_pred must be provided for grouped random effects");
  const int K = re_->K();
  if ((int)label_index_.size() != K) Fatal("the model has no label index (created without re_group_data)");
  const bool want_unc = predict_cov_mat || predict_var;
  if (predict_cov_mat && n_pred > 40000)
    Fatal("predictive covariance matrices are limited to 40000 prediction points by gpboost_amd");
  const std::vector<double> b = Blup(cov_pars, y, fixed_effects, nullptr);
  // labels column-major, as re_group_data (re_model_template.h:3081-3085): seen levels to their global
  // index, new labels to -1; fresh[k][i] numbers the distinct new labels (the same-new-label covariance terms
  // compare these ids, not the strings)
  std::vector<int> idx((size_t)n_pred * K, -1);
  std::vector<std::vector<int>> fresh(want_unc ? K : 0);
  std::vector<double> mu(n_pred, 0.);
  const char* p = re_group_data_pred;
  int off = 0;
  for (int k = 0; k < K; ++k) {
    std::unordered_map<std::string, int> fresh_ids;
    if (want_unc) fresh[k].assign(n_pred, -1);
    for (int i = 0; i < n_pred; ++i) {
      std::string label(p);
      p += label.size() + 1;
      auto it = label_index_[k].find(label);
      if (it != label_index_[k].end()) {
        mu[i] += b[off + it->second];   // a new level contributes 0
        idx[(size_t)i * K + k] = off + it->second;
      } else if (want_unc) {
        fresh[k][i] = fresh_ids.emplace(std::move(label), (int)fresh_ids.size()).first->second;
      }
    }
    off += re_->levels_per_effect()[k];
  }
  for (int i = 0; i < n_pred; ++i) out[i] = mu[i] + (fixed_effects_pred ? fixed_effects_pred[i] : 0.);
  if (!want_unc) return;
  std::vector<double> cp;
  if (cov_pars != nullptr) cp.assign(cov_pars, cov_pars + 1 + K);
  else cp = last_cov_pars_;
  std::vector<double> tau(K);
  for (int k = 0; k < K; ++k) tau[k] = cp[1 + k] / cp[0];
  const double nug = predict_response ? 1. : 0., s2 = cp[0];
  double* o = out + n_pred;
  re_->PredCov(n_pred, idx, predict_cov_mat, o);
  if (predict_cov_mat) {
    for (int q = 0; q < n_pred; ++q)
      for (int i = 0; i < n_pred; ++i) {
        double v = o[(size_t)q * n_pred + i] + (i == q ? nug : 0.);
        for (int k = 0; k < K; ++k)
          if (fresh[k][i] >= 0 && fresh[k][i] == fresh[k][q]) v += tau[k];
        o[(size_t)q * n_pred + i] = v * s2;
      }
  } else {
    for (int i = 0; i < n_pred; ++i) {
      double v = o[i] + nug;
      for (int k = 0; k < K; ++k)
        if (idx[(size_t)i * K + k] < 0) v += tau[k];
      o[i] = v * s2;
    }
  }
}


std::vector<int> GroupedModel::PredLevels(int n_pred, const char* re_group_data_pred,
                                          std::vector<std::vector<std::string>>* labels) const {
  const int K = re_->K();
  std::vector<int> lev((size_t)K * n_pred, -1);
  if (labels) labels->assign(K, std::vector<std::string>(n_pred));
  const char* p = re_group_data_pred;
  for (int k = 0; k < K; ++k) {
    std::unordered_map<std::string, int> fresh;
    for (int i = 0; i < n_pred; ++i) {
      std::string label(p);
      p += label.size() + 1;
      auto it = label_index_[k].find(label);
      if (it != label_index_[k].end()) {
        lev[(size_t)k * n_pred + i] = it->second;
      } else {
        auto f = fresh.emplace(label, (int)fresh.size()).first;
        lev[(size_t)k * n_pred + i] = -1 - f->second;
      }
      if (labels) (*labels)[k][i] = std::move(label);
    }
  }
  return lev;
}

void GroupedModel::PredictCombined(const double* y, int n_pred, const char* re_group_data_pred,
                                   const double* gp_coords_pred, const double* cov_pars, bool predict_cov_mat,
                                   bool predict_var, bool predict_response, const double* fixed_effects,
                                   const double* fixed_effects_pred, double* out) {
  // CalcPred, !use_woodbury_identity_ branch (re_model_template.h:10165-10244, 10265-10266, 10361-10365,
  // 10526-10534): cross-covariance = grouped indicators + GP cross-covariance, mean = cross_cov Psi^-1 y,
  // cov = Sigma_pp - cross_cov Psi^-1 cross_cov^T, times sigma^2, plus the nugget for responses
  if (n_pred <= 0) Fatal("num_data_pred must be > 0");
  if (re_group_data_pred == nullptr || gp_coords_pred == nullptr)
    Fatal("predictions of GP + grouped random effects models need both group_data_pred and gp_coords_pred");
  if (predict_cov_mat && n_pred > 40000)
    Fatal("predictive covariance matrices are limited to 40000 prediction points by gpboost_amd");
  UseDevice();
  const int K = re_->K(), P = num_cov_pars();
  std::vector<double> cp;
  if (cov_pars != nullptr) cp.assign(cov_pars, cov_pars + P);
  else if (!last_cov_pars_.empty()) cp = last_cov_pars_;
  else Fatal("Covariance parameters have not been estimated or correctly set ");
  for (double v : cp)
    if (!(v > 0.)) Fatal("covariance parameters must be > 0");
  if (y != nullptr || fixed_effects != nullptr) SetResponseAndOffset(y, fixed_effects);
  if (!y_set_) Fatal("Response variable data is not provided and has not been set before");
  std::vector<double> trafo(P);
  ToTrafo(cp.data(), trafo.data());
  const std::vector<int> plev = PredLevels(n_pred, re_group_data_pred, nullptr);
  DevBuf<int> d_plev(plev.size());
  HIP_CHECK(hipMemcpyAsync(d_plev.get(), plev.data(), sizeof(int) * plev.size(), hipMemcpyHostToDevice, stream_));
  std::vector<double> xp((size_t)n_pred * gp_d_);
  for (int i = 0; i < n_pred; ++i)
    for (int q = 0; q < gp_d_; ++q) xp[(size_t)i * gp_d_ + q] = gp_coords_pred[(size_t)q * n_pred + i];
  dense_->SetGrouped(K, d_lev_.get(), trafo.data() + 1);
  dense_->SetGroupedPred(n_pred, d_plev.get());
  std::vector<double> mean(n_pred), var(predict_var && !predict_cov_mat ? n_pred : 0),
      cov(predict_cov_mat ? (size_t)n_pred * n_pred : 0);
  dense_->Predict(cov_type_, trafo[1 + K], trafo[2 + K], d_y_.get(), xp.data(), n_pred,
                  predict_var && !predict_cov_mat, predict_cov_mat, mean.data(), var.data(), cov.data());
  dense_->SetGroupedPred(0, nullptr);
  const double nug = predict_response ? 1. : 0., s2 = cp[0];
  for (int i = 0; i < n_pred; ++i) out[i] = mean[i] + (fixed_effects_pred ? fixed_effects_pred[i] : 0.);
  if (predict_cov_mat) {
    for (int q = 0; q < n_pred; ++q)
      for (int i = 0; i < n_pred; ++i)
        out[n_pred + (size_t)q * n_pred + i] = (cov[(size_t)q * n_pred + i] + (i == q ? nug : 0.)) * s2;
  } else if (predict_var) {
    for (int i = 0; i < n_pred; ++i) out[n_pred + i] = (var[i] + nug) * s2;
  }
}

void GroupedModel::StdDevCovPars(const double* cov_pars, double* sd) {
  if (has_gp())
    Fatal("standard deviations of covariance parameters for GP + grouped random effects models are not "
          "supported by gpboost_amd");
  if (iterative())
    Fatal("standard deviations of covariance parameters for grouped random effects with matrix_inversion_method = "
          "'iterative' (the reference's stochastic estimate) are not supported by gpboost_amd (use 'cholesky')");
  UseDevice();
  const int K = re_->K(), P = 1 + K;
  for (int k = 0; k < P; ++k)
    if (!(cov_pars[k] > 0.)) Fatal("covariance parameters must be > 0");
  std::vector<double> tau(K), FI((size_t)P * P);
  for (int k = 0; k < K; ++k) tau[k] = cov_pars[1 + k] / cov_pars[0];
  re_->Fisher(tau.data(), cov_pars[0], FI.data());
  // FI.inverse() (re_model_template.h:9788): Gauss-Jordan with partial pivoting on the small P x P matrix
  std::vector<double> inv((size_t)P * P, 0.);
  for (int i = 0; i < P; ++i) inv[(size_t)i * P + i] = 1.;
  for (int c = 0; c < P; ++c) {
    int piv = c;
    for (int r = c + 1; r < P; ++r)
      if (std::fabs(FI[(size_t)r * P + c]) > std::fabs(FI[(size_t)piv * P + c])) piv = r;
    if (!(FI[(size_t)piv * P + c] != 0.) || !std::isfinite(FI[(size_t)piv * P + c]))
      Fatal("the Fisher information is singular");
    for (int j = 0; j < P; ++j) {
      std::swap(FI[(size_t)c * P + j], FI[(size_t)piv * P + j]);
      std::swap(inv[(size_t)c * P + j], inv[(size_t)piv * P + j]);
    }
    const double d = FI[(size_t)c * P + c];
    for (int j = 0; j < P; ++j) {
      FI[(size_t)c * P + j] /= d;
      inv[(size_t)c * P + j] /= d;
    }
    for (int r = 0; r < P; ++r) {
      if (r == c) continue;
      const double f = FI[(size_t)r * P + c];
      for (int j = 0; j < P; ++j) {
        FI[(size_t)r * P + j] -= f * FI[(size_t)c * P + j];
        inv[(size_t)r * P + j] -= f * inv[(size_t)c * P + j];
      }
    }
  }
  for (int k = 0; k < P; ++k) sd[k] = std::sqrt(inv[(size_t)k * P + k]);
}

}  // namespace gpb_amd
