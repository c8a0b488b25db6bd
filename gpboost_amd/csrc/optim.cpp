// GPB_OptimCovPar: L-BFGS covariance-parameter estimation over the device likelihood.
// See optim.h for the reference functions this restates.
#include "optim.h"

#include <algorithm>
#include <cmath>
#include <limits>
#include <numeric>
#include <random>

#include "cov.h"
#include "covariates.h"
#include "re_model.h"

namespace gpb_amd {

namespace {

double dot(const std::vector<double>& a, const std::vector<double>& b) {
  double s = 0.;
  for (size_t i = 0; i < a.size(); ++i) s += a[i] * b[i];
  return s;
}

double norm2(const std::vector<double>& a) { return std::sqrt(dot(a, a)); }

// LineSearchBacktracking::LineSearch with the Armijo rule and GPBoost's changes
// (LineSearchBacktracking.h:45-143): shrink by 1/2, or by 1/32 after a large increase;
// after max_linesearch trials fall back to xp (step 0).
void backtracking(LbfgsObjective& f, const LbfgsSettings& s, const std::vector<double>& xp,
                  const std::vector<double>& drt, double& step, double& fx, std::vector<double>& grad,
                  std::vector<double>& x) {
  if (step <= 0.) Fatal("GPModel lbfgs: 'step' must be positive");
  const double fx_init = fx;
  const double dg_init = dot(grad, drt);
  if (dg_init > 0) Fatal("GPModel lbfgs: the moving direction increases the objective function value");
  const double test_decr = s.ftol * dg_init;
  int iter = 0;
  for (; iter < s.max_linesearch; ++iter) {
    for (size_t i = 0; i < x.size(); ++i) x[i] = xp[i] + step * drt[i];
    fx = f.Eval(x, grad, true, false, iter == 0);
    if (fx > fx_init + step * test_decr || fx != fx) {
      const double width = (fx - fx_init) > 2. * std::max(std::fabs(fx_init), 1.) ? 0.5 / 16. : 0.5;
      step *= width;
    } else {
      break;   // Armijo condition met
    }
  }
  if (iter >= s.max_linesearch) {
    x = xp;
    f.ResetProfiledOutVariablesToLag1();
    fx = fx_init;
    step = 0.;
  }
}

}  // namespace

void InverseHessian::Reset(int dim, int m) {
  // BFGSMat::reset (BFGSMat.h:89-105): no corrections, theta = 1
  dim_ = dim;
  m_ = m;
  s_.assign(m, std::vector<double>(dim));
  y_.assign(m, std::vector<double>(dim));
  ys_.assign(m, 0.);
  alpha_.assign(m, 0.);
  theta_ = 1.;
  count_ = 0;
  ptr_ = 0;
}

void InverseHessian::Add(const std::vector<double>& s, const std::vector<double>& y) {
  const int loc = ptr_ % m_;
  s_[loc] = s;
  y_[loc] = y;
  ys_[loc] = dot(s, y);
  theta_ = dot(y, y) / ys_[loc];
  if (count_ < m_) ++count_;
  ptr_ = loc + 1;
}

void InverseHessian::Apply(const std::vector<double>& v, double a, std::vector<double>& out) {
  out.resize(v.size());
  for (size_t i = 0; i < v.size(); ++i) out[i] = a * v[i];
  int j = ptr_ % m_;
  for (int k = 0; k < count_; ++k) {   // newest to oldest
    j = (j + m_ - 1) % m_;
    alpha_[j] = dot(s_[j], out) / ys_[j];
    for (size_t i = 0; i < out.size(); ++i) out[i] -= alpha_[j] * y_[j][i];
  }
  for (double& o : out) o /= theta_;
  for (int k = 0; k < count_; ++k) {   // oldest to newest
    const double beta = dot(y_[j], out) / ys_[j];
    for (size_t i = 0; i < out.size(); ++i) out[i] += (alpha_[j] - beta) * s_[j][i];
    j = (j + 1) % m_;
  }
}

int lbfgs_minimize(LbfgsObjective& f, std::vector<double>& x, double& fx, const LbfgsSettings& s, InverseHessian* given,
                   bool reuse) {
  // LBFGS.h:86-301 (past = 1, epsilon = epsilon_rel = 1e-20, no neighbour re-determination).
  // given: the caller's m_bfgs (REModelTemplate::GetMBFGS): with reuse it seeds the first direction
  // -H g at step 1 (when it holds corrections of this dimension, LBFGS.h:158-171); it receives the
  // final approximation on convergence (LBFGS.h:262, 299).
  const int n = (int)x.size();
  InverseHessian H(n, s.m);
  std::vector<double> grad(n), xp(n), gradp(n), drt(n), vs(n), vy(n);
  fx = f.Eval(x, grad, true, true, true);
  if (std::isnan(fx) || std::isinf(fx))
    Fatal("%s occurred in initial negative log-likelihood. Possible solutions: try other initial values ('init_cov_pars')",
          std::isnan(fx) ? "NaN" : "Inf");
  const double eps_grad = 1e-20;
  double gnorm = norm2(grad);
  double fx_lag = fx;
  if (gnorm <= eps_grad || gnorm <= eps_grad * norm2(x)) return 1;
  double step;
  if (reuse && given != nullptr && given->count() > 0 && given->dim() == n) {
    H = *given;
    step = 1.;
    H.Apply(grad, -1., drt);
  } else {
    for (int i = 0; i < n; ++i) drt[i] = -grad[i];
    step = s.initial_step_factor / norm2(drt);
  }
  const double eps = std::numeric_limits<double>::epsilon();
  for (int k = 1;; ++k) {
    xp = x;
    gradp = grad;
    // GetMaximalLearningRate (optim_utils.h:497-534 -> MaximalLearningRateCovAuxPars,
    // re_model_template.h:4937-4945): no parameter changes by more than a factor of 100 per step
    double max_abs = 0.;
    for (int i = 0; i < n; ++i) max_abs = std::max(max_abs, std::fabs(drt[i]));
    const double max_lr = s.max_log_change / max_abs;
    if (max_lr < step) step = max_lr;
    backtracking(f, s, xp, drt, step, fx, grad, x);
    f.Eval(x, grad, false, true, false);   // gradient at the accepted point
    gnorm = norm2(grad);
    bool converged = gnorm <= eps_grad || gnorm <= eps_grad * norm2(x);
    if ((fx_lag - fx) <= s.delta * std::max(std::fabs(fx_lag), 1.)) converged = true;
    if (s.max_iterations != 0 && k >= s.max_iterations) converged = true;
    f.SetNumIter(k - 1);
    f.SetLag1ProfiledOutVariables();
    if (converged) {
      if (given != nullptr) *given = H;
      return k;
    }
    for (int i = 0; i < n; ++i) {
      vs[i] = x[i] - xp[i];
      vy[i] = grad[i] - gradp[i];
    }
    if (dot(vs, vy) > eps * dot(vy, vy)) H.Add(vs, vy);
    step = 1.;
    H.Apply(grad, -1., drt);
    fx_lag = fx;
  }
}

bool is_internal_optimizer(const std::string& name) { return name == "gradient_descent" || name == "fisher_scoring"; }

int internal_optimize(InternalObjective& f, std::vector<double>& pars, const InternalSettings& s, double* nll_out,
                      InternalCoefHook* coef) {
  const bool gd = s.optimizer == "gradient_descent";
  if (!gd && s.optimizer != "fisher_scoring") Fatal("internal optimizer '%s' is not supported", s.optimizer.c_str());
  const bool profile = gd;                  // profile_out_error_variance_ (re_model_template.h:946-948)
  const bool nest = gd && s.nesterov;       // Nesterov acceleration for gradient descent only (:960-965)
  if (nest && s.schedule != 0 && s.schedule != 1)
    Fatal("NesterovSchedule: version = %d is not supported ", s.schedule);
  if (nest && s.schedule == 1) Fatal("Armijo condition backtracking is not implemented when nesterov_schedule_version = 1 ");
  const double kMaxLogUpdate = std::log(100.);   // MAX_GRADIENT_UPDATE_LOG_SCALE_ (:5287-5289)
  const double kCArmijo = 1e-4, kCArmijoMom = 1e-4;   // C_ARMIJO_DEFAULT_, C_ARMIJO_MOM_DEFAULT_ (:5317-5319)
  const int kMaxShrink = 30;                     // MAX_NUMBER_LR_SHRINKAGE_STEPS_DEFAULT_ (:5255)
  const int P = (int)pars.size();
  double lr_cov = s.lr < 0. ? (gd ? 0.1 : 1.) : s.lr;   // SetInitialValueLRCov (:7505-7521)
  auto schedule = [&](int it, double acc) { return it < s.momentum_offset ? 0. : acc; };   // NesterovSchedule v0
  double nll = f.Nll(pars);   // initial objective (:1233-1262)
  if (!std::isfinite(nll))
    Fatal("%s occurred in initial negative log-likelihood. Possible solutions: try other initial values ('init_cov_pars')",
          std::isnan(nll) ? "NaN" : "Inf");
  std::vector<double> after_grad = pars, after_grad_lag1 = pars;
  int num_it = s.max_iter;
  for (int it = 0; it < s.max_iter; ++it) {
    const double nll_lag1 = nll;
    const std::vector<double> pars_lag1 = pars;
    // neg_log_likelihood_after_lin_coef_update_ (:1327-1330, 1356)
    const double base = coef != nullptr ? coef->Update(pars) : nll_lag1;
    std::vector<double> grad, step;
    if (gd) {
      double s2 = 0.;
      grad = f.Grad(pars, true, &s2);   // ProfileOutSigma2 then CalcGradPars without the nugget (:1363-1372)
      pars[0] = s2;
      step = grad;
      double mx = 0.;   // AvoidTooLargeLearningRatesCovAuxPars (:7539-7560, MaximalLearningRateCovAuxPars :4937-4945)
      for (double v : step) mx = std::max(mx, std::fabs(v));
      const double max_lr = kMaxLogUpdate / mx;
      if (lr_cov > max_lr) lr_cov = max_lr;
    } else {
      grad = f.Grad(pars, false, nullptr);   // with the nugget (:1378-1384)
      std::vector<double> F = f.FisherTrafo(pars);
      // approx_Hessian.llt().solve(grad)
      std::vector<double> L(F.size(), 0.);
      for (int j = 0; j < P; ++j) {
        double d = F[(size_t)j * P + j];
        for (int k = 0; k < j; ++k) d -= L[(size_t)j * P + k] * L[(size_t)j * P + k];
        if (!(d > 0.)) Fatal("the Fisher information is not positive definite in Fisher scoring");
        L[(size_t)j * P + j] = std::sqrt(d);
        for (int i = j + 1; i < P; ++i) {
          double v = F[(size_t)i * P + j];
          for (int k = 0; k < j; ++k) v -= L[(size_t)i * P + k] * L[(size_t)j * P + k];
          L[(size_t)i * P + j] = v / L[(size_t)j * P + j];
        }
      }
      step = grad;
      for (int i = 0; i < P; ++i) {
        for (int k = 0; k < i; ++k) step[i] -= L[(size_t)i * P + k] * step[k];
        step[i] /= L[(size_t)i * P + i];
      }
      for (int i = P - 1; i >= 0; --i) {
        for (int k = i + 1; k < P; ++k) step[i] -= L[(size_t)k * P + i] * step[k];
        step[i] /= L[(size_t)i * P + i];
      }
    }
    // CalcDirDerivArmijoAndLearningRateConstChangeCovAuxPars (armijo_condition_ = true)
    const int ng = (int)step.size();
    double dir_deriv = 0.;
    for (int i = 0; i < ng; ++i) dir_deriv -= grad[i] * step[i];
    double mom_dir_deriv = 0.;
    if (nest) {
      for (int i = 0; i < ng; ++i) {
        const int p = profile ? i + 1 : i;
        mom_dir_deriv += grad[i] * (std::log(pars[p]) - std::log(after_grad[p]));
      }
    }
    // UpdateCovAuxPars: step on the log scale, momentum, Armijo backtracking
    double lr = lr_cov, acc = s.acc_rate;
    bool found = false, halving = false;
    std::vector<double> np(P);
    for (int ih = 0; ih < kMaxShrink; ++ih) {
      std::vector<double> upd(ng);
      for (int i = 0; i < ng; ++i) {
        upd[i] = lr * step[i];
        if (!gd) upd[i] = std::min(std::max(upd[i], -kMaxLogUpdate), kMaxLogUpdate);
      }
      if (profile) {
        np[0] = pars[0];
        for (int i = 0; i < ng; ++i) np[i + 1] = std::exp(std::log(pars[i + 1]) - upd[i]);
      } else {
        for (int i = 0; i < P; ++i) np[i] = std::exp(std::log(pars[i]) - upd[i]);
      }
      if (nest) {   // ApplyMomentumStep(exclude_first_log_scale = profile)
        after_grad = np;
        const double mu = schedule(it, acc);
        for (int i = profile ? 1 : 0; i < P; ++i)
          np[i] = std::exp((mu + 1.) * std::log(after_grad[i]) - mu * std::log(after_grad_lag1[i]));
        if (profile) np[0] = after_grad[0];
      }
      nll = f.Nll(np);
      const double mu = nest ? schedule(it, acc) : 0.;
      if (nll <= base + kCArmijo * lr * dir_deriv + kCArmijoMom * mu * mom_dir_deriv) {
        found = true;
        break;
      }
      halving = true;
      lr *= 0.5;    // LR_SHRINKAGE_FACTOR_
      acc *= 0.5;
    }
    (void)found;
    if (halving && gd) lr_cov = lr;   // permanently decreased for gradient descent (:7978-7979)
    if (nest) after_grad_lag1 = after_grad;
    pars = np;
    bool bad = !std::isfinite(nll);
    for (double v : pars) bad = bad || !std::isfinite(v);
    if (bad)
      Fatal("NaN or Inf occurred in covariance parameter optimization using '%s' (the reference's nelder_mead restart "
            "is not supported by gpboost_amd)", s.optimizer.c_str());
    bool conv;
    if (s.crit_params) {
      double dn = 0., ln = 0.;
      for (int i = 0; i < P; ++i) {
        dn += (pars[i] - pars_lag1[i]) * (pars[i] - pars_lag1[i]);
        ln += pars_lag1[i] * pars_lag1[i];
      }
      // with covariates: both the coefficients and the covariance parameters (strict <, :1712-1716)
      conv = coef != nullptr ? coef->CoefConverged(s.delta) && std::sqrt(dn) < s.delta * std::sqrt(ln)
                             : std::sqrt(dn) <= s.delta * std::sqrt(ln);
    } else {
      conv = (nll_lag1 - nll) <= s.delta * std::max(std::fabs(nll_lag1), 1.);
    }
    if (conv) {
      num_it = it + 1;
      break;
    }
  }
  *nll_out = nll;
  return num_it;
}

int nelder_mead(const std::function<double(const std::vector<double>&)>& f, std::vector<double>& x0, int iter_max,
                double tol_obj, double tol_sol, double* fval) {
  const int nv = (int)x0.size();
  const double alpha = 1., beta = 0.75 - 1. / (2. * nv), gamma = 1. + 2. / nv, delta = 1. - 1. / nv;   // adaptive_pars
  std::vector<std::vector<double>> P(nv + 1, x0);
  std::vector<double> F(nv + 1);
  F[0] = f(x0);
  for (int i = 1; i <= nv; ++i) {
    const double xi = x0[i - 1];
    P[i][i - 1] = xi + (xi != 0. ? 0.05 * xi : 0.00025);
    F[i] = f(P[i]);
  }
  auto max_abs = [](double v, double acc) { return std::max(acc, std::fabs(v)); };
  std::vector<std::vector<double>> Pold = P;
  std::vector<double> Fold = F;
  int iter = 0;
  bool converged = false;
  while (!converged) {
    ++iter;
    bool next = false;
    // step 1: sort the vertices by value (get_sort_index: std::sort of the indices)
    std::vector<int> idx(nv + 1);
    std::iota(idx.begin(), idx.end(), 0);
    std::sort(idx.begin(), idx.end(), [&](int a, int b) { return F[a] < F[b]; });
    {
      std::vector<std::vector<double>> P2(nv + 1);
      std::vector<double> F2(nv + 1);
      for (int i = 0; i <= nv; ++i) { P2[i] = P[idx[i]]; F2[i] = F[idx[i]]; }
      P.swap(P2);
      F.swap(F2);
    }
    // step 2: centroid of the best nv vertices, reflection
    std::vector<double> c(nv, 0.);
    for (int j = 0; j < nv; ++j) {
      double sacc = 0.;
      for (int i = 0; i < nv; ++i) sacc += P[i][j];
      c[j] = sacc / (double)nv;
    }
    auto along = [&](double t, const std::vector<double>& dir_end) {   // c + t (dir_end - c)
      std::vector<double> out(nv);
      for (int j = 0; j < nv; ++j) out[j] = c[j] + t * (dir_end[j] - c[j]);
      return out;
    };
    std::vector<double> xr(nv);
    for (int j = 0; j < nv; ++j) xr[j] = c[j] + alpha * (c[j] - P[nv][j]);
    const double fr = f(xr);
    if (fr >= F[0] && fr < F[nv - 1]) {
      P[nv] = xr;
      F[nv] = fr;
      next = true;
    }
    // step 3: expansion
    if (!next && fr < F[0]) {
      std::vector<double> xe = along(gamma, xr);
      const double fe = f(xe);
      if (fe < fr) { P[nv] = xe; F[nv] = fe; }
      else { P[nv] = xr; F[nv] = fr; }
      next = true;
    }
    // steps 4, 5: contractions
    if (!next && fr >= F[nv - 1]) {
      if (fr < F[nv]) {
        std::vector<double> xoc = along(beta, xr);
        const double foc = f(xoc);
        if (foc <= fr) { P[nv] = xoc; F[nv] = foc; next = true; }
      } else {
        std::vector<double> xic = along(beta, P[nv]);
        const double fic = f(xic);
        if (fic < F[nv]) { P[nv] = xic; F[nv] = fic; next = true; }
      }
    }
    // step 6: shrink toward the best vertex
    if (!next) {
      for (int i = 1; i <= nv; ++i)
        for (int j = 0; j < nv; ++j) P[i][j] = P[0][j] + delta * (P[i][j] - P[0][j]);
      for (int i = 1; i <= nv; ++i) F[i] = f(P[i]);
    }
    // convergence (nm.hpp:303-311): changes against the previous iteration's (unsorted) arrays
    double dF = 0., mF = 0.;
    for (int i = 0; i <= nv; ++i) { dF = max_abs(F[i] - Fold[i], dF); mF = max_abs(Fold[i], mF); }
    const double rel_obj = dF / (1.0e-08 + mF);
    Fold = F;
    double rel_sol = 2. * std::fabs(tol_sol);
    if (tol_sol >= 0.) {
      double dP = 0., mP = 0.;
      for (int i = 0; i <= nv; ++i)
        for (int j = 0; j < nv; ++j) { dP = max_abs(P[i][j] - Pold[i][j], dP); mP = max_abs(Pold[i][j], mP); }
      rel_sol = dP / (1.0e-08 + mP);
      Pold = P;
    }
    converged = !(rel_obj > tol_obj && rel_sol > tol_sol && iter < iter_max);
  }
  int best = 0;   // index_min
  for (int i = 1; i <= nv; ++i)
    if (F[i] < F[best]) best = i;
  x0 = P[best];
  *fval = f(x0);
  return iter;
}

// ---------------------------------------------------------------------------------------------
// REModelAMD: initial values and the optimization driver

namespace {

// utils.h:189-202 CalculateMedianPartiallySortInput
double median_partial_sort(std::vector<double>& v) {
  const int num = (int)v.size();
  const int pos = num / 2;
  std::nth_element(v.begin(), v.begin() + pos, v.end());
  double med = v[pos];
  if (num % 2 == 0) {
    std::nth_element(v.begin(), v.begin() + pos - 1, v.end());
    med = (med + v[pos - 1]) / 2.;
  }
  return med;
}

constexpr double kEpsilonNumbers = 1e-10;   // EPSILON_NUMBERS (utils.h)

}  // namespace

double REModelAMD::InitialRangeTrafo() const {
  // cov_fcts.h:1275-1450 FindInitCovPar: median distance among (at most 1000 sampled) points;
  // correlation 0.05 at half the median distance. The sample draws continue the model's
  // mt19937(seed) after the Vecchia ordering shuffle (re_model_template.h:154,
  // Vecchia_utils.cpp:1094-1095).
  // the GP component's coordinates: all points, or the unique locations of a latent model with
  // repeated coordinates (RECompGP::coords_, re_comp.h:1232-1244)
  // FITC: the inducing points' component (re_comps_ip_, re_model_template.h:4474-4476), the draws
  // continuing the generator after the inducing-point selection; full_scale_vecchia: the Vecchia component
  // (all points in the model order, :4452-4456) with the generator after the shuffle and the selection
  const std::vector<double>& X = fitc_ ? fitc_->inducing_points() : coords_vo_;
  std::mt19937 rng(cfg_.seed);
  if ((int)(X.size() / cfg_.d) > 1000) {
    if (fitc_ || vif_) rng = fitc_rng_;   // full_scale_vecchia: after the shuffle and the inducing points
    if (vecchia_ && cfg_.vecchia_ordering == "random") {   // the ordering shuffle of the n observations
      std::vector<int> dummy(cfg_.n);
      std::iota(dummy.begin(), dummy.end(), 0);
      std::shuffle(dummy.begin(), dummy.end(), rng);
    }
  }
  return init_range_trafo(X, cfg_.d, cfg_.cov_type, rng);
}

double init_range_trafo(const std::vector<double>& X, int d, int cov_type, std::mt19937& rng) {
  const int n = (int)(X.size() / d);
  const int kMaxPoints = 1000;
  const int nf = std::min(n, kMaxPoints);
  std::vector<int> idx(nf);
  if (nf < n) {
    std::uniform_int_distribution<> dis(0, n - 1);
    for (int i = 0; i < nf; ++i) idx[i] = dis(rng);
  } else {
    std::iota(idx.begin(), idx.end(), 0);
  }
  std::vector<double> dist((size_t)nf * (nf - 1) / 2);
  size_t p = 0;
  for (int i = 0; i < nf - 1; ++i)
    for (int j = i + 1; j < nf; ++j) {
      double s = 0.;
      for (int q = 0; q < d; ++q) {
        const double t = X[(size_t)idx[i] * d + q] - X[(size_t)idx[j] * d + q];
        s += t * t;
      }
      dist[p++] = std::sqrt(s);
    }
  if (dist.empty()) Fatal("Cannot find an initial value for the range parameter with a single data point");
  double med = median_partial_sort(dist);
  if (med < kEpsilonNumbers) med = std::accumulate(dist.begin(), dist.end(), 0.) / (double)dist.size();
  if (med < kEpsilonNumbers)
    Fatal("Cannot find an initial value for the range parameter since both the median and the average distances among coordinates are zero %s",
          nf < n ? "on a random sub-sample of size 1000 " : "");
  switch (cov_type) {
    case kMatern05: return 2. * 3. / med;
    case kMatern15: return 2. * 4.7 / med;
    case kMatern25: return 2. * 5.9 / med;
    default: return 3. / std::pow(med / 2., 2.);
  }
}

void REModelAMD::FindInitCovPar(const double* y, double* trafo) const {
  // re_model_template.h:4388-4504 for one GP component
  const int n = cfg_.n;
  double var = 0.;
  const bool gauss_data = !cfg_.latent || cfg_.lik == kLikGaussian;
  if (gauss_data) {
    double mean = 0.;
    for (int i = 0; i < n; ++i) mean += y[i];
    mean /= n;
    for (int i = 0; i < n; ++i) var += (y[i] - mean) * (y[i] - mean);
    var /= (n - 1);
  }
  if (!cfg_.latent) {
    trafo[0] = var / 2.;   // nugget
    trafo[1] = 1.;         // marginal variance / nugget
    trafo[2] = InitialRangeTrafo();
  } else {
    // init_marg_var: var / 2 for the gaussian latent likelihood, 0.1 with nelder_mead, else 1 (re_model_template.h:4444-4451)
    trafo[0] = cfg_.lik == kLikGaussian ? var / 2. : (isettings_.optimizer == "nelder_mead" ? 0.1 : 1.);
    trafo[1] = InitialRangeTrafo();
  }
}

void REModelAMD::InitCovParsIfNotDefined(const double* y, const double* fixed_effects) {
  // REModel::InitializeCovParsIfNotDefined (re_model.cpp:1142-1164): init_cov_pars when given (set by
  // SetOptimSettings), else FindInitCovPar on y - F (latent models: the stored response)
  if (cov_pars_initialized_) return;
  const int n = cfg_.n;
  std::vector<double> yv;
  if (cfg_.latent) {
    if (y != nullptr) yv.assign(y, y + n);
    else if (!y_raw_.empty()) yv = y_raw_;
    else Fatal("Response variable data has not been set");
  } else {
    if (y == nullptr) Fatal("initial covariance parameters need the response variable y");
    yv.assign(y, y + n);
    if (fixed_effects != nullptr)
      for (int i = 0; i < n; ++i) yv[i] -= fixed_effects[i];
  }
  double trafo[3];
  FindInitCovPar(yv.data(), trafo);
  if (cfg_.latent) cov_pars_orig_ = {trafo[0], range_back(cfg_.cov_type, trafo[1])};
  else cov_pars_orig_ = {trafo[0], trafo[1] * trafo[0], range_back(cfg_.cov_type, trafo[2])};
  init_used_ = cov_pars_orig_;
  cov_pars_initialized_ = true;
}

void REModelAMD::SetOptimSettings(const double* init_cov_pars, double lr, int max_iter, double delta_rel_conv,
                                  const char* optimizer, int m_lbfgs) {
  // re_model.cpp:264-279 and re_model_template.h:710-823
  if (optimizer != nullptr && optimizer[0] != '\0') {
    const std::string o(optimizer);
    if (o != "lbfgs" && o != "nelder_mead" && !is_internal_optimizer(o))
      Fatal("Optimizer option '%s' is not supported for covariance parameters by gpboost_amd (supported: lbfgs, "
            "gradient_descent, fisher_scoring, nelder_mead)", o.c_str());
    isettings_.optimizer = o == "lbfgs" ? "" : o;
  }
  isettings_.lr = lr;
  isettings_.max_iter = max_iter;
  // SetInitialValueDeltaRelConv (re_model_template.h:7524-7533): 1e-8 for nelder_mead, else 1e-6
  isettings_.delta = delta_rel_conv < 0. ? (isettings_.optimizer == "nelder_mead" ? 1e-8 : 1e-6) : delta_rel_conv;
  if (init_cov_pars != nullptr) {
    init_cov_pars_.assign(init_cov_pars, init_cov_pars + num_cov_pars());
    for (double v : init_cov_pars_)
      if (!(v > 0.)) Fatal("init_cov_pars must be > 0");
    cov_pars_orig_ = init_cov_pars_;
    cov_pars_initialized_ = true;
  }
  optim_.initial_step_factor = lr < 0. ? 1. : lr;               // SetInitialValueLRCov :7505-7521
  optim_.max_iterations = max_iter;
  optim_.delta = delta_rel_conv < 0. ? 1e-6 : delta_rel_conv;   // SetInitialValueDeltaRelConv :7524-7533
  if (m_lbfgs > 0) optim_.m = m_lbfgs;
}

namespace {

// EvalLLforLBFGSpp for the Gaussian likelihood with the nugget profiled out
// (optim_utils.h:269-313, 333-348): x = log(sigma1^2 / sigma^2, phi). With estimate_cov_par_index (idx, original
// order [nugget, sigma1^2, range]): fixed parameters get a zero gradient (CalcGradPars skips them,
// re_model_template.h:1773-1816); a fixed nugget is not profiled (ProfileOutSigma2 :2407-2412), a fixed marginal
// variance stays constant on the original scale through the last profiled sigma^2 (MaybeKeepVarianceConstant
// :7104-7121: tau = sigma1^2_init / sigma^2).
class GaussianProfiledObjective : public LbfgsObjective {
 public:
  GaussianProfiledObjective(REModelAMD* m, std::vector<int> idx = {}, double sigma2_init = 1., double var_init = 1.)
      : m_(m), idx_(std::move(idx)), sigma2_(sigma2_init), sigma2_lag1_(sigma2_init), var_orig_(var_init) {}
  double Eval(const std::vector<double>& x, std::vector<double>& grad, bool eval_ll, bool calc_grad,
              bool hint_grad) override {
    if (eval_ll || !(has_grad_ && x == x_)) {
      const bool fix_nug = !idx_.empty() && idx_[0] <= 0;
      const bool fix_var = !idx_.empty() && idx_[1] <= 0;
      double trafo[3] = {fix_nug ? sigma2_ : 1., std::exp(x[0]), std::exp(x[1])};
      if (fix_var && !fix_nug) trafo[1] = var_orig_ / sigma2_;
      EvalResult r = m_->EvalTrafo(trafo, calc_grad || hint_grad, fix_nug ? 0 : 1);
      x_ = x;
      nll_ = r.nll;
      if (!fix_nug) sigma2_ = r.sigma2;
      has_grad_ = calc_grad || hint_grad;
      if (has_grad_) {
        grad_ = r.grad;
        if (fix_nug) grad_.erase(grad_.begin());   // include_error_var = false
        if (!idx_.empty())
          for (int k = 0; k < 2; ++k)
            if (idx_[k + 1] <= 0) grad_[k] = 0.;
      }
    }
    if (calc_grad) grad = grad_;
    return nll_;
  }
  // sigma1^2 / sigma^2 actually used at x (the fixed-variance form rescales it)
  double tau_at(const std::vector<double>& x) const {
    const bool fix_nug = !idx_.empty() && idx_[0] <= 0;
    if (!idx_.empty() && idx_[1] <= 0 && !fix_nug) return var_orig_ / sigma2_;
    return std::exp(x[0]);
  }
  void SetLag1ProfiledOutVariables() override { sigma2_lag1_ = sigma2_; }
  void ResetProfiledOutVariablesToLag1() override { sigma2_ = sigma2_lag1_; }
  double sigma2() const { return sigma2_; }

 private:
  REModelAMD* m_;
  std::vector<int> idx_;
  std::vector<double> x_, grad_;
  double nll_ = 0., sigma2_ = 1., sigma2_lag1_ = 1., var_orig_ = 1.;
  bool has_grad_ = false;
};

// EvalLLforLBFGSpp for the Gaussian likelihood with covariates, optimizer_coef "wls": the
// coefficients are profiled out by GLS at every likelihood evaluation (optim_utils.h:297-313,
// ProfileOutCoef re_model_template.h:2427-2445), then the nugget (:303-312); x as above.
class GaussianWlsObjective : public LbfgsObjective {
 public:
  GaussianWlsObjective(REModelAMD* m) : m_(m) {}
  double Eval(const std::vector<double>& x, std::vector<double>& grad, bool eval_ll, bool calc_grad,
              bool hint_grad) override {
    if (eval_ll || !(has_grad_ && x == x_)) {
      const double trafo[3] = {1., std::exp(x[0]), std::exp(x[1])};
      EvalResult r = m_->EvalTrafoWls(trafo, calc_grad || hint_grad, /*fatal_on_nan=*/false, &beta_);
      x_ = x;
      nll_ = r.nll;
      sigma2_ = r.sigma2;
      has_grad_ = calc_grad || hint_grad;
      if (has_grad_) grad_ = r.grad;
    }
    if (calc_grad) grad = grad_;
    return nll_;
  }
  void SetLag1ProfiledOutVariables() override { sigma2_lag1_ = sigma2_; beta_lag1_ = beta_; }
  void ResetProfiledOutVariablesToLag1() override { sigma2_ = sigma2_lag1_; beta_ = beta_lag1_; }
  double sigma2() const { return sigma2_; }
  const std::vector<double>& beta() const { return beta_; }

 private:
  REModelAMD* m_;
  std::vector<double> x_, grad_, beta_, beta_lag1_;
  double nll_ = 0., sigma2_ = 1., sigma2_lag1_ = 1.;
  bool has_grad_ = false;
};

// EvalLLforLBFGSpp for the latent (Laplace) models: x = log(sigma1^2, phi[, aux]).
class LatentObjective : public LbfgsObjective {
 public:
  // idx: estimate_cov_par_index (empty: all estimated); fixed parameters get a zero gradient (:1773-1816)
  LatentObjective(REModelAMD* m, bool with_aux, std::vector<int> idx = {})
      : m_(m), with_aux_(with_aux), idx_(std::move(idx)) {}
  double Eval(const std::vector<double>& x, std::vector<double>& grad, bool eval_ll, bool calc_grad,
              bool hint_grad) override {
    if (eval_ll || !(has_grad_ && x == x_)) {
      const double trafo[2] = {std::exp(x[0]), std::exp(x[1])};
      if (with_aux_) {
        const double aux = std::exp(x[2]);
        m_->SetAuxPars(&aux);
      }
      // the L-BFGS objective continues from the previous evaluation's mode (mode_initialized_,
      // likelihoods.h:2782-2789); a gradient-only call at the point just evaluated uses that
      // evaluation's mode as it stands (eval_likelihood = false, optim_utils.h:314-330)
      const bool grad_only = !eval_ll && has_x_ && x == x_;
      EvalResult r = m_->EvalLatentTrafo(trafo, calc_grad || hint_grad, /*fatal_on_nan=*/false,
                                         grad_only ? LatentVecchia::ModeStart::kKeep : LatentVecchia::ModeStart::kWarm);
      has_x_ = true;
      bool bad = !std::isfinite(r.nll);
      for (double g : r.grad) bad = bad || !std::isfinite(g);
      if (bad) m_->ResetLatentModeToPrevious();   // EvalLLforLBFGSpp, optim_utils.h:349-360
      x_ = x;
      nll_ = r.nll;
      has_grad_ = calc_grad || hint_grad;
      if (has_grad_) {
        grad_ = r.grad;
        for (size_t k = 0; k < idx_.size() && k < grad_.size(); ++k)
          if (idx_[k] <= 0) grad_[k] = 0.;
      }
    }
    if (calc_grad) grad = grad_;
    return nll_;
  }

 private:
  REModelAMD* m_;
  bool with_aux_;
  std::vector<int> idx_;
  std::vector<double> x_, grad_;
  double nll_ = 0.;
  bool has_grad_ = false, has_x_ = false;
};

// The reference's internal optimizers on the exact Gaussian likelihood (internal_optimize).
class InternalAdapter : public InternalObjective {
 public:
  explicit InternalAdapter(REModelAMD* m) : m_(m) {}
  double Nll(const std::vector<double>& t) override { return m_->EvalTrafo(t.data(), false, 0, false).nll; }
  std::vector<double> Grad(const std::vector<double>& t, bool profile, double* sigma2) override {
    EvalResult r = m_->EvalTrafo(t.data(), true, profile ? 1 : 0, false);
    if (sigma2) *sigma2 = r.sigma2;
    return r.grad;
  }
  std::vector<double> FisherTrafo(const std::vector<double>& t) override { return m_->FisherTrafo(t.data()); }

 private:
  REModelAMD* m_;
};

// optimizer_coef "wls" inside the internal optimizers: GLS at the current parameters, the residual response
// y - F - X beta for the covariance step
class WlsCoefHook : public InternalCoefHook {
 public:
  WlsCoefHook(REModelAMD* m, const std::vector<double>& y, const std::vector<double>& F, const std::vector<double>& X,
              int p, std::vector<double> beta0)
      : m_(m), y_(y), F_(F), X_(X), p_(p), beta_(std::move(beta0)) {
    SetResidual();
  }
  double Update(const std::vector<double>& trafo) override {
    beta_lag1_ = beta_;
    std::vector<double> b;
    const double nll = m_->EvalTrafoWls(trafo.data(), false, /*fatal_on_nan=*/false, &b).nll;   // ProfileOutCoef (:2427-2445)
    if (std::isnan(nll) || (int)b.size() != p_)   // a non-finite Gram matrix leaves no coefficients: stop cleanly
      Fatal("NaN or Inf occurred in the generalized least squares coefficients of the covariance parameter step");
    beta_ = b;
    SetResidual();
    return m_->EvalTrafo(trafo.data(), false, 0, false).nll;   // EvalNegLogLikelihoodOnlyUpdateFixedEffects
  }
  bool CoefConverged(double delta) const override {
    double dn = 0., ln = 0.;
    for (int k = 0; k < p_; ++k) {
      dn += (beta_[k] - beta_lag1_[k]) * (beta_[k] - beta_lag1_[k]);
      ln += beta_lag1_[k] * beta_lag1_[k];
    }
    return std::sqrt(dn) <= delta * std::sqrt(ln);
  }
  const std::vector<double>& beta() const { return beta_; }

 private:
  void SetResidual() {
    const int n = (int)y_.size();
    std::vector<double> off(n);
    for (int i = 0; i < n; ++i) {
      double v = F_.empty() ? 0. : F_[i];
      for (int k = 0; k < p_; ++k) v += X_[(size_t)k * n + i] * beta_[k];
      off[i] = v;
    }
    m_->SetResponseAndOffset(y_.data(), off.data());
  }
  REModelAMD* m_;
  const std::vector<double>& y_;
  const std::vector<double>& F_;
  const std::vector<double>& X_;
  int p_;
  std::vector<double> beta_, beta_lag1_;
};

}  // namespace

std::vector<double> REModelAMD::FisherTrafo(const double* trafo) {
  // CalcFisherInformation(transf_scale = true, include_error_var = true), dense branch (re_model_template.h:
  // 9203-9209, 9219-9227): FI_00 = n / 2, FI_0k = tr(Psi^-1 dPsi_k) / 2, FI_kl = tr(Psi^-1 dPsi_k Psi^-1 dPsi_l) / 2
  // with dPsi / dlog v = v corr, dPsi / dlog phi = v dcorr / dlog phi
  if (!dense_) Fatal("the transformed-scale Fisher information is available for gp_approx = 'none' only");
  const double v = trafo[1], phi = trafo[2];
  double sums[6], kms[2], t[6];
  dense_->Eval(cfg_.cov_type, v, phi, d_y_.get(), true, sums, kms);   // tr(dPsi_k Psi^-1) = sums[4], sums[5]
  dense_->Fisher(cfg_.cov_type, v, phi, v, t);
  const double n = cfg_.n;
  return {n / 2., sums[4] / 2., sums[5] / 2.,
          sums[4] / 2., 0.5 * v * v * t[3], 0.5 * v * t[4],
          sums[5] / 2., 0.5 * v * t[4], 0.5 * t[5]};
}

void REModelAMD::OptimCovPar(const double* y, const double* fixed_effects, bool called_in_boosting, bool reuse_lr) {
  // REModel::OptimCovPar (re_model.cpp:339-401) -> OptimLinRegrCoefCovPar without covariates
  // (re_model_template.h:846-1700) -> OptimExternal "lbfgs" (optim_utils.h:561-706)
  UseDevice();
  const int n = cfg_.n;
  if (reuse_lr && !called_in_boosting)
    Fatal("reuse_learning_rates_from_previous_call requires called_in_GPBoost_algorithm");   // :1026-1028
  // reuse_m_bfgs_from_previous_call (re_model_template.h:880-881)
  const bool reuse_m_bfgs = reuse_lr && called_in_boosting && cov_est_once_ && cov_est_last_call_;
  if (y == nullptr) {   // the stored response (re_model_template.h:1188-1191, GetY)
    if (y_raw_.empty()) Fatal("response variable y has not been set");
    y = y_raw_.data();
  }
  for (int i = 0; i < n; ++i)
    if (std::isnan(y[i]) || std::isinf(y[i])) Fatal("NaN or Inf in response variable / label ");
  std::vector<double> yraw(y, y + n);   // y may alias y_raw_
  SetResponseAndOffset(yraw.data(), fixed_effects);   // Gaussian: y - F; latent: location mode + F
  if (fixed_effects != nullptr && !called_in_boosting) {   // saved for prediction (re_model_template.h:1051-1054)
    fixed_effects_.assign(fixed_effects, fixed_effects + n);
    has_fixed_effects_ = true;
  }
  std::vector<double> yv(yraw);
  if (fixed_effects != nullptr)
    for (int i = 0; i < n; ++i) yv[i] -= fixed_effects[i];
  has_covariates_ = false;   // REModel::OptimCovPar (re_model.cpp:396)
  num_covariates_ = 0;
  X_cov_.clear();
  coef_.clear();
  InitializeOptimizerNames();
  EnsureStructure();
  const bool with_aux = cfg_.latent && estimate_aux_pars && !aux_pars_.empty();
  // initial values on the transformed scale (InitializeCovParsIfNotDefined re_model.cpp:1142-1164)
  double trafo[3];
  if (cov_pars_initialized_) {
    if (cfg_.latent) { trafo[0] = cov_pars_orig_[0]; trafo[1] = range_trafo_of(cov_pars_orig_[1]); }
    else TransformCovPars(cov_pars_orig_.data(), trafo);
  } else {
    if (yv.empty()) Fatal("initial covariance parameters need the response variable y");
    FindInitCovPar(yv.data(), trafo);
  }
  if (with_aux && !aux_pars_set_) {
    if (yv.empty()) Fatal("initial auxiliary parameters need the response variable y");
    if (cfg_.lik == kLikGamma) {
      // likelihoods.h:1116-1145 (FindInitialAuxPars, gamma): approximate MLE of the shape ignoring the random
      // effects, s = log(mean y e^-F) - mean(log y - F), k = (3 - s + sqrt((s - 3)^2 + 24 s)) / (12 s)
      double log_avg = 0., avg_log = 0.;
      for (int i = 0; i < n; ++i) {
        const double f = fixed_effects != nullptr ? fixed_effects[i] : 0.;
        log_avg += fixed_effects != nullptr ? yraw[i] / std::exp(f) : yraw[i];
        avg_log += fixed_effects != nullptr ? std::log(yraw[i]) - f : std::log(yraw[i]);
      }
      log_avg = std::log(log_avg / n);
      avg_log /= n;
      const double sv = log_avg - avg_log;
      aux_pars_[0] = (3. - sv + std::sqrt((sv - 3.) * (sv - 3.) + 24. * sv)) / (12. * sv);
    } else {
      // likelihoods.h:1087-1116, 1223-1225 (FindInitialAuxPars, gaussian): sample variance / 2
      double avg = 0., sum_sq = 0.;
      for (int i = 0; i < n; ++i) { avg += yv[i]; sum_sq += yv[i] * yv[i]; }
      avg /= n;
      const double sample_var = std::max((sum_sq - n * avg * avg) / (n - 1), 1e-6);
      aux_pars_[0] = sample_var / 2.;
    }
    aux_pars_set_ = true;   // SetAuxPars marks them set (likelihoods.h:1809): a refit continues from here
  }
  std::vector<double> start_orig;
  if (cfg_.latent) start_orig = {trafo[0], range_back(cfg_.cov_type, trafo[1])};
  else start_orig = {trafo[0], trafo[1] * trafo[0], range_back(cfg_.cov_type, trafo[2])};
  if (!cov_pars_initialized_) init_used_ = start_orig;   // FindInitCovPar's values (re_model.cpp:1159-1160)
  if (optim_.max_iterations <= 0) {   // max_iter_ = 0 (re_model_template.h:1223): the parameters stay at their initial values
    num_it_ = 0;
    cov_pars_orig_ = start_orig;
    cov_pars_initialized_ = true;
    last_cov_pars_ = cov_pars_orig_;
    return;
  }
  if (!reuse_m_bfgs) m_bfgs_ = InverseHessian();   // a fresh solver state (LBFGS.h:42-48)
  std::vector<double> x;
  double fx = 0.;
  if (!est_idx_.empty() && !isettings_.optimizer.empty() && !(cfg_.latent && isettings_.optimizer == "gradient_descent"))
    Fatal("estimate_cov_par_index (fixing covariance parameters) is supported by gpboost_amd with optimizer_cov = "
          "'lbfgs' only");
  if (isettings_.optimizer == "nelder_mead") {   // OptimExternal "nelder_mead" (optim_utils.h:642-643, 680-700)
    const double tol_obj = isettings_.crit_params ? 1e-20 : isettings_.delta;
    const double tol_sol = isettings_.crit_params ? isettings_.delta : 1e-20;
    double s2 = 1.;
    if (!cfg_.latent) {   // EvalLLforOptimLib with the nugget profiled out: x = log(sigma1^2 / sigma^2, phi)
      x = {std::log(trafo[1]), std::log(trafo[2])};
      auto fn = [&](const std::vector<double>& v) {
        const double t[3] = {1., std::exp(v[0]), std::exp(v[1])};
        EvalResult r = EvalTrafo(t, false, 1, /*fatal_on_nan=*/false);
        s2 = r.sigma2;
        return r.nll;
      };
      num_it_ = nelder_mead(fn, x, isettings_.max_iter, tol_obj, tol_sol, &fx);
      fn(x);   // OptimExternal re-evaluates at the solution for the profiled sigma^2 (:683-686)
      cov_pars_orig_ = {s2, std::exp(x[0]) * s2, range_back(cfg_.cov_type, std::exp(x[1]))};
    } else {   // x = log(sigma1^2, phi[, aux]); the Laplace mode continues from the previous evaluation
      x = {std::log(trafo[0]), std::log(trafo[1])};
      if (with_aux) x.push_back(std::log(aux_pars_[0]));
      auto fn = [&](const std::vector<double>& v) {
        const double t[2] = {std::exp(v[0]), std::exp(v[1])};
        if (with_aux) {
          const double aux = std::exp(v[2]);
          SetAuxPars(&aux);
        }
        EvalResult r = EvalLatentTrafo(t, false, /*fatal_on_nan=*/false, LatentVecchia::ModeStart::kWarm);
        if (!std::isfinite(r.nll)) ResetLatentModeToPrevious();   // EvalLLforOptimLib, optim_utils.h:196-199
        return r.nll;
      };
      num_it_ = nelder_mead(fn, x, isettings_.max_iter, tol_obj, tol_sol, &fx);
      cov_pars_orig_ = {std::exp(x[0]), range_back(cfg_.cov_type, std::exp(x[1]))};
      if (with_aux) aux_pars_[0] = std::exp(x[2]);
    }
  } else if (isettings_.optimizer == "gradient_descent" && cfg_.latent) {
    // Laplace models: OptimLinRegrCoefCovPar's loop without profiling (re_model_template.h:1290-1549), the
    // covariance parameters and the auxiliary parameters on the log scale with their own learning rates
    // (lr_cov_, lr_aux_pars_; AvoidTooLargeLearningRatesCovAuxPars :7539-7560), separate Armijo conditions for
    // both blocks (UpdateCovAuxPars :7850-7990), Nesterov momentum over all of them (ApplyMomentumStep), the
    // Laplace mode continued across evaluations and reset to its previous value after a rejected trial.
    const int nc = 2, na = with_aux ? 1 : 0, P = nc + na;
    std::vector<double> pars = {trafo[0], trafo[1]};
    if (with_aux) pars.push_back(aux_pars_[0]);
    const double kMaxLog = std::log(100.);
    double lr_cov = isettings_.lr < 0. ? 0.1 : isettings_.lr, lr_aux = lr_cov;   // SetInitialValueLRCov :7505-7521
    const bool nest = isettings_.nesterov;
    if (nest && isettings_.schedule != 0) Fatal("NesterovSchedule: version = %d is not supported ", isettings_.schedule);
    auto sched = [&](int it, double acc) { return it < isettings_.momentum_offset ? 0. : acc; };
    auto eval_nll = [&](const std::vector<double>& v) {
      const double t[2] = {v[0], v[1]};
      if (with_aux) SetAuxPars(&v[2]);
      EvalResult r = EvalLatentTrafo(t, false, /*fatal_on_nan=*/false, LatentVecchia::ModeStart::kWarm);
      return r.nll;
    };
    double nll = eval_nll(pars);
    if (!std::isfinite(nll)) Fatal("NaN or Inf occurred in initial approximate negative marginal log-likelihood");
    std::vector<double> after = pars, after_lag1 = pars;
    num_it_ = isettings_.max_iter;
    for (int it = 0; it < isettings_.max_iter; ++it) {
      const double nll_lag1 = nll;
      const std::vector<double> pars_lag1 = pars;
      const double t[2] = {pars[0], pars[1]};
      EvalResult gr = EvalLatentTrafo(t, true, false, LatentVecchia::ModeStart::kKeep);   // CalcGradPars at the mode
      std::vector<double> g = gr.grad;
      if ((int)g.size() < P) Fatal("internal error: latent gradient has %d entries", (int)g.size());
      g.resize(P);
      for (size_t k = 0; k < est_idx_.size() && k < (size_t)nc; ++k)
        if (est_idx_[k] <= 0) g[k] = 0.;
      double mc = 0., ma = 0.;
      for (int k = 0; k < nc; ++k) mc = std::max(mc, std::fabs(g[k]));
      for (int k = nc; k < P; ++k) ma = std::max(ma, std::fabs(g[k]));
      if (mc > 0. && lr_cov > kMaxLog / mc) lr_cov = kMaxLog / mc;
      if (na && ma > 0. && lr_aux > kMaxLog / ma) lr_aux = kMaxLog / ma;
      double dd_c = 0., dd_a = 0., md_c = 0., md_a = 0.;
      for (int k = 0; k < nc; ++k) dd_c -= g[k] * g[k];
      for (int k = nc; k < P; ++k) dd_a -= g[k] * g[k];
      if (nest) {
        for (int k = 0; k < nc; ++k) md_c += g[k] * (std::log(pars[k]) - std::log(after[k]));
        for (int k = nc; k < P; ++k) md_a += g[k] * (std::log(pars[k]) - std::log(after[k]));
      }
      double lc = lr_cov, la = lr_aux, acc = isettings_.acc_rate;
      bool halving = false;
      std::vector<double> np(P);
      for (int ih = 0; ih < 30; ++ih) {
        for (int k = 0; k < P; ++k) np[k] = std::exp(std::log(pars[k]) - (k < nc ? lc : la) * g[k]);
        const double mu = nest ? sched(it, acc) : 0.;
        if (nest) {
          after = np;
          for (int k = 0; k < P; ++k) np[k] = std::exp((mu + 1.) * std::log(after[k]) - mu * std::log(after_lag1[k]));
        }
        nll = eval_nll(np);
        bool ok = nll <= nll_lag1 + 1e-4 * lc * dd_c + 1e-4 * mu * md_c;
        if (na) ok = ok && nll <= nll_lag1 + 1e-4 * la * dd_a + 1e-4 * mu * md_a;
        if (ok) break;
        halving = true;
        lc *= 0.5;
        la *= 0.5;
        acc *= 0.5;
        ResetLatentModeToPrevious();
      }
      if (halving) { lr_cov = lc; lr_aux = la; }
      if (nest) after_lag1 = after;
      pars = np;
      bool bad = !std::isfinite(nll);
      for (double v : pars) bad = bad || !std::isfinite(v);
      if (bad) Fatal("NaN or Inf occurred in covariance parameter optimization using 'gradient_descent'");
      bool conv;
      if (isettings_.crit_params) {
        double dn = 0., ln = 0.;
        for (int k = 0; k < P; ++k) { dn += (pars[k] - pars_lag1[k]) * (pars[k] - pars_lag1[k]); ln += pars_lag1[k] * pars_lag1[k]; }
        conv = std::sqrt(dn) <= isettings_.delta * std::sqrt(ln);
      } else {
        conv = (nll_lag1 - nll) <= isettings_.delta * std::max(std::fabs(nll_lag1), 1.);
      }
      if (conv) { num_it_ = it + 1; break; }
    }
    fx = nll;
    x = {std::log(pars[0]), std::log(pars[1])};
    cov_pars_orig_ = {pars[0], range_back(cfg_.cov_type, pars[1])};
    if (with_aux) aux_pars_[0] = pars[2];
  } else if (!isettings_.optimizer.empty()) {   // "gradient_descent" / "fisher_scoring" (re_model_template.h:1287-1549)
    if (cfg_.latent)
      Fatal("optimizer_cov = '%s' is supported by gpboost_amd for the Gaussian likelihood only (use 'lbfgs')",
            isettings_.optimizer.c_str());
    if (isettings_.optimizer == "fisher_scoring" && !dense_)
      Fatal("optimizer_cov = 'fisher_scoring' is supported by gpboost_amd for gp_approx = 'none' only (use 'lbfgs')");
    std::vector<double> tv(trafo, trafo + 3);
    InternalAdapter obj(this);
    num_it_ = internal_optimize(obj, tv, isettings_, &fx);
    cov_pars_orig_ = {tv[0], tv[1] * tv[0], range_back(cfg_.cov_type, tv[2])};
  } else if (!cfg_.latent) {
    x = {std::log(trafo[1]), std::log(trafo[2])};
    GaussianProfiledObjective obj(this, est_idx_, trafo[0], trafo[1] * trafo[0]);
    num_it_ = lbfgs_minimize(obj, x, fx, optim_, &m_bfgs_, reuse_m_bfgs);
    const double s2 = obj.sigma2();
    cov_pars_orig_ = {s2, obj.tau_at(x) * s2, range_back(cfg_.cov_type, std::exp(x[1]))};
  } else {
    x = {std::log(trafo[0]), std::log(trafo[1])};
    if (with_aux) x.push_back(std::log(aux_pars_[0]));
    LatentObjective obj(this, with_aux, est_idx_);
    num_it_ = lbfgs_minimize(obj, x, fx, optim_, &m_bfgs_, reuse_m_bfgs);
    cov_pars_orig_ = {std::exp(x[0]), range_back(cfg_.cov_type, std::exp(x[1]))};
    if (with_aux) aux_pars_[0] = std::exp(x[2]);
  }
  for (double v : x)
    if (std::isnan(v) || std::isinf(v))
      Fatal("NaN or Inf occurred in covariance parameter optimization using 'lbfgs' (the reference's nelder_mead restart is not supported by gpboost_amd)");
  cov_pars_initialized_ = true;
  cov_est_once_ = true;          // re_model_template.h:1614-1616
  cov_est_last_call_ = true;
  last_nll_ = fx;
  last_cov_pars_ = cov_pars_orig_;
}

void REModelAMD::InitializeOptimizerNames() {
  // InitializeOptimSettings (re_model_template.h:7463-7474)
  if (optimizer_cov_.empty()) optimizer_cov_ = "lbfgs";
  if (optimizer_coef_.empty()) optimizer_coef_ = cfg_.latent ? "lbfgs" : "wls";
}

void REModelAMD::OptimLinRegrCoefCovPar(const double* y, const double* X, int p, const double* fixed_effects) {
  if (!est_idx_.empty() && X != nullptr && p > 0)
    Fatal("estimate_cov_par_index (fixing covariance parameters) with linear regression covariates is not supported by "
          "gpboost_amd");
  if (!isettings_.optimizer.empty() && !is_internal_optimizer(isettings_.optimizer) && X != nullptr && p > 0)
    Fatal("optimizer_cov = '%s' with linear regression covariates is not supported by gpboost_amd (use 'lbfgs', "
          "'gradient_descent' or 'fisher_scoring')", isettings_.optimizer.c_str());
  // REModel::OptimLinRegrCoefCovPar (re_model.cpp:403-469) -> REModelTemplate::OptimLinRegrCoefCovPar
  // with covariates (re_model_template.h:846-1700): Gaussian likelihood, optimizer_cov "lbfgs",
  // optimizer_coef "wls" (its default, :7467-7470): OptimExternal with profile_out_coef = true
  UseDevice();
  const int n = cfg_.n;
  if (X == nullptr || p <= 0) {
    OptimCovPar(y, fixed_effects);
    return;
  }
  if (cfg_.latent)
    Fatal("linear regression covariates for likelihood '%s' are not supported by gpboost_amd (Gaussian likelihood "
          "only)", cfg_.likelihood.c_str());
  if (p + 1 > kCovMaxCols) Fatal("at most %d covariates are supported by gpboost_amd (got %d)", kCovMaxCols - 1, p);
  if (y == nullptr) Fatal("response variable y must be provided");   // re_model_template.h:1078
  for (int i = 0; i < n; ++i)
    if (std::isnan(y[i]) || std::isinf(y[i])) Fatal("NaN or Inf in response variable / label ");
  for (size_t i = 0; i < (size_t)n * p; ++i)
    if (std::isnan(X[i]) || std::isinf(X[i])) Fatal("NaN or Inf in covariate data");
  InitializeOptimizerNames();
  if (optimizer_coef_ != "wls")
    Fatal("optimizer_coef '%s' is not supported by gpboost_amd for the Gaussian likelihood (supported: wls)",
          optimizer_coef_.c_str());
  std::vector<double> yraw(y, y + n);
  y_raw_ = yraw;
  if (fixed_effects != nullptr) {
    fixed_effects_.assign(fixed_effects, fixed_effects + n);
    has_fixed_effects_ = true;
  } else {
    has_fixed_effects_ = false;
    fixed_effects_.clear();
  }
  X_cov_.assign(X, X + (size_t)n * p);
  num_covariates_ = p;
  has_covariates_ = true;
  coef_std_dev_valid_ = false;
  EnsureStructure();
  UploadCovariates();
  // initial values: init_cov_pars, the previous estimate, or FindInitCovPar on y - offset
  // (re_model.cpp:407 InitializeCovParsIfNotDefined; re_model_template.h:4388-4435)
  double trafo[3];
  if (cov_pars_initialized_) {
    TransformCovPars(cov_pars_orig_.data(), trafo);
  } else {
    std::vector<double> yv(yraw);
    if (fixed_effects != nullptr)
      for (int i = 0; i < n; ++i) yv[i] -= fixed_effects[i];
    FindInitCovPar(yv.data(), trafo);
  }
  const std::vector<double> start_orig = {trafo[0], trafo[1] * trafo[0], range_back(cfg_.cov_type, trafo[2])};
  if (!cov_pars_initialized_) init_used_ = start_orig;
  if (optim_.max_iterations <= 0) {   // parameters stay; coefficients by GLS at them
    num_it_ = 0;
    cov_pars_orig_ = start_orig;
    cov_pars_initialized_ = true;
    EvalTrafoWls(trafo, false, true, nullptr);
    last_cov_pars_ = cov_pars_orig_;
    return;
  }
  if (is_internal_optimizer(isettings_.optimizer)) {   // gradient descent / Fisher scoring with "wls" coefficients
    if (isettings_.optimizer == "fisher_scoring" && !dense_)
      Fatal("optimizer_cov = 'fisher_scoring' is supported by gpboost_amd for gp_approx = 'none' only (use 'lbfgs')");
    // initial coefficients: OLS of y - F on X (re_model_template.h:1110-1140), then GLS in every iteration
    std::vector<double> yF(yraw);
    if (fixed_effects != nullptr)
      for (int i = 0; i < n; ++i) yF[i] -= fixed_effects[i];
    std::vector<double> XtX((size_t)p * p, 0.), Xty(p, 0.);
    for (int a = 0; a < p; ++a) {
      for (int i = 0; i < n; ++i) Xty[a] += X[(size_t)a * n + i] * yF[i];
      for (int b = 0; b < p; ++b)
        for (int i = 0; i < n; ++i) XtX[(size_t)a * p + b] += X[(size_t)a * n + i] * X[(size_t)b * n + i];
    }
    std::vector<double> b0 = Xty;   // solve by Gaussian elimination (p small)
    {
      std::vector<double> A = XtX;
      for (int c = 0; c < p; ++c) {
        int piv = c;
        for (int r = c + 1; r < p; ++r)
          if (std::fabs(A[(size_t)r * p + c]) > std::fabs(A[(size_t)piv * p + c])) piv = r;
        for (int k = 0; k < p; ++k) std::swap(A[(size_t)c * p + k], A[(size_t)piv * p + k]);
        std::swap(b0[c], b0[piv]);
        for (int r = c + 1; r < p; ++r) {
          const double f = A[(size_t)r * p + c] / A[(size_t)c * p + c];
          for (int k = c; k < p; ++k) A[(size_t)r * p + k] -= f * A[(size_t)c * p + k];
          b0[r] -= f * b0[c];
        }
      }
      for (int c = p - 1; c >= 0; --c) {
        for (int k = c + 1; k < p; ++k) b0[c] -= A[(size_t)c * p + k] * b0[k];
        b0[c] /= A[(size_t)c * p + c];
      }
    }
    std::vector<double> Fv = fixed_effects != nullptr ? std::vector<double>(fixed_effects, fixed_effects + n)
                                                       : std::vector<double>();
    WlsCoefHook hook(this, yraw, Fv, X_cov_, p, b0);
    std::vector<double> tv(trafo, trafo + 3);
    InternalAdapter obj(this);
    double fx = 0.;
    num_it_ = internal_optimize(obj, tv, isettings_, &fx, &hook);
    cov_pars_orig_ = {tv[0], tv[1] * tv[0], range_back(cfg_.cov_type, tv[2])};
    coef_ = hook.beta();
    for (double v : coef_)
      if (std::isnan(v) || std::isinf(v)) Fatal("NaN or Inf occurred in the linear regression coefficients");
    cov_pars_initialized_ = true;
    cov_est_once_ = true;
    cov_est_last_call_ = true;
    last_nll_ = fx;
    last_cov_pars_ = cov_pars_orig_;
    return;
  }
  std::vector<double> x = {std::log(trafo[1]), std::log(trafo[2])};
  double fx = 0.;
  GaussianWlsObjective obj(this);
  m_bfgs_ = InverseHessian();
  num_it_ = lbfgs_minimize(obj, x, fx, optim_, &m_bfgs_, false);
  for (double v : x)
    if (std::isnan(v) || std::isinf(v))
      Fatal("NaN or Inf occurred in covariance parameter optimization using 'lbfgs' (the reference's nelder_mead restart is not supported by gpboost_amd)");
  const double s2 = obj.sigma2();
  cov_pars_orig_ = {s2, std::exp(x[0]) * s2, range_back(cfg_.cov_type, std::exp(x[1]))};
  coef_ = obj.beta();
  for (double v : coef_)
    if (std::isnan(v) || std::isinf(v)) Fatal("NaN or Inf occurred in the linear regression coefficients");
  cov_pars_initialized_ = true;
  cov_est_once_ = true;
  cov_est_last_call_ = true;
  last_nll_ = fx;
  last_cov_pars_ = cov_pars_orig_;
}

void REModelAMD::GetInitCovPar(double* out) const {
  const std::vector<double>& v = !init_cov_pars_.empty() ? init_cov_pars_ : init_used_;
  for (int k = 0; k < num_cov_pars(); ++k) out[k] = v.empty() ? -1. : v[k];
}

void REModelAMD::StdDevCovPars(const double* orig, double* sd) {
  // CalcFisherInformation, dense branch (re_model_template.h:9179-9230), transf_scale = false,
  // include_error_var = true: with Sigma^-1 = Psi^-1 / sigma^2 and dSigma_k on the original scale
  // (sigma^2: I; sigma1^2: the correlation matrix; rho: sigma1^2 dcorr/drho)
  //   FI_00 = tr(Sigma^-2) / 2, FI_0k = tr(Sigma^-2 dSigma_k) / 2, FI_kl = tr(Sigma^-1 dSigma_k Sigma^-1 dSigma_l) / 2
  if (cfg_.latent || vif_)
    Fatal("standard deviations of covariance parameters are supported by gpboost_amd only for gp_approx = 'none', "
          "'vecchia' and 'fitc' with the Gaussian likelihood");
  UseDevice();
  EnsureStructure();
  double trafo[3];
  TransformCovPars(orig, trafo);
  double F[3][3];
  if (vecchia_) {
    // CalcFisherInformation_Vecchia, stochastic-trace form (re_model_template.h:9246-9298); probes from
    // (seed_rand_vec_trace, cg_generator_counter_ = 0: a Cholesky-based Gaussian model never draws)
    if (world_ > 1) Fatal("standard deviations of covariance parameters are only available on single-rank models");
    if (!vfisher_)
      vfisher_.reset(new VecchiaFisher(cfg_.n, cfg_.d, cfg_.num_neighbors, d_X_.get(), d_nbr_.get(), nbr_, stream_));
    vfisher_->Fisher(cfg_.cov_type, orig, trafo, iter.num_rand_vec_trace, iter.seed_rand_vec_trace, 0, &F[0][0]);
  } else if (fitc_) {
    // CalcFisherInformation_FITC_FSA (re_model_template.h:9363-9548), the same probes
    fitc_->Fisher(cfg_.cov_type, orig, trafo, iter.num_rand_vec_trace, iter.seed_rand_vec_trace, 0, &F[0][0]);
  } else {
    const double s2 = orig[0], rho = orig[2];
    const double dlogphi_drho = (cfg_.cov_type == kGaussian ? -2. : -1.) / rho;
    double t[6];
    dense_->Fisher(cfg_.cov_type, trafo[1], trafo[2], orig[1] * dlogphi_drho, t);
    const double c = 0.5 / (s2 * s2);
    const double Fd[3][3] = {{c * t[0], c * t[1], c * t[2]}, {c * t[1], c * t[3], c * t[4]},
                             {c * t[2], c * t[4], c * t[5]}};
    std::copy(&Fd[0][0], &Fd[0][0] + 9, &F[0][0]);
  }
  // inverse of the symmetric 3 x 3 matrix by cofactors (FI.inverse(), :9788)
  const double c00 = F[1][1] * F[2][2] - F[1][2] * F[2][1];
  const double c11 = F[0][0] * F[2][2] - F[0][2] * F[2][0];
  const double c22 = F[0][0] * F[1][1] - F[0][1] * F[1][0];
  const double det = F[0][0] * c00 - F[0][1] * (F[1][0] * F[2][2] - F[1][2] * F[2][0]) +
                     F[0][2] * (F[1][0] * F[2][1] - F[1][1] * F[2][0]);
  if (!(det != 0.) || !std::isfinite(det)) Fatal("the Fisher information is singular");
  sd[0] = std::sqrt(c00 / det);
  sd[1] = std::sqrt(c11 / det);
  sd[2] = std::sqrt(c22 / det);
}

}  // namespace gpb_amd
