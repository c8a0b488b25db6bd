// Covariance-parameter estimation (GPB_OptimCovPar) on top of the device likelihood.
//
// The reference's default optimizer for covariance parameters is "lbfgs"
// (re_model_template.h:7463-7466): L-BFGS on the log of the transformed parameters with an
// Armijo backtracking line search, run by its vendored and modified LBFGSpp
// (external_libs/LBFGSpp/include/LBFGS.h:86-301, LineSearchBacktracking.h:45-143,
// BFGSMat.h:89-186) through the objective EvalLLforLBFGSpp (optim_utils.h:243-364) and the
// driver OptimExternal (optim_utils.h:561-706). This is a restatement of that algorithm in plain
// C++ (host side, O(P) work per iteration for P <= 3 parameters); every objective value and
// gradient comes from the device evaluation of REModelAMD.
#pragma once

#include <functional>
#include <string>
#include <vector>

namespace gpb_amd {

// LBFGSParam values set by OptimExternal (optim_utils.h:654-662) and the LBFGSpp defaults it
// keeps (Param.h:182-190: ftol = 1e-4).
struct LbfgsSettings {
  int m = 6;                       // m_lbfgs_ (re_model_template.h:5355)
  int max_iterations = 1000;       // max_iter_ (:5200)
  double delta = 1e-6;             // delta_rel_conv_ (SetInitialValueDeltaRelConv :7524-7533), past = 1
  double initial_step_factor = 1.; // lr_cov_init_ (SetInitialValueLRCov :7505-7521)
  int max_linesearch = 20;
  double ftol = 1e-4;
  double max_log_change = 4.605170185988092;   // log(MAX_REL_CHANGE_GRADIENT_UPDATE_ = 100) (:5287-5289)
};

// Objective in the optimizer's coordinates x (log of the transformed parameters).
class LbfgsObjective {
 public:
  virtual ~LbfgsObjective() = default;
  // EvalLLforLBFGSpp::operator()(pars, gradient, eval_likelihood, calc_gradient). hint_grad: the
  // caller expects to ask for the gradient at this x next (lets a device evaluation compute both).
  virtual double Eval(const std::vector<double>& x, std::vector<double>& grad, bool eval_ll, bool calc_grad,
                      bool hint_grad) = 0;
  virtual void SetLag1ProfiledOutVariables() {}     // optim_utils.h (EvalLLforLBFGSpp) / LBFGS.h:232
  virtual void ResetProfiledOutVariablesToLag1() {} // LineSearchBacktracking.h:133
  virtual void SetNumIter(int) {}                   // LBFGS.h:231 (f.SetNumIter(k - 1))
};

// Limited-memory inverse-Hessian approximation: a ring of the last m (s, y) pairs and the
// two-loop recursion (Nocedal & Wright Alg. 7.4), as BFGSMat.h:89-105 / 160-186 keeps it.
class InverseHessian {
 public:
  InverseHessian() = default;
  InverseHessian(int dim, int m) { Reset(dim, m); }
  void Reset(int dim, int m);
  void Add(const std::vector<double>& s, const std::vector<double>& y);
  void Apply(const std::vector<double>& v, double a, std::vector<double>& out);   // out = a H v
  int count() const { return count_; }   // BFGSMat::get_m_ncorr
  int dim() const { return dim_; }       // BFGSMat::get_dim_param

 private:
  int dim_ = 0, m_ = 1;
  std::vector<std::vector<double>> s_, y_;
  std::vector<double> ys_, alpha_;
  double theta_ = 1.;
  int count_ = 0;
  int ptr_ = 0;   // ptr_ % m_ is the next slot (BFGSMat reset sets m_ptr = m, i.e. slot 0)
};

// LBFGSSolver::minimize with LineSearchBacktracking (Armijo) as GPBoost runs it: returns the
// number of iterations; x is overwritten with the minimiser and fx with its objective value.
// given / reuse: the m_bfgs kept across calls (reuse_m_bfgs_from_previous_call, LBFGS.h:86-171).
int lbfgs_minimize(LbfgsObjective& f, std::vector<double>& x, double& fx, const LbfgsSettings& s,
                   InverseHessian* given = nullptr, bool reuse = false);

// ---- the reference's internal optimizers for covariance parameters (Gaussian likelihood, no covariates):
// "gradient_descent" (with Nesterov acceleration by default) and "fisher_scoring" (OptimLinRegrCoefCovPar's
// loop re_model_template.h:1290-1549 with AvoidTooLargeLearningRatesCovAuxPars :7539-7560,
// CalcDirDerivArmijoAndLearningRateConstChangeCovAuxPars :7587-7634, UpdateCovAuxPars :7850-8000,
// ApplyMomentumStep :4600-4623, NesterovSchedule :5643-5662, CheckOptimizerHasConverged :1708-1729; settings
// SetOptimConfig :710-755, SetInitialValueLRCov :7505-7521, constants :5255-5345).
struct InternalSettings {
  std::string optimizer;           // "gradient_descent" | "fisher_scoring"
  double lr = -1.;                 // lr_cov (< 0: 0.1 for gradient descent, 1 for Fisher scoring)
  double acc_rate = 0.5;           // acc_rate_cov
  bool nesterov = true;            // use_nesterov_acc (gradient descent only)
  int schedule = 0;                // nesterov_schedule_version
  int momentum_offset = 2;
  int max_iter = 1000;
  double delta = 1e-6;             // delta_rel_conv
  bool crit_params = false;        // convergence_criterion = "relative_change_in_parameters"
};

// The objective on the transformed scale (trafo[0] = sigma^2, then the log-scale parameters' values).
class InternalObjective {
 public:
  virtual ~InternalObjective() = default;
  // negative log-likelihood at trafo (sigma^2 = trafo[0] as given); NaN allowed (non-fatal)
  virtual double Nll(const std::vector<double>& trafo) = 0;
  // gradient wrt the log of the transformed parameters: profile -> sigma^2 = q / n (returned) and no nugget
  // entry (include_error_var = false), else the nugget first
  virtual std::vector<double> Grad(const std::vector<double>& trafo, bool profile, double* sigma2) = 0;
  // Fisher information of the log transformed parameters incl. the nugget (CalcFisherInformation with
  // transf_scale = true, include_error_var = true), row-major
  virtual std::vector<double> FisherTrafo(const std::vector<double>& trafo) = 0;
};

// Linear regression coefficients updated by GLS at the start of every iteration (optimizer_coef "wls",
// re_model_template.h:1327-1330): Update returns the objective after the update (the Armijo baseline,
// EvalNegLogLikelihoodOnlyUpdateFixedEffects); CoefConverged tests |beta - beta_lag1| <= delta |beta_lag1| (:1712-1716).
class InternalCoefHook {
 public:
  virtual ~InternalCoefHook() = default;
  virtual double Update(const std::vector<double>& trafo) = 0;
  virtual bool CoefConverged(double delta) const = 0;
};

// Runs the optimizer from trafo (overwritten with the estimate; trafo[0] the final sigma^2); returns the
// number of iterations (the reference's num_it) and the final objective value in *nll.
int internal_optimize(InternalObjective& f, std::vector<double>& trafo, const InternalSettings& s, double* nll,
                      InternalCoefHook* coef = nullptr);
bool is_internal_optimizer(const std::string& name);

// "nelder_mead": OptimLib's Nelder-Mead as OptimExternal runs it (optim_utils.h:626-643, 680-700;
// external_libs/OptimLib/unconstrained/nm.hpp nm_impl with adaptive parameters, algo_settings_t defaults):
// the initial simplex x0 + 0.05 x0_i e_i (0.00025 e_i for a zero entry), reflection / expansion / outside and
// inside contraction / shrink, convergence when the largest change of the vertex values relative to
// 1e-8 + max |old value| is <= tol_obj, or the same for the vertices <= tol_sol, or iter_max iterations.
// x is overwritten with the best vertex; returns the reference's opt_iter and the objective at x in *fval
// (error_reporting's final evaluation).
int nelder_mead(const std::function<double(const std::vector<double>&)>& f, std::vector<double>& x, int iter_max,
                double tol_obj, double tol_sol, double* fval);

}  // namespace gpb_amd
