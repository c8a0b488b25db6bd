// GroupedModel: the model object behind the GPB_* C ABI for Gaussian models whose random effects
// are K grouped (crossed or nested) effects — the reference's REModelTemplate<sp_mat_rm_t, ...>
// with num_re_group > 0 and no GP (re_model.cpp:21-111, re_model_template.h:95-465). Parameters
// (original scale): [sigma^2 (error variance), sigma_1^2, ..., sigma_K^2]; transformed scale
// [sigma^2, tau_1, ..., tau_K], tau_k = sigma_k^2 / sigma^2 (TransformCovPars). The likelihood runs
// on the device in GroupedRE (grouped.h); this class keeps the configuration, the response and the
// optimizer state.
#pragma once

#include <hip/hip_runtime.h>

#include <memory>
#include <string>
#include <unordered_map>
#include <vector>

#include "grouped.h"
#include "optim.h"
#include "re_model.h"

namespace gpb_amd {

class GroupedModel {
 public:
  // levels: K x n level indices (order of first appearance, as RECompGroup numbers its labels,
  // re_comp.h:245-264). matrix_inversion_method: "default" -> "iterative" for K >= 2, "cholesky"
  // for K == 1 (UseIterativeByDefault, re_model_template.h:6719-6724).
  GroupedModel(int n, const std::vector<std::vector<int>>& levels, const std::string& matrix_inversion_method,
               int seed, std::vector<std::unordered_map<std::string, int>> label_index = {});
  ~GroupedModel();
  // Combined model (re_model_template.h:236-239 allows grouped random effects beside a GP for
  // gp_approx = "none"): one dense GP component on coords (host column-major n x d, as GPB_CreateREModel passes
  // them) with covariance cov_type. Parameters [sigma^2, sigma_1^2 .. sigma_K^2, sigma_gp^2, rho] (the
  // reference's component order: grouped effects first); the likelihood on DenseSolver with the grouped term.
  void AttachGP(int d, const double* coords_colmajor, int cov_type, int seed);
  bool has_gp() const { return dense_ != nullptr; }
  int gp_dim() const { return gp_d_; }

  int n() const { return n_; }
  int K() const { return re_->K(); }
  int num_cov_pars() const { return 1 + re_->K() + (has_gp() ? 2 : 0); }
  const std::string& matrix_inversion_method() const { return mim_; }
  bool iterative() const { return mim_ == "iterative"; }
  std::string cg_preconditioner_type() const { return iterative() ? "ssor" : ""; }
  const std::vector<int>& levels_per_effect() const { return re_->levels_per_effect(); }

  // y - fixed_effects (nullable) is the response; y (nullable: keep) is stored for GetResponseData.
  void SetResponseAndOffset(const double* y, const double* fixed_effects);
  bool HasY() const { return y_set_; }
  void GetResponseData(double* y) const;

  // cov_pars on the original scale. profile: 0 -> gradient wrt log of all 1 + K parameters
  // (include_error_var), 1 -> sigma^2 profiled out, gradient wrt log tau (the L-BFGS unit).
  EvalResult Eval(const double* cov_pars_orig, bool want_grad, int profile);
  EvalResult EvalTrafo(const double* trafo, bool want_grad, int profile, bool fatal_on_nan = true);

  void SetOptimSettings(const double* init_cov_pars, double lr, int max_iter, double delta_rel_conv,
                        const char* optimizer, int m_lbfgs);
  void SetPreconditioner(const char* preconditioner);
  void SetInternalOptimSettings(double acc_rate, bool nesterov, int schedule, int momentum_offset,
                                const char* convergence_criterion) {
    isettings_.acc_rate = acc_rate;
    isettings_.nesterov = nesterov;
    isettings_.schedule = schedule;
    isettings_.momentum_offset = momentum_offset;
    if (convergence_criterion != nullptr && convergence_criterion[0] != '\0')
      isettings_.crit_params = check_convergence_criterion(convergence_criterion);
  }
  // Fisher information of the log transformed parameters (Fisher scoring; cholesky, no GP), row-major
  std::vector<double> FisherTrafo(const double* trafo);
  const std::string& optimizer_cov() const { return optimizer_name_; }
  // OptimCovPar (re_model.cpp:339-401 -> OptimExternal "lbfgs", optim_utils.h:561-706): L-BFGS on
  // log tau with sigma^2 profiled out (EvalLLforLBFGSpp, optim_utils.h:269-313).
  void OptimCovPar(const double* y, const double* fixed_effects);
  void SetNumIter(int it) { num_iter_ = it; }
  int num_it() const { return num_it_; }
  double last_nll() const { return last_nll_; }
  const std::vector<double>& last_cov_pars() const { return last_cov_pars_; }
  void GetInitCovPar(double* out) const;
  // GPB_GetNumCGSteps / GetNumCGStepsTridiag (re_model_template.h:527-552)
  int num_cg_steps() const { return last_cg_its_; }
  int num_cg_steps_tridiag() const { return last_lanczos_; }
  // GPB_PredictREModelTrainingDataRandomEffects (re_model.cpp -> PredictTrainingDataRandomEffects,
  // grouped branch re_model_template.h:4065-4167): out[k n + i] = posterior mean of effect k at
  // observation i's level; calc_var (cholesky only, as the reference's iterative branch refuses it):
  // out[K n + k n + i] = its posterior variance. cov_pars original scale (null: the last ones).
  void PredictTrainingDataRandomEffects(const double* cov_pars, const double* y, double* out,
                                        const double* fixed_effects, bool calc_var);
  // GPB_PredictREModel with re_group_data_pred (re_model_template.h:3146 -> CalcPred :10026-10535, Woodbury branch): means; with
  // predict_var / predict_cov_mat (cholesky only; iterative: the reference's simulation, refused) the
  // predictive (co)variances nugget [predict_response] + sum_k tau_k [new level, same label] + e_p^T A^-1 e_q,
  // e_p the indicator of p's seen levels (derivation in grouped.h), times sigma^2.
  // Combined models: gp_coords_pred (column-major n_pred x d) required; mean = Sigma_po Psi^-1 y, (co)variances
  // from the dense factor with the grouped cross-covariances (DenseSolver::Predict).
  void Predict(const double* y, int n_pred, const char* re_group_data_pred, const double* gp_coords_pred,
               const double* cov_pars, bool predict_cov_mat, bool predict_var, bool predict_response,
               const double* fixed_effects, const double* fixed_effects_pred, double* out);
  // GPB_GetCovPar(calc_std_dev) (CalcStdDevCovPar re_model_template.h:9775-9789 ->
  // CalcFisherInformation_Only_Grouped_REs_Woodbury :9559-9651): sqrt(diag(FI^-1)) at the original-scale
  // cov_pars; cholesky only (the iterative branch is a stochastic estimate: refused)
  void StdDevCovPars(const double* cov_pars, double* sd);
  bool CanCalculateStandardErrorsCovPars() const { return !iterative() && !has_gp(); }
  IterativeConfig iter;

 private:
  void UseDevice() const;
  void FindInitCovPar(const double* y, double* trafo) const;
  // transformed <-> original scale: tau_k = sigma_k^2 / sigma^2, v = sigma_gp^2 / sigma^2, phi = range_trafo(rho)
  void ToTrafo(const double* orig, double* trafo) const;
  void ToOrig(const double* trafo, double sigma2, double* orig) const;
  EvalResult EvalDense(const double* trafo, bool want_grad, int profile, bool fatal_on_nan);
  // the prediction points' level indices (K x n_pred, effect-major; -1 - id for labels not seen in training,
  // equal ids for equal new labels) and the per-effect label strings (nullable)
  void PredictCombined(const double* y, int n_pred, const char* re_group_data_pred, const double* gp_coords_pred,
                       const double* cov_pars, bool predict_cov_mat, bool predict_var, bool predict_response,
                       const double* fixed_effects, const double* fixed_effects_pred, double* out);
  std::vector<int> PredLevels(int n_pred, const char* re_group_data_pred, std::vector<std::vector<std::string>>* labels) const;
  std::vector<double> Blup(const double* cov_pars, const double* y, const double* fixed_effects,
                           std::vector<double>* var);

  int n_;
  int device_ = 0;
  std::string mim_;
  hipStream_t stream_ = nullptr;
  std::unique_ptr<GroupedRE> re_;
  std::vector<std::vector<int>> levels_;                       // K x n
  std::vector<std::unordered_map<std::string, int>> label_index_;   // label -> level, per effect
  std::vector<double> y_raw_, y_;
  bool y_set_ = false;

  LbfgsSettings optim_;
  InternalSettings isettings_;
  std::string optimizer_name_ = "lbfgs";
  std::vector<double> init_cov_pars_, cov_pars_orig_, init_used_, last_cov_pars_;
  bool cov_pars_initialized_ = false;
  int num_it_ = 0;
  int num_iter_ = 0;   // the reference's num_iter_ (warm starts of the A^-1 Z^T y solve)
  double last_nll_ = 0.;
  int last_cg_its_ = 0, last_lanczos_ = 0;
  // combined GP + grouped (AttachGP)
  std::unique_ptr<DenseSolver> dense_;
  int gp_d_ = 0, cov_type_ = 0, seed_ = 0;
  std::vector<double> coords_;   // row-major n x d
  DevBuf<double> d_X_, d_y_;
  DevBuf<int> d_lev_;            // K x n
};

// Parses re_group_data (column-major K x n NUL-terminated labels, re_model_template.h:6246-6270)
// into level indices numbered in order of first appearance per effect.
// label_index (nullable) receives the per-effect label -> level maps.
std::vector<std::vector<int>> parse_group_levels(int n, int K, const char* re_group_data,
                                                 std::vector<std::unordered_map<std::string, int>>* label_index = nullptr);

}  // namespace gpb_amd
