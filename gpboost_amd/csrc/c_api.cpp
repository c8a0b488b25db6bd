// extern "C" boundary: the GPB_* / LGBM_* symbols of include/gpboost_amd.h.
// Error convention of the reference (src/LightGBM/c_api.cpp:54-58, include/LightGBM/c_api.h:1798-1810):
// every call returns 0 / -1, the message goes to a 512-byte thread-local buffer read by
// LGBM_GetLastError. Logging goes through LGBM_RegisterLogCallback when registered
// (log.h:171-191 semantics: "[GPBoost] [Info] ..."), else stderr.
#include "gpboost_amd.h"

#include <cmath>
#include <cstdarg>
#include <cstring>
#include <exception>
#include <mutex>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "grouped_model.h"
#include "re_model.h"

using gpb_amd::GroupedModel;
using gpb_amd::REModelAMD;

namespace {

// Handles of grouped-random-effects models (GroupedModel); every other handle is an REModelAMD.
std::mutex g_grouped_mu;
std::unordered_set<const void*> g_grouped;

GroupedModel* as_grouped(REModelHandle h) {
  std::lock_guard<std::mutex> lk(g_grouped_mu);
  return g_grouped.count(h) ? reinterpret_cast<GroupedModel*>(h) : nullptr;
}

// Prediction data saved by GPB_SetPredictionData for GPB_PredictREModel(use_saved_data = true)
// (REModelTemplate::SetPredictionData / Predict, re_model_template.h:3061-3119, 3168-3206): copies, per
// handle; a later call replaces the kinds of data it gives.
struct SavedPred {
  int num_data_pred = 0;
  std::vector<double> gp_coords;     // column-major num_data_pred x dim
  std::vector<double> covariates;    // column-major num_data_pred x p
  std::vector<char> re_group;        // num_data_pred x K NUL-terminated level strings, effect-major
};
std::mutex g_saved_mu;
std::unordered_map<const void*, SavedPred> g_saved;

thread_local char g_last_error[512] = "Everything is fine";
void (*g_log_callback)(const char*) = nullptr;

void set_last_error(const char* msg) {
  std::strncpy(g_last_error, msg, sizeof(g_last_error) - 1);
  g_last_error[sizeof(g_last_error) - 1] = '\0';
}

void vlog(const char* level, const char* fmt, va_list ap) {
  char buf[1024];
  int k = std::snprintf(buf, sizeof(buf), "[GPBoost] [%s] ", level);
  std::vsnprintf(buf + k, sizeof(buf) - k, fmt, ap);
  std::strncat(buf, "\n", sizeof(buf) - std::strlen(buf) - 1);
  if (g_log_callback) g_log_callback(buf);
  else std::fputs(buf, stderr);
}

REModelAMD* model(REModelHandle h) {
  if (h == nullptr) gpb_amd::Fatal("REModelHandle is NULL");
  if (as_grouped(h) != nullptr)
    gpb_amd::Fatal("this function is not supported for models with grouped random effects by gpboost_amd");
  return reinterpret_cast<REModelAMD*>(h);
}

std::string str_or(const char* s, const char* def) { return s ? std::string(s) : std::string(def); }

void copy_name(const std::string& name, char* out_str, int* num_char) {
  if (num_char) *num_char = (int)name.size() + 1;
  if (out_str) std::memcpy(out_str, name.c_str(), name.size() + 1);
}

}  // namespace

namespace gpb_amd {

void Fatal(const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  std::vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  throw std::runtime_error(buf);
}

void Info(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vlog("Info", fmt, ap);
  va_end(ap);
}

void Warning(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vlog("Warning", fmt, ap);
  va_end(ap);
}

}  // namespace gpb_amd

#define API_BEGIN() try {
#define API_END()                                  \
  }                                                \
  catch (std::exception & ex) {                    \
    set_last_error(ex.what());                     \
    return -1;                                     \
  }                                                \
  catch (std::string & ex) {                       \
    set_last_error(ex.c_str());                    \
    return -1;                                     \
  }                                                \
  catch (...) {                                    \
    set_last_error("unknown exception");           \
    return -1;                                     \
  }                                                \
  return 0;

extern "C" {

const char* LGBM_GetLastError(void) { return g_last_error; }

int LGBM_RegisterLogCallback(void (*callback)(const char*)) {
  API_BEGIN();
  g_log_callback = callback;
  API_END();
}

int GPB_CreateREModel(int32_t num_data, const int32_t* cluster_ids_data, const char* re_group_data,
                      int32_t num_re_group, const double* re_group_rand_coef_data,
                      const int32_t* ind_effect_group_rand_coef, int32_t num_re_group_rand_coef,
                      const int* drop_intercept_group_rand_effect, int32_t num_gp, const double* gp_coords_data,
                      const int dim_gp_coords, const double* gp_rand_coef_data, int32_t num_gp_rand_coef,
                      const char* cov_fct, double cov_fct_shape, const char* gp_approx, double cov_fct_taper_range,
                      double cov_fct_taper_shape, int num_neighbors, const char* vecchia_ordering,
                      int num_ind_points, double cover_tree_radius, const char* ind_points_selection,
                      const char* likelihood, double likelihood_additional_param,
                      const char* matrix_inversion_method, int seed, int num_parallel_threads, bool GPU_use,
                      bool has_weights, const double* weights, double likelihood_learning_rate,
                      REModelHandle* out) {
  API_BEGIN();
  (void)re_group_rand_coef_data; (void)ind_effect_group_rand_coef; (void)drop_intercept_group_rand_effect;
  (void)cov_fct_taper_range; (void)cov_fct_taper_shape;
  (void)likelihood_additional_param; (void)num_parallel_threads; (void)GPU_use;
  (void)weights; (void)likelihood_learning_rate;
  if (out == nullptr) gpb_amd::Fatal("'out' is NULL");
  if (num_re_group_rand_coef > 0 || num_gp_rand_coef > 0 || gp_rand_coef_data != nullptr)
    gpb_amd::Fatal("random coefficients are out of scope for gpboost_amd (SURVEY.md §8)");
  if (has_weights) gpb_amd::Fatal("'weights' are not supported by gpboost_amd");
  if (cluster_ids_data != nullptr) {
    for (int32_t i = 1; i < num_data; ++i)
      if (cluster_ids_data[i] != cluster_ids_data[0]) gpb_amd::Fatal("multiple clusters (cluster_ids) are out of scope for gpboost_amd");
  }
  if (seed < 0) gpb_amd::Fatal("seed must be >= 0");
  if (num_re_group > 0 || re_group_data != nullptr) {   // grouped random effects (GroupedModel)
    if (num_re_group <= 0 || re_group_data == nullptr) gpb_amd::Fatal("re_group_data and num_re_group must be given together");
    if ((num_gp > 0) != (gp_coords_data != nullptr)) gpb_amd::Fatal("num_gp and gp_coords_data must be given together");
    if (num_gp > 1) gpb_amd::Fatal("gpboost_amd supports at most one GP component (num_gp = 1)");
    if (num_gp == 1 && str_or(gp_approx, "none") != "none")
      gpb_amd::Fatal("GP + grouped random effects models with gp_approx = '%s' are not supported (the reference "
                     "allows only 'none' there, re_model_template.h:236-239)", gp_approx);
    if (str_or(likelihood, "gaussian") != "gaussian")
      gpb_amd::Fatal("grouped random effects with likelihood '%s' are not supported by gpboost_amd (supported: gaussian)",
                     likelihood);
    if (num_data <= 0) gpb_amd::Fatal("num_data must be > 0");
    std::vector<std::unordered_map<std::string, int>> index;
    auto levels = gpb_amd::parse_group_levels(num_data, num_re_group, re_group_data, &index);
    std::string mim = str_or(matrix_inversion_method, "default");
    if (num_gp == 1 && mim == "default") mim = "cholesky";   // a GP beside: the dense path
    std::unique_ptr<GroupedModel> gm(new GroupedModel(num_data, levels, mim, seed, std::move(index)));
    if (num_gp == 1)
      gm->AttachGP(dim_gp_coords, gp_coords_data, gpb_amd::parse_cov(str_or(cov_fct, "exponential"), cov_fct_shape),
                   seed);
    auto* g = gm.release();
    {
      std::lock_guard<std::mutex> lk(g_grouped_mu);
      g_grouped.insert(g);
    }
    *out = g;
    return 0;   // (inside API_BEGIN's try; API_END's trailing return is not reached)
  }
  if (num_gp != 1 || gp_coords_data == nullptr) gpb_amd::Fatal("gpboost_amd requires exactly one GP component (num_gp = 1)");
  gpb_amd::ModelConfig cfg;
  cfg.n = num_data;
  cfg.d = dim_gp_coords;
  cfg.cov_fct = str_or(cov_fct, "exponential");
  cfg.shape = cov_fct_shape;
  cfg.gp_approx = str_or(gp_approx, "none");
  cfg.num_neighbors = num_neighbors;
  cfg.vecchia_ordering = str_or(vecchia_ordering, "random");
  cfg.likelihood = str_or(likelihood, "gaussian");
  cfg.matrix_inversion_method = str_or(matrix_inversion_method, "default");
  cfg.seed = seed;
  cfg.num_ind_points = num_ind_points;
  cfg.cover_tree_radius = cover_tree_radius;
  cfg.ind_points_selection = str_or(ind_points_selection, "kmeans++");
  *out = new REModelAMD(cfg, gp_coords_data);
  API_END();
}

int GPB_REModelFree(REModelHandle handle) {
  API_BEGIN();
  {
    std::lock_guard<std::mutex> lk(g_saved_mu);
    g_saved.erase(handle);
  }
  if (GroupedModel* g = as_grouped(handle)) {
    {
      std::lock_guard<std::mutex> lk(g_grouped_mu);
      g_grouped.erase(handle);
    }
    delete g;
    return 0;
  }
  delete reinterpret_cast<REModelAMD*>(handle);
  API_END();
}

int GPB_SetOptimConfig(REModelHandle handle, double* init_cov_pars, double lr, double acc_rate_cov, int max_iter,
                       double delta_rel_conv, bool use_nesterov_acc, int nesterov_schedule_version, bool trace,
                       const char* optimizer, int momentum_offset, const char* convergence_criterion,
                       int num_covariates, double* init_coef, double lr_coef, double acc_rate_coef,
                       const char* optimizer_coef, int cg_max_num_it, int cg_max_num_it_tridiag,
                       double cg_delta_conv, int num_rand_vec_trace, bool reuse_rand_vec_trace,
                       const char* cg_preconditioner_type, int seed_rand_vec_trace, int piv_chol_rank,
                       double* init_aux_pars, bool estimate_aux_pars, const int* estimate_cov_par_index,
                       int m_lbfgs, double delta_conv_mode_finding) {
  // re_model.cpp:234-332 / re_model_template.h:686-823: the settings of the likelihood path and
  // of the covariance-parameter optimizer (GPB_OptimCovPar; "lbfgs" only). Settings of the
  // gradient-descent / Nesterov / coefficient optimizers have no effect here (no covariates).
  API_BEGIN();
  // acc_rate_cov / use_nesterov_acc / nesterov_schedule_version / momentum_offset / convergence_criterion drive the
  // internal optimizers ("gradient_descent", "fisher_scoring"); L-BFGS always tests the relative change of the
  // objective (optim_utils.h:656-657)
  (void)trace;
  (void)lr_coef; (void)acc_rate_coef; (void)piv_chol_rank;
  if (GroupedModel* g = as_grouped(handle)) {   // Gaussian grouped model: no aux parameters, no coefficients
    (void)num_covariates; (void)init_coef; (void)optimizer_coef; (void)init_aux_pars; (void)estimate_aux_pars;
    (void)delta_conv_mode_finding;
    g->SetOptimSettings(init_cov_pars, lr, max_iter, delta_rel_conv, optimizer, m_lbfgs);
    g->SetInternalOptimSettings(acc_rate_cov, use_nesterov_acc, nesterov_schedule_version, momentum_offset,
                                convergence_criterion);
    if (g->iterative()) {
      g->SetPreconditioner(cg_preconditioner_type);
      g->iter.cg_max_num_it = cg_max_num_it;
      g->iter.cg_max_num_it_tridiag = cg_max_num_it_tridiag;
      g->iter.cg_delta_conv = cg_delta_conv;
    }
    if (num_rand_vec_trace <= 0) gpb_amd::Fatal("num_rand_vec_trace must be > 0");
    g->iter.num_rand_vec_trace = num_rand_vec_trace;
    g->iter.seed_rand_vec_trace = seed_rand_vec_trace;
    g->iter.reuse_rand_vec_trace = reuse_rand_vec_trace;
    if (estimate_cov_par_index != nullptr && estimate_cov_par_index[0] >= 0) {
      for (int k = 0; k < g->num_cov_pars(); ++k)
        if (estimate_cov_par_index[k] <= 0) gpb_amd::Fatal("estimate_cov_par_index: fixing covariance parameters is not supported by gpboost_amd");
    }
    return 0;
  }
  REModelAMD* m = model(handle);
  (void)num_covariates; (void)init_coef;   // the "wls" coefficient update profiles beta out at every evaluation
  const bool iterative = m->config().matrix_inversion_method == "iterative";
  if (iterative && cg_preconditioner_type != nullptr && std::string(cg_preconditioner_type) != "") {
    // ParsePreconditionerAlias (re_model_template.h:6756): the VADU aliases only
    const std::string p(cg_preconditioner_type);
    if (p != "vadu" && p != "VADU" && p != "vecchia_approximation_with_diagonal_update" && p != "Sigma_inv_plus_BtWB")
      gpb_amd::Fatal("cg_preconditioner_type '%s' is not supported by gpboost_amd (supported: vadu)", p.c_str());
  }
  m->SetOptimSettings(init_cov_pars, lr, max_iter, delta_rel_conv, optimizer, m_lbfgs);
  m->SetInternalOptimSettings(acc_rate_cov, use_nesterov_acc, nesterov_schedule_version, momentum_offset,
                              convergence_criterion);
  // validated above; the preconditioner name is recorded for iterative models only (canonical "vadu")
  m->SetOptimizerNames(optimizer, optimizer_coef, iterative ? cg_preconditioner_type : nullptr);
  if (iterative) {   // :775-801
    m->iter.cg_max_num_it = cg_max_num_it;
    m->iter.cg_max_num_it_tridiag = cg_max_num_it_tridiag;
    m->iter.cg_delta_conv = cg_delta_conv;
  }
  if (num_rand_vec_trace <= 0) gpb_amd::Fatal("num_rand_vec_trace must be > 0");
  m->iter.num_rand_vec_trace = num_rand_vec_trace;   // :771-773
  m->iter.seed_rand_vec_trace = seed_rand_vec_trace;
  m->iter.reuse_rand_vec_trace = reuse_rand_vec_trace;
  if (delta_conv_mode_finding > 0.) m->iter.delta_conv_mode_finding = delta_conv_mode_finding;   // :820-822
  if (init_aux_pars != nullptr) m->SetInitAuxPars(init_aux_pars);
  m->estimate_aux_pars = estimate_aux_pars;   // :803
  if (estimate_cov_par_index != nullptr && estimate_cov_par_index[0] >= 0)   // SetOptimConfig :806-816
    m->SetEstimateCovParIndex(std::vector<int>(estimate_cov_par_index, estimate_cov_par_index + m->num_cov_pars()));
  API_END();
}

int GPB_EvalNegLogLikelihood(REModelHandle handle, const double* y_data, double* cov_pars,
                             const double* fixed_effects, double* negll) {
  API_BEGIN();
  if (GroupedModel* g = as_grouped(handle)) {
    if (cov_pars == nullptr)
      gpb_amd::Fatal("cov_pars is NULL: evaluating at the initial values is not supported for grouped random effects "
                     "models by gpboost_amd");
    if (fixed_effects != nullptr && y_data == nullptr)
      gpb_amd::Fatal("EvalNegLogLikelihood: 'y_data' cannot nullptr when 'fixed_effects' is provided");
    g->SetResponseAndOffset(y_data, fixed_effects);
    negll[0] = g->Eval(cov_pars, false, 0).nll;
    return 0;
  }
  REModelAMD* m = model(handle);
  if (fixed_effects != nullptr && y_data == nullptr && !m->config().latent)
    gpb_amd::Fatal("EvalNegLogLikelihood: 'y_data' cannot nullptr when 'fixed_effects' is provided");
  m->SetResponseAndOffset(y_data, fixed_effects);
  if (cov_pars == nullptr) {   // re_model.cpp:598-605: the current parameters, initialised if not defined
    if (y_data != nullptr) m->InitCovParsIfNotDefined(y_data, fixed_effects);
    else if (m->config().latent) m->InitCovParsIfNotDefined(nullptr, nullptr);
    if (m->current_cov_pars().empty()) gpb_amd::Fatal("Covariance parameters have not been initialized");
    const std::vector<double> cp = m->current_cov_pars();
    negll[0] = m->Eval(cp.data(), false, 0).nll;
    return 0;
  }
  negll[0] = m->Eval(cov_pars, false, 0).nll;
  API_END();
}

int GPB_SetPredictionData(REModelHandle handle, int32_t num_data_pred, const int32_t* cluster_ids_data_pred,
                          const char* re_group_data_pred, const double* re_group_rand_coef_data_pred,
                          double* gp_coords_data_pred, const double* gp_rand_coef_data_pred,
                          const double* covariate_data_pred, const char* vecchia_pred_type, int num_neighbors_pred,
                          double cg_delta_conv_pred, int nsim_var_pred, int rank_pred_approx_matrix_lanczos) {
  API_BEGIN();
  (void)cg_delta_conv_pred;   // the Vecchia-Laplace draws use the model's cg_delta_conv (likelihoods.h:12052)
  (void)rank_pred_approx_matrix_lanczos;
  if (handle == nullptr) gpb_amd::Fatal("REModelHandle is NULL");
  if (cluster_ids_data_pred != nullptr || re_group_rand_coef_data_pred != nullptr || gp_rand_coef_data_pred != nullptr)
    gpb_amd::Fatal("GPB_SetPredictionData: clusters and random coefficients are not supported by gpboost_amd");
  GroupedModel* g = as_grouped(handle);
  const bool has_data = re_group_data_pred != nullptr || gp_coords_data_pred != nullptr || covariate_data_pred != nullptr;
  if (has_data) {
    if (num_data_pred <= 0) gpb_amd::Fatal("num_data_pred must be > 0 when prediction data is given");   // CHECK :3075
    if (g != nullptr && ((gp_coords_data_pred != nullptr && !g->has_gp()) || covariate_data_pred != nullptr))
      gpb_amd::Fatal("GP coordinates or covariates for a grouped random effects model are not supported by gpboost_amd");
    if (g == nullptr && re_group_data_pred != nullptr)
      gpb_amd::Fatal("grouped random effects data for a GP model are not supported by gpboost_amd");
    SavedPred sp;
    {
      std::lock_guard<std::mutex> lk(g_saved_mu);
      auto it = g_saved.find(handle);
      if (it != g_saved.end()) sp = it->second;
    }
    if (sp.num_data_pred != num_data_pred) {   // kinds saved for another size would be read past their end
      if (gp_coords_data_pred == nullptr) sp.gp_coords.clear();
      if (covariate_data_pred == nullptr) sp.covariates.clear();
      if (re_group_data_pred == nullptr) sp.re_group.clear();
    }
    sp.num_data_pred = num_data_pred;
    if (gp_coords_data_pred != nullptr) {
      const size_t cnt = (size_t)num_data_pred * (g != nullptr ? g->gp_dim() : model(handle)->config().d);
      sp.gp_coords.assign(gp_coords_data_pred, gp_coords_data_pred + cnt);
    }
    if (covariate_data_pred != nullptr) {
      const int p = model(handle)->num_covariates();
      if (p <= 0) gpb_amd::Fatal("Covariate data 'X_pred' is provided but the model has no covariates");
      sp.covariates.assign(covariate_data_pred, covariate_data_pred + (size_t)num_data_pred * p);
    }
    if (re_group_data_pred != nullptr) {   // num_data_pred x K NUL-terminated strings
      const char* e = re_group_data_pred;
      for (long k = 0; k < (long)num_data_pred * g->K(); ++k) e += std::strlen(e) + 1;
      sp.re_group.assign(re_group_data_pred, e);
    }
    std::lock_guard<std::mutex> lk(g_saved_mu);
    g_saved[handle] = std::move(sp);
  }
  if (g == nullptr) model(handle)->SetPredictionData(vecchia_pred_type, num_neighbors_pred, nsim_var_pred);
  API_END();
}

int GPB_PredictREModel(REModelHandle handle, const double* y_data, int32_t num_data_pred, double* out_predict,
                       bool predict_cov_mat, bool predict_var, bool predict_response,
                       const int32_t* cluster_ids_data_pred, const char* re_group_data_pred,
                       const double* re_group_rand_coef_data_pred, double* gp_coords_data_pred,
                       const double* gp_rand_coef_data_pred, const double* cov_pars,
                       const double* covariate_data_pred, bool use_saved_data, const double* fixed_effects,
                       const double* fixed_effects_pred) {
  API_BEGIN();
  if (out_predict == nullptr) gpb_amd::Fatal("out_predict is NULL");
  SavedPred saved;
  if (use_saved_data) {   // re_model_template.h:3168-3206: the saved data replaces the arguments
    {
      std::lock_guard<std::mutex> lk(g_saved_mu);
      auto it = g_saved.find(handle);
      if (it == g_saved.end() || it->second.num_data_pred <= 0)
        gpb_amd::Fatal("No data has been set for making predictions. Call set_prediction_data first");
      saved = it->second;
    }
    if (num_data_pred > 0 && num_data_pred != saved.num_data_pred)
      gpb_amd::Fatal("num_data_pred (%d) differs from the saved prediction data (%d)", num_data_pred, saved.num_data_pred);
    num_data_pred = saved.num_data_pred;
    cluster_ids_data_pred = nullptr;
    re_group_rand_coef_data_pred = nullptr;
    gp_rand_coef_data_pred = nullptr;
    re_group_data_pred = saved.re_group.empty() ? nullptr : saved.re_group.data();
    gp_coords_data_pred = saved.gp_coords.empty() ? nullptr : saved.gp_coords.data();
    covariate_data_pred = saved.covariates.empty() ? nullptr : saved.covariates.data();
  }
  if (GroupedModel* g = as_grouped(handle)) {
    if (cluster_ids_data_pred != nullptr || re_group_rand_coef_data_pred != nullptr ||
        gp_rand_coef_data_pred != nullptr || covariate_data_pred != nullptr)
      gpb_amd::Fatal("predictions with clusters, random coefficients or covariates are not supported "
                     "for grouped random effects models by gpboost_amd");
    g->Predict(y_data, num_data_pred, re_group_data_pred, gp_coords_data_pred, cov_pars, predict_cov_mat, predict_var,
               predict_response, fixed_effects, fixed_effects_pred, out_predict);
    return 0;
  }
  if (cluster_ids_data_pred != nullptr || re_group_data_pred != nullptr || re_group_rand_coef_data_pred != nullptr ||
      gp_rand_coef_data_pred != nullptr)
    gpb_amd::Fatal("predictions with clusters, grouped random effects or random coefficients are not "
                   "supported by gpboost_amd");
  REModelAMD* m = model(handle);
  std::vector<double> r;
  const double* y = y_data;
  if (m->has_covariates()) {   // y - X beta - offset (SetYCalcCovCalcYAuxForPred, re_model_template.h:3386-3410)
    if (covariate_data_pred == nullptr)
      gpb_amd::Fatal("Covariate data 'X_pred' is not provided but the model has covariates");
    r = m->ResidualResponse(y_data, fixed_effects);
    y = r.data();
  } else if (covariate_data_pred != nullptr) {
    gpb_amd::Fatal("Covariate data 'X_pred' is provided but the model has no covariates");
  } else if (m->config().latent) {   // non-Gaussian: F is the offset of the location parameter (the mode);
    m->SetLatentOffset(m->ResolveOffset(fixed_effects));   // none given: the saved one (re_model_template.h:3306-3312)
  } else if (fixed_effects != nullptr) {   // the GP part of the response (re_model_template.h:3386-3393)
    if (y_data == nullptr) gpb_amd::Fatal("'y_data' cannot be NULL when 'fixed_effects' is provided");
    r.resize(m->config().n);
    for (int i = 0; i < m->config().n; ++i) r[i] = y_data[i] - fixed_effects[i];
    y = r.data();
  }
  // fixed_effects_pred (and X_pred beta) join the predictive mean before any response transform
  // (re_model_template.h:3929-3946)
  std::vector<double> mean_add;
  if (m->has_covariates() || fixed_effects_pred != nullptr) {
    mean_add.assign(num_data_pred, 0.);
    if (m->has_covariates()) m->AddLinearPredictor(covariate_data_pred, num_data_pred, mean_add.data());
    if (fixed_effects_pred != nullptr)
      for (int i = 0; i < num_data_pred; ++i) mean_add[i] += fixed_effects_pred[i];
  }
  m->Predict(y, num_data_pred, gp_coords_data_pred, cov_pars, predict_cov_mat, predict_var, predict_response,
             out_predict, mean_add.empty() ? nullptr : mean_add.data());
  API_END();
}

int GPB_EvalNegLogLikelihoodGrad(REModelHandle handle, const double* y_data, const double* cov_pars,
                                 const double* fixed_effects, int profile_sigma2, double* negll, double* grad,
                                 double* sigma2_out) {
  API_BEGIN();
  if (cov_pars == nullptr || negll == nullptr || grad == nullptr) gpb_amd::Fatal("NULL argument");
  gpb_amd::EvalResult res;
  if (GroupedModel* g = as_grouped(handle)) {
    g->SetResponseAndOffset(y_data, fixed_effects);
    res = g->Eval(cov_pars, true, profile_sigma2 ? 1 : 0);
  } else {
    REModelAMD* m = model(handle);
    m->SetResponseAndOffset(y_data, fixed_effects);
    res = m->Eval(cov_pars, true, profile_sigma2 ? 1 : 0);
  }
  negll[0] = res.nll;
  for (size_t k = 0; k < res.grad.size(); ++k) {
    double g = res.grad[k];
    if (std::isnan(g) || std::isinf(g)) {  // re_model_template.h:1944-1955
      gpb_amd::Warning("NaN or Inf occurred in gradient wrt covariance parameter number %d; it is set to 0", (int)k);
      g = 0.;
    }
    grad[k] = g;
  }
  if (sigma2_out) sigma2_out[0] = res.sigma2;
  API_END();
}

int GPB_GetCurrentNegLogLikelihood(REModelHandle handle, double* negll) {
  API_BEGIN();
  if (GroupedModel* g = as_grouped(handle)) {
    negll[0] = g->last_nll();
    return 0;
  }
  negll[0] = model(handle)->last_nll();
  API_END();
}

int GPB_GetCovPar(REModelHandle handle, double* cov_par, bool calc_std_dev) {
  API_BEGIN();
  // re_model.cpp:767-811: cov_par[0, P) = parameters, cov_par[P, 2P) = std devs if calc_std_dev
  if (GroupedModel* g = as_grouped(handle)) {
    const auto& p = g->last_cov_pars();
    if (p.empty()) gpb_amd::Fatal("Covariance parameters have not been estimated or correctly set ");
    for (size_t k = 0; k < p.size(); ++k) cov_par[k] = p[k];
    if (calc_std_dev) g->StdDevCovPars(p.data(), cov_par + p.size());
    return 0;
  }
  REModelAMD* m = model(handle);
  const auto p = m->last_cov_pars();
  if (p.empty()) gpb_amd::Fatal("Covariance parameters have not been estimated or correctly set ");
  for (size_t k = 0; k < p.size(); ++k) cov_par[k] = p[k];
  if (calc_std_dev) m->StdDevCovPars(p.data(), cov_par + p.size());
  API_END();
}

int GPB_GetNumIt(REModelHandle handle, int* num_it) {
  API_BEGIN();
  if (GroupedModel* g = as_grouped(handle)) {
    num_it[0] = g->num_it();
    return 0;
  }
  num_it[0] = model(handle)->num_it();
  API_END();
}

int GPB_GetInitCovPar(REModelHandle handle, double* init_cov_pars) {
  API_BEGIN();
  if (GroupedModel* g = as_grouped(handle)) {
    g->GetInitCovPar(init_cov_pars);
    return 0;
  }
  model(handle)->GetInitCovPar(init_cov_pars);
  API_END();
}

int GPB_OptimCovPar(REModelHandle handle, const double* y_data, const double* fixed_effects) {
  // c_api.cpp GPB_OptimCovPar -> REModel::OptimCovPar(y, fixed_effects, false, false)
  API_BEGIN();
  if (GroupedModel* g = as_grouped(handle)) {
    g->OptimCovPar(y_data, fixed_effects);
    return 0;
  }
  model(handle)->OptimCovPar(y_data, fixed_effects);
  API_END();
}

int GPB_OptimLinRegrCoefCovPar(REModelHandle handle, const double* y_data, const double* covariate_data,
                               int num_covariates, const double* fixed_effects) {
  // c_api.cpp:2843-2852 -> REModel::OptimLinRegrCoefCovPar (re_model.cpp:403-469)
  API_BEGIN();
  if (GroupedModel* g = as_grouped(handle)) {
    if (covariate_data != nullptr && num_covariates > 0)
      gpb_amd::Fatal("linear regression covariates with grouped random effects are not supported by gpboost_amd");
    g->OptimCovPar(y_data, fixed_effects);
    return 0;
  }
  model(handle)->OptimLinRegrCoefCovPar(y_data, covariate_data, num_covariates, fixed_effects);
  API_END();
}

int GPB_OptimCovParBoosting(REModelHandle handle, const double* y_data, const double* fixed_effects,
                            bool called_in_GPBoost_algorithm, bool reuse_learning_rates_from_previous_call) {
  // REModel::OptimCovPar(y, F, called_in_GPBoost_algorithm, reuse) (re_model.cpp:339-401)
  API_BEGIN();
  if (as_grouped(handle) != nullptr)
    gpb_amd::Fatal("the GPBoost-algorithm covariance update is not supported for grouped random effects models by "
                   "gpboost_amd");
  model(handle)->OptimCovPar(y_data, fixed_effects, called_in_GPBoost_algorithm, reuse_learning_rates_from_previous_call);
  API_END();
}

int GPB_GetInducingPoints(REModelHandle handle, int32_t* num_ind_points, double* ind_points) {
  API_BEGIN();
  if (as_grouped(handle) != nullptr) gpb_amd::Fatal("model does not use gp_approx = 'fitc'");
  const std::vector<double>& Z = model(handle)->InducingPoints();
  const int d = model(handle)->config().d;
  if (num_ind_points != nullptr) *num_ind_points = (int32_t)(Z.size() / d);
  if (ind_points != nullptr) std::copy(Z.begin(), Z.end(), ind_points);
  API_END();
}

int GPB_CalcGradientF(REModelHandle handle, double* y, const double* fixed_effects, bool calc_cov_factor) {
  // REModel::CalcGradient (re_model.cpp:667-680), the call the boosting objective makes
  // (regression_objective.hpp:164-179)
  API_BEGIN();
  model(handle)->CalcGradientF(y, fixed_effects, calc_cov_factor);
  API_END();
}

int GPB_CanCalculateStandardErrorsCovPars(REModelHandle handle, int* out) {
  API_BEGIN();
  if (GroupedModel* g = as_grouped(handle)) {   // cholesky: exact Fisher information; iterative: refused
    out[0] = (int)g->CanCalculateStandardErrorsCovPars();
    return 0;
  }
  out[0] = (int)model(handle)->CanCalculateStandardErrorsCovPars();
  API_END();
}

int GPB_GetCoef(REModelHandle handle, double* optim_coef, bool calc_std_dev) {
  API_BEGIN();
  model(handle)->GetCoef(optim_coef, calc_std_dev);
  API_END();
}

int GPB_PredictREModelTrainingDataRandomEffects(REModelHandle handle, const double* cov_pars_pred, const double* y_obs,
                                                double* out_predict, const double* fixed_effects, bool calc_var) {
  API_BEGIN();
  if (out_predict == nullptr) gpb_amd::Fatal("out_predict is NULL");
  if (GroupedModel* g = as_grouped(handle)) {
    g->PredictTrainingDataRandomEffects(cov_pars_pred, y_obs, out_predict, fixed_effects, calc_var);
    return 0;
  }
  model(handle)->PredictTrainingDataRandomEffects(cov_pars_pred, y_obs, out_predict, fixed_effects, calc_var);
  API_END();
}

int GPB_GetOptimizerCovPars(REModelHandle handle, char* out_str, int* num_char) {
  API_BEGIN();
  if (GroupedModel* g = as_grouped(handle)) {   // InitializeOptimSettings (re_model_template.h:7463-7474)
    copy_name(g->optimizer_cov(), out_str, num_char);
    return 0;
  }
  copy_name(model(handle)->optimizer_cov(), out_str, num_char);
  API_END();
}

int GPB_GetOptimizerCoef(REModelHandle handle, char* out_str, int* num_char) {
  API_BEGIN();
  if (as_grouped(handle) != nullptr) {
    copy_name("wls", out_str, num_char);
    return 0;
  }
  copy_name(model(handle)->optimizer_coef(), out_str, num_char);
  API_END();
}

int GPB_GetCGPreconditionerType(REModelHandle handle, char* out_str, int* num_char) {
  API_BEGIN();
  if (GroupedModel* g = as_grouped(handle)) {
    copy_name(g->cg_preconditioner_type(), out_str, num_char);
    return 0;
  }
  copy_name(model(handle)->cg_preconditioner_type(), out_str, num_char);
  API_END();
}

int GPB_GetNumCGSteps(REModelHandle handle, int* num_cg_steps) {
  // re_model_template.h:527-537: defined for models of several grouped random effects only
  API_BEGIN();
  GroupedModel* g = as_grouped(handle);
  if (g == nullptr) (void)model(handle);
  if (g == nullptr || !g->iterative())
    gpb_amd::Fatal("GetNumCGStepLast: this function is currently only implemented when having multiple grouped random "
                   "effects and iterative methods are used ");
  num_cg_steps[0] = g->num_cg_steps();
  API_END();
}

int GPB_GetNumCGStepsTridiag(REModelHandle handle, int* num_cg_steps) {
  API_BEGIN();   // re_model_template.h:542-552
  GroupedModel* g = as_grouped(handle);
  if (g == nullptr) (void)model(handle);
  if (g == nullptr || !g->iterative())
    gpb_amd::Fatal("GetNumCGStepLast: this function is currently only implemented when having multiple grouped random "
                   "effects and iterative methods are used ");
  num_cg_steps[0] = g->num_cg_steps_tridiag();
  API_END();
}

int GPB_SetLikelihood(REModelHandle handle, const char* likelihood) {
  API_BEGIN();
  if (likelihood == nullptr) gpb_amd::Fatal("likelihood is NULL");
  if (as_grouped(handle) != nullptr) {
    if (std::string(likelihood) != "gaussian")
      gpb_amd::Fatal("grouped random effects with likelihood '%s' are not supported by gpboost_amd (supported: "
                     "gaussian)", likelihood);
    return 0;
  }
  model(handle)->SetLikelihood(std::string(likelihood));
  API_END();
}

int GPB_GetResponseData(REModelHandle handle, double* response_data) {
  API_BEGIN();
  if (GroupedModel* g = as_grouped(handle)) {
    g->GetResponseData(response_data);
    return 0;
  }
  model(handle)->GetResponseData(response_data);
  API_END();
}

int GPB_GetCovariateData(REModelHandle handle, double* covariate_data) {
  API_BEGIN();
  model(handle)->GetCovariateData(covariate_data);
  API_END();
}

int GPB_GetOffsetData(REModelHandle handle, double* fixed_effects) {
  API_BEGIN();
  model(handle)->GetOffsetData(fixed_effects);
  API_END();
}

int GPB_SetOffsetData(REModelHandle handle, const double* fixed_effects) {
  API_BEGIN();
  model(handle)->SetOffsetData(fixed_effects);
  API_END();
}

int GPB_GetInitAuxPars(REModelHandle handle, double* aux_pars) {
  API_BEGIN();
  model(handle)->GetInitAuxPars(aux_pars);
  API_END();
}

int GPB_GetLikelihoodName(REModelHandle handle, char* out_str, int* num_char) {
  API_BEGIN();
  const std::string s = as_grouped(handle) != nullptr ? std::string("gaussian") : model(handle)->config().likelihood;
  std::memcpy(out_str, s.c_str(), s.size() + 1);
  num_char[0] = (int)s.size() + 1;
  API_END();
}

int GPB_GetNumAuxPars(REModelHandle handle, int* num_aux_pars) {
  API_BEGIN();
  num_aux_pars[0] = as_grouped(handle) != nullptr ? 0 : model(handle)->num_aux_pars();
  API_END();
}

int GPB_GetAuxPars(REModelHandle handle, double* aux_pars, char* out_str) {
  API_BEGIN();
  if (as_grouped(handle) != nullptr) {
    (void)aux_pars;
    if (out_str != nullptr) out_str[0] = '\0';
    return 0;
  }
  REModelAMD* m = model(handle);
  const auto& a = m->aux_pars();
  for (size_t k = 0; k < a.size(); ++k) aux_pars[k] = a[k];
  const std::string name = m->aux_par_name();
  if (out_str != nullptr) std::memcpy(out_str, name.c_str(), name.size() + 1);
  API_END();
}

int GPB_GetLatentVecchiaFactor(REModelHandle handle, const double* cov_pars, double* D_inv, double* B_vals,
                               double* dD_range, double* dB_range_vals) {
  API_BEGIN();
  model(handle)->GetLatentVecchiaFactor(cov_pars, D_inv, B_vals, dD_range, dB_range_vals);
  API_END();
}

int GPB_GetLastIterationInfo(REModelHandle handle, double* info) {
  API_BEGIN();
  model(handle)->GetLastIterationInfo(info);
  API_END();
}

int GPB_GetCholeskyPlanInfo(REModelHandle handle, double* info) {
  API_BEGIN();
  if (info == nullptr) gpb_amd::Fatal("NULL argument");
  model(handle)->CholeskyPlanInfo(info);
  API_END();
}

int GPB_GetNumCovPars(REModelHandle handle, int* num_cov_pars) {
  API_BEGIN();
  GroupedModel* g = as_grouped(handle);
  num_cov_pars[0] = g != nullptr ? g->num_cov_pars() : model(handle)->num_cov_pars();
  API_END();
}

int GPB_EvalVecchiaPartials(REModelHandle handle, const double* cov_pars, int32_t row_begin, int32_t row_end,
                            double* sums) {
  API_BEGIN();
  model(handle)->EvalVecchiaPartials(cov_pars, row_begin, row_end, sums);
  API_END();
}

int GPB_GetVecchiaStructure(REModelHandle handle, int32_t* perm, int32_t* neighbors) {
  API_BEGIN();
  model(handle)->GetVecchiaStructure(perm, neighbors);
  API_END();
}

int GPB_GetVecchiaFactor(REModelHandle handle, const double* cov_pars, double* D_inv, double* B_vals) {
  API_BEGIN();
  model(handle)->GetVecchiaFactor(cov_pars, D_inv, B_vals);
  API_END();
}

int GPB_GetLastKernelTimes(REModelHandle handle, double* kernel_ms) {
  API_BEGIN();
  model(handle)->GetLastKernelTimes(kernel_ms);
  API_END();
}

int GPB_BenchLatentOperators(REModelHandle handle, int t, int reps, double* out) {
  API_BEGIN();
  model(handle)->BenchLatentOperators(t, reps, out);
  API_END();
}

int GPB_CommIdSize(void) { return (int)sizeof(ncclUniqueId); }

int GPB_CommCreateId(char* id_out) {
  API_BEGIN();
  ncclUniqueId id;
  ncclResult_t r = ncclGetUniqueId(&id);
  if (r != ncclSuccess) gpb_amd::Fatal("ncclGetUniqueId failed: %s", ncclGetErrorString(r));
  std::memcpy(id_out, &id, sizeof(id));
  API_END();
}

int GPB_SetDistributed(REModelHandle handle, int rank, int world_size, const char* comm_id) {
  API_BEGIN();
  ncclUniqueId id;
  std::memset(&id, 0, sizeof(id));
  if (world_size > 1 && comm_id == nullptr) gpb_amd::Fatal("comm_id is NULL");
  if (comm_id != nullptr) std::memcpy(&id, comm_id, sizeof(id));
  // a given id joins an RCCL communicator even at world_size 1 (one-rank communicator: the same
  // in-library all-reduce path, which the single-GPU tests exercise)
  model(handle)->SetDistributed(rank, world_size, id, comm_id != nullptr);
  API_END();
}

int GPB_SetDistributedHostReduce(REModelHandle handle, int rank, int world_size,
                                 void (*allreduce)(double* buf, int count, void* user), void* user) {
  API_BEGIN();
  model(handle)->SetDistributedHost(rank, world_size, allreduce, user);
  API_END();
}

int GPB_PartitionRows(int32_t num_data, int world_size, int rank, int32_t* row_begin, int32_t* row_end) {
  API_BEGIN();
  if (world_size < 1 || rank < 0 || rank >= world_size) gpb_amd::Fatal("invalid rank/world_size");
  const int base = num_data / world_size, rem = num_data % world_size;
  row_begin[0] = rank * base + (rank < rem ? rank : rem);
  row_end[0] = row_begin[0] + base + (rank < rem ? 1 : 0);
  API_END();
}

int GPB_CombinePartials(const double* sums, int32_t num_data, double sigma2, int profile_sigma2, double* negll,
                        double* grad, double* sigma2_out) {
  API_BEGIN();
  gpb_amd::combine_partials(sums, num_data, sigma2, profile_sigma2 ? 1 : 0, negll, grad, sigma2_out);
  API_END();
}

}  // extern "C"
