/*
 * gpboost_amd — MI355X-native GP / mixed-effects likelihood engine.
 * C-ABI drop-in boundary (plain pointers and sizes, no torch or HIP types).
 *
 * Every GPB_* / LGBM_* entry point below has the signature and semantics of the
 * reference GPBoost C API it replaces (cited per function, paths relative to the
 * reference repository), so GPBoost's Python/R packages can bind this library
 * instead of lib_gpboost.so for the REModel likelihood path. Functions marked
 * EXTENSION do not exist in the reference (the reference exposes
 * no gradient entry point); they are additive.
 *
 * Conventions (identical to the reference): every function returns 0 on success
 * and -1 on failure; the failure message is kept in a thread-local buffer that
 * LGBM_GetLastError() returns (include/LightGBM/c_api.h:1798-1810,
 * src/LightGBM/c_api.cpp:54-58). Input arrays are borrowed for the duration of
 * the call and copied; output arrays are caller-allocated. A handle is not
 * thread-safe.
 *
 * All 29 GPB_* functions of the reference (include/LightGBM/c_api.h:1358-1786) are exported with
 * their signatures. Scope of this build: one GP component (num_gp = 1) with
 * cov_fct in {exponential, matern (shape 0.5/1.5/2.5), gaussian}; gp_approx "none" (dense
 * Cholesky) and "vecchia" with likelihood "gaussian" (exact), "vecchia" with "bernoulli_logit" and
 * "vecchia_latent" with "gaussian" (Laplace approximation, iterative methods); linear regression
 * covariates for the Gaussian likelihood (GLS, optimizer_coef "wls"); OR grouped random effects
 * (num_gp = 0, re_group_data with num_re_group >= 1 grouping variables, Gaussian likelihood; K = 1
 * closed form, K >= 2 iterative SSOR-PCG + SLQ as the reference's default). Latent models accept
 * repeated coordinates (the reference's unique-location form). Anything else fails with -1 and a
 * message naming the unsupported option.
 * The compute path is HIP on gfx950; there is no CPU fallback: if no GPU is
 * visible, GPB_CreateREModel fails.
 */
#ifndef GPBOOST_AMD_H_
#define GPBOOST_AMD_H_

#include <stdbool.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GPBOOST_AMD_EXPORT __attribute__((visibility("default")))

typedef void* REModelHandle;

/* ---------------------------------------------------------------- errors / logging */

/* replaces LGBM_GetLastError (include/LightGBM/c_api.h:54; c_api.cpp:1008) */
GPBOOST_AMD_EXPORT const char* LGBM_GetLastError(void);

/* replaces LGBM_RegisterLogCallback (include/LightGBM/c_api.h:61; c_api.cpp:1012) */
GPBOOST_AMD_EXPORT int LGBM_RegisterLogCallback(void (*callback)(const char*));

/* ---------------------------------------------------------------- model lifecycle */

/* replaces GPB_CreateREModel (include/LightGBM/c_api.h:1358-1390; c_api.cpp:2693-2762) */
GPBOOST_AMD_EXPORT int GPB_CreateREModel(int32_t num_data,
    const int32_t* cluster_ids_data,
    const char* re_group_data,
    int32_t num_re_group,
    const double* re_group_rand_coef_data,
    const int32_t* ind_effect_group_rand_coef,
    int32_t num_re_group_rand_coef,
    const int* drop_intercept_group_rand_effect,
    int32_t num_gp,
    const double* gp_coords_data,
    const int dim_gp_coords,
    const double* gp_rand_coef_data,
    int32_t num_gp_rand_coef,
    const char* cov_fct,
    double cov_fct_shape,
    const char* gp_approx,
    double cov_fct_taper_range,
    double cov_fct_taper_shape,
    int num_neighbors,
    const char* vecchia_ordering,
    int num_ind_points,
    double cover_tree_radius,
    const char* ind_points_selection,
    const char* likelihood,
    double likelihood_additional_param,
    const char* matrix_inversion_method,
    int seed,
    int num_parallel_threads,
    bool GPU_use,
    bool has_weights,
    const double* weights,
    double likelihood_learning_rate,
    REModelHandle* out);

/* replaces GPB_REModelFree (include/LightGBM/c_api.h:1397; c_api.cpp:2764-2768) */
GPBOOST_AMD_EXPORT int GPB_REModelFree(REModelHandle handle);

/* replaces GPB_SetOptimConfig (include/LightGBM/c_api.h:1433-1462; c_api.cpp:2770-2830).
 * Stored: the iterative-solver fields (cg_*, num_rand_vec_trace, seed_rand_vec_trace,
 * delta_conv_mode_finding), init_aux_pars / estimate_aux_pars, and the covariance-parameter
 * optimizer fields GPB_OptimCovPar uses: init_cov_pars (original scale), lr (L-BFGS initial
 * step factor, < 0: 1), max_iter, delta_rel_conv (< 0: 1e-6), optimizer (NULL / "" / "lbfgs";
 * others fail), optimizer_coef (NULL / "" / "wls"), m_lbfgs (<= 0: 6). init_coef has no effect:
 * the "wls" update profiles the coefficients out at every evaluation. */
GPBOOST_AMD_EXPORT int GPB_SetOptimConfig(REModelHandle handle,
    double* init_cov_pars,
    double lr,
    double acc_rate_cov,
    int max_iter,
    double delta_rel_conv,
    bool use_nesterov_acc,
    int nesterov_schedule_version,
    bool trace,
    const char* optimizer,
    int momentum_offset,
    const char* convergence_criterion,
    int num_covariates,
    double* init_coef,
    double lr_coef,
    double acc_rate_coef,
    const char* optimizer_coef,
    int cg_max_num_it,
    int cg_max_num_it_tridiag,
    double cg_delta_conv,
    int num_rand_vec_trace,
    bool reuse_rand_vec_trace,
    const char* cg_preconditioner_type,
    int seed_rand_vec_trace,
    int piv_chol_rank,
    double* init_aux_pars,
    bool estimate_aux_pars,
    const int* estimate_cov_par_index,
    int m_lbfgs,
    double delta_conv_mode_finding);

/* ---------------------------------------------------------------- likelihood evaluation */

/* replaces GPB_EvalNegLogLikelihood (include/LightGBM/c_api.h:1500; c_api.cpp:2854-2863).
 * cov_pars on the ORIGINAL scale: (sigma2, sigma1^2, rho) for the Gaussian likelihood,
 * (sigma1^2, rho) for latent models (likelihood "bernoulli_logit", or gp_approx
 * "vecchia_latent" whose error variance is the aux par set by GPB_SetOptimConfig's
 * init_aux_pars); for latent models negll is the Laplace-approximated value computed with
 * iterative methods (PCG + stochastic Lanczos quadrature, likelihoods.h:2765-3076).
 * nll written to negll[0]. y may be NULL to reuse the response set by the previous call. */
GPBOOST_AMD_EXPORT int GPB_EvalNegLogLikelihood(REModelHandle handle,
    const double* y_data,
    double* cov_pars,
    const double* fixed_effects,
    double* negll);

/* EXTENSION. nll and its gradient in one evaluation.
 * profile_sigma2 == 0: gradient with respect to log of every covariance parameter on the
 *   reference's transformed scale (sigma2, sigma1^2/sigma2, range transform), i.e.
 *   REModelTemplate::CalcGradPars(..., include_error_var=true) (re_model_template.h:1748-1818);
 *   grad has num_cov_pars entries.
 * profile_sigma2 == 1: the reference's L-BFGS objective unit
 *   (include/GPBoost/optim_utils.h:243-364): sigma2 is profiled out (yT Psi^-1 y / n),
 *   negll is the profiled nll, grad has num_cov_pars-1 entries (sigma2 excluded), and
 *   sigma2_out (may be NULL) receives the profiled sigma2.
 * Latent models (profile_sigma2 must be 0): gradient of the approximate negative marginal
 *   log-likelihood with respect to log(sigma1^2), log(range transform) and, for
 *   "vecchia_latent" with estimate_aux_pars, log(error variance) — what
 *   CalcGradPars -> CalcGradNegMargLikelihoodLaplaceApproxVecchia returns
 *   (likelihoods.h:4951-5206); grad needs num_cov_pars + num_aux_pars entries.
 * y may be NULL (reuse). */
GPBOOST_AMD_EXPORT int GPB_EvalNegLogLikelihoodGrad(REModelHandle handle,
    const double* y_data,
    const double* cov_pars,
    const double* fixed_effects,
    int profile_sigma2,
    double* negll,
    double* grad,
    double* sigma2_out);

/* replaces GPB_GetCurrentNegLogLikelihood (include/LightGBM/c_api.h:1512) */
GPBOOST_AMD_EXPORT int GPB_GetCurrentNegLogLikelihood(REModelHandle handle, double* negll);

/* replaces GPB_GetCovPar (include/LightGBM/c_api.h:1526; re_model.cpp:767-811): the estimated (or
 * last evaluated) cov_pars on the original scale in cov_par[0, P); calc_std_dev = true also writes
 * their standard deviations to cov_par[P, 2P) — square roots of the diagonal of the inverse Fisher
 * information (CalcStdDevCovPar re_model_template.h:9775-9789), computed on the device for dense
 * Gaussian models (gp_approx "none"); other models fail with a message. */
GPBOOST_AMD_EXPORT int GPB_GetCovPar(REModelHandle handle, double* cov_par, bool calc_std_dev);

/* replaces GPB_GetNumIt (include/LightGBM/c_api.h:1559): iterations of the last GPB_OptimCovPar */
GPBOOST_AMD_EXPORT int GPB_GetNumIt(REModelHandle handle, int* num_it);

/* replaces GPB_GetInitCovPar (include/LightGBM/c_api.h:1537; re_model.cpp:813-834): the initial
 * covariance parameters on the original scale (given by GPB_SetOptimConfig or determined by the
 * last GPB_OptimCovPar), -1 each when there are none yet */
GPBOOST_AMD_EXPORT int GPB_GetInitCovPar(REModelHandle handle, double* init_cov_pars);

/* replaces GPB_OptimCovPar (include/LightGBM/c_api.h:1471; c_api.cpp GPB_OptimCovPar ->
 * re_model.cpp:339-401): estimates the covariance parameters (and, for "vecchia_latent", the
 * error variance aux par) with the reference's default optimizer "lbfgs" (optim_utils.h:561-706:
 * L-BFGS on the log of the transformed parameters, Armijo backtracking, nugget profiled out for
 * the Gaussian likelihood). Initial values: init_cov_pars of GPB_SetOptimConfig, the previous
 * estimate, or the reference's FindInitCovPar heuristic (re_model_template.h:4388-4504). y may be
 * NULL to reuse the response already set; fixed_effects (length n) is an offset (Gaussian:
 * subtracted from y). Results: GPB_GetCovPar, GPB_GetAuxPars, GPB_GetNumIt,
 * GPB_GetCurrentNegLogLikelihood. */
GPBOOST_AMD_EXPORT int GPB_OptimCovPar(REModelHandle handle, const double* y_data, const double* fixed_effects);

/* replaces GPB_GetLikelihoodName (include/LightGBM/c_api.h:1659) */
GPBOOST_AMD_EXPORT int GPB_GetLikelihoodName(REModelHandle handle, char* out_str, int* num_char);

/* replaces GPB_GetNumAuxPars (include/LightGBM/c_api.h:1776) */
GPBOOST_AMD_EXPORT int GPB_GetNumAuxPars(REModelHandle handle, int* num_aux_pars);

/* replaces GPB_GetAuxPars (include/LightGBM/c_api.h:1766; c_api.cpp:3098-3107): aux_pars
 * caller-allocated (num_aux_pars), out_str receives the name of the first parameter. */
GPBOOST_AMD_EXPORT int GPB_GetAuxPars(REModelHandle handle, double* aux_pars, char* out_str);

/* replaces GPB_OptimLinRegrCoefCovPar (include/LightGBM/c_api.h:1485; c_api.cpp:2843-2852 ->
 * re_model.cpp:403-469): covariance parameters by L-BFGS (nugget profiled out) with the linear
 * regression coefficients profiled out by generalised least squares at every objective evaluation
 * (the reference's default optimizer_coef "wls" for the Gaussian likelihood,
 * re_model_template.h:7467-7470, optim_utils.h:297-313). covariate_data column-major
 * num_data x num_covariates (num_covariates + 1 <= 32); fixed_effects: an offset (nullable).
 * Gaussian likelihood only; results through GPB_GetCovPar / GPB_GetCoef. */
GPBOOST_AMD_EXPORT int GPB_OptimLinRegrCoefCovPar(REModelHandle handle,
    const double* y_data,
    const double* covariate_data,
    int num_covariates,
    const double* fixed_effects);

/* replaces GPB_CanCalculateStandardErrorsCovPars (include/LightGBM/c_api.h:1515; c_api.cpp:2873-2879;
 * re_model_template.h:1630-1632): out[0] = 1 for Gaussian-likelihood models, 0 for latent ones. */
GPBOOST_AMD_EXPORT int GPB_CanCalculateStandardErrorsCovPars(REModelHandle handle, int* out);

/* replaces GPB_GetCoef (include/LightGBM/c_api.h:1548; re_model.cpp:836-870): the coefficients
 * estimated by GPB_OptimLinRegrCoefCovPar in optim_coef[0, p); calc_std_dev also writes their
 * standard deviations sqrt(diag((X^T Psi^-1 X / sigma^2)^-1)) to optim_coef[p, 2p)
 * (CalcStdDevCoef, re_model_template.h:9797-9814). */
GPBOOST_AMD_EXPORT int GPB_GetCoef(REModelHandle handle, double* optim_coef, bool calc_std_dev);

/* replaces GPB_PredictREModelTrainingDataRandomEffects (include/LightGBM/c_api.h:1645;
 * re_model.cpp PredictTrainingDataRandomEffects): cov_pars_pred on the original scale (NULL: the
 * estimated / last evaluated ones), y_obs NULL: the stored response. Gaussian likelihood (dense and
 * Vecchia): out[0, n) = y - Psi^-1 y (minus X beta and the offset first), with calc_var
 * out[n, 2n) = sigma^2 (1 - diag(Psi^-1)); latent models: out[0, n) = the posterior mode
 * (calc_var fails). */
GPBOOST_AMD_EXPORT int GPB_PredictREModelTrainingDataRandomEffects(REModelHandle handle,
    const double* cov_pars_pred,
    const double* y_obs,
    double* out_predict,
    const double* fixed_effects,
    bool calc_var);

/* replace GPB_GetOptimizerCovPars / GPB_GetOptimizerCoef / GPB_GetCGPreconditionerType
 * (include/LightGBM/c_api.h:1670, 1681, 1692; re_model.cpp:174-208): the optimizer names ("" until
 * set or fitted, then "lbfgs" / "wls" for the Gaussian, "lbfgs" for latent models) and the CG
 * preconditioner ("vadu" for latent Vecchia models, "" otherwise). out_str must hold the name;
 * num_char receives its length + 1. */
GPBOOST_AMD_EXPORT int GPB_GetOptimizerCovPars(REModelHandle handle, char* out_str, int* num_char);
GPBOOST_AMD_EXPORT int GPB_GetOptimizerCoef(REModelHandle handle, char* out_str, int* num_char);
GPBOOST_AMD_EXPORT int GPB_GetCGPreconditionerType(REModelHandle handle, char* out_str, int* num_char);

/* replace GPB_GetNumCGSteps / GPB_GetNumCGStepsTridiag (include/LightGBM/c_api.h:1702, 1711): as in
 * the reference (re_model_template.h:527-552) they are defined for models with several grouped
 * random effects only and fail with the reference's message here. */
GPBOOST_AMD_EXPORT int GPB_GetNumCGSteps(REModelHandle handle, int* num_cg_steps);
GPBOOST_AMD_EXPORT int GPB_GetNumCGStepsTridiag(REModelHandle handle, int* num_cg_steps);

/* replaces GPB_SetLikelihood (include/LightGBM/c_api.h:1720; re_model.cpp:142-160): switches between
 * "gaussian" and "bernoulli_logit" before a model is estimated (Vecchia: exact <-> Laplace). */
GPBOOST_AMD_EXPORT int GPB_SetLikelihood(REModelHandle handle, const char* likelihood);

/* replace GPB_GetResponseData / GPB_GetCovariateData / GPB_GetOffsetData / GPB_SetOffsetData
 * (include/LightGBM/c_api.h:1729, 1738, 1747, 1756; re_model_template.h:5762-5825): the stored
 * response (original order, n), covariates (column-major n x p) and offset (n). */
GPBOOST_AMD_EXPORT int GPB_GetResponseData(REModelHandle handle, double* response_data);
GPBOOST_AMD_EXPORT int GPB_GetCovariateData(REModelHandle handle, double* covariate_data);
GPBOOST_AMD_EXPORT int GPB_GetOffsetData(REModelHandle handle, double* fixed_effects);
GPBOOST_AMD_EXPORT int GPB_SetOffsetData(REModelHandle handle, const double* fixed_effects);

/* replaces GPB_GetInitAuxPars (include/LightGBM/c_api.h:1785; re_model.cpp:1226-1238): the aux
 * parameters given by GPB_SetOptimConfig's init_aux_pars, -1 each when none were given. */
GPBOOST_AMD_EXPORT int GPB_GetInitAuxPars(REModelHandle handle, double* aux_pars);

/* EXTENSION (the reference has it as a C++ method only): REModel::OptimCovPar(y, fixed_effects,
 * called_in_GPBoost_algorithm, reuse_learning_rates_from_previous_call) (re_model.cpp:339-401), the
 * covariance update the GPBoost boosting objective runs every boosting round
 * (regression_objective.hpp:164, 178: Gaussian OptimCovPar(F - label, NULL, true, reuse), latent
 * OptimCovPar(NULL, score, true, reuse); reuse = the booster's reuse_learning_rates_gp_model, default
 * true). With called_in_GPBoost_algorithm the offset is not saved for prediction
 * (re_model_template.h:1051); with reuse as well, the L-BFGS inverse-Hessian approximation of the
 * previous call seeds the first direction at step 1 when both calls estimated the covariance
 * parameters (:880-881; LBFGS.h:158-171). GPB_OptimCovPar is this call with both flags false. */
GPBOOST_AMD_EXPORT int GPB_OptimCovParBoosting(REModelHandle handle, const double* y_data, const double* fixed_effects,
    bool called_in_GPBoost_algorithm, bool reuse_learning_rates_from_previous_call);

/* EXTENSION: the inducing points of a gp_approx = "fitc" model (the reference keeps them in
 * REModelTemplate::gp_coords_ip_mat_, chosen by CreateREComponentsFITC_FSA re_model_template.h:6931-7073:
 * kmeans++ GP_utils.cpp:269-295 or random utils.h:323-337). *num_ind_points receives m; ind_points
 * (nullable) receives them row-major m x dim_gp_coords. */
GPBOOST_AMD_EXPORT int GPB_GetInducingPoints(REModelHandle handle, int32_t* num_ind_points, double* ind_points);

/* EXTENSION (the reference has it as a C++ method only): REModel::CalcGradient (re_model.cpp:667-680
 * -> CalcGradientF re_model_template.h:3021-3043), what the GPBoost boosting objective calls after
 * GPB_OptimCovPar(handle, NULL, score) (regression_objective.hpp:164-179): the gradient of the
 * (approximate marginal) negative log-likelihood wrt the fixed effects F at the current covariance
 * parameters, written on y (length n, original order). Gaussian likelihood: input y = F - label,
 * output Psi^-1 y / sigma^2; latent models (Laplace): y is output only and F = fixed_effects, output
 * -dlog p(y|mode+F)/dF + the stochastic implicit-derivative terms (likelihoods.h:5337-5367).
 * calc_cov_factor = false (the booster's call after GPB_OptimCovParBoosting) keeps the Laplace mode
 * of the last evaluation; true re-runs the mode finding from it. */
GPBOOST_AMD_EXPORT int GPB_CalcGradientF(REModelHandle handle, double* y, const double* fixed_effects,
    bool calc_cov_factor);

/* ---------------------------------------------------------------- EXTENSION: introspection */

/* Number of covariance parameters (incl. sigma2) of the model. */
GPBOOST_AMD_EXPORT int GPB_GetNumCovPars(REModelHandle handle, int* num_cov_pars);

/* Vecchia ordering permutation (perm[i] = original index of the i-th point in the
 * Vecchia order) and neighbour lists (n x num_neighbors, -1 padded) exactly as the
 * reference builds them (Vecchia_utils.cpp:1094-1161). Arrays caller-allocated. */
GPBOOST_AMD_EXPORT int GPB_GetVecchiaStructure(REModelHandle handle, int32_t* perm, int32_t* neighbors);

/* Vecchia factor at the given cov_pars (original scale): D^-1 (n, Vecchia order) and
 * B values (n x num_neighbors; B(i, nbr) = -A_i, 0-padded). Computed on the GPU. */
GPBOOST_AMD_EXPORT int GPB_GetVecchiaFactor(REModelHandle handle, const double* cov_pars,
    double* D_inv, double* B_vals);

/* Latent Vecchia factor at cov_pars = (sigma1^2, rho) (latent models): D^-1 (n), B values
 * (n x num_neighbors) and their derivatives with respect to log(range transform)
 * (Vecchia_utils.cpp:1307-1632 with gauss_likelihood = false). Computed on the GPU. */
GPBOOST_AMD_EXPORT int GPB_GetLatentVecchiaFactor(REModelHandle handle, const double* cov_pars,
    double* D_inv, double* B_vals, double* dD_range, double* dB_range_vals);

/* Iterative-method statistics of the last latent evaluation: info[0] Newton iterations,
 * info[1] mode-finding (and gradient) CG iterations, info[2] Lanczos steps of the SLQ
 * block CG, info[3] the estimate of log|Sigma W + I|. */
GPBOOST_AMD_EXPORT int GPB_GetLastIterationInfo(REModelHandle handle, double* info);

/* Latent Vecchia models with matrix_inversion_method = "cholesky" (the sparse Cholesky of Sigma^-1 + W;
 * replaces the reference's SimplicialLLT analyzePattern / factorize, likelihoods.h:2946-2950): statistics of
 * the symbolic plan (built on first use): info[0] supernodes, info[1] levels of the supernodal tree,
 * info[2] entries of L (incl. amalgamation zeros), info[3] doubles of the dense fronts, info[4]
 * factorization flops, info[5] largest front, info[6] widest supernode, info[7] host analysis time (ms),
 * info[8] device time of the last factorization (ms). No reference counterpart (measurement only). */
GPBOOST_AMD_EXPORT int GPB_GetCholeskyPlanInfo(REModelHandle handle, double* info);

/* Timing of the last evaluation's dominant kernel (ms, HIP events on the model's stream),
 * for the benchmark's live roofline. kernel_ms[0] = factor/Cholesky kernel,
 * kernel_ms[1] = whole device-side evaluation. Exact Vecchia models record the events only for
 * evaluations after the first call of this function (they cost ~10 us of host time each);
 * before that it returns zeros. */
GPBOOST_AMD_EXPORT int GPB_GetLastKernelTimes(REModelHandle handle, double* kernel_ms);

/* Benchmark support (latent Vecchia, iterative): device time of the operator
 * A = B^T D^-1 B + W and of the VADU preconditioner on t columns, on the factor of the last
 * evaluation (HIP events, averaged over reps). out[0] = ms per A application, out[1] = ms
 * per preconditioner application, out[2] = nnz(B) incl. the unit diagonal, out[3] = dependent
 * kernel launches per preconditioner application (level sets of the tail + the head
 * kernels). No reference counterpart (measurement only). */
GPBOOST_AMD_EXPORT int GPB_BenchLatentOperators(REModelHandle handle, int t, int reps, double* out);

/* ---------------------------------------------------------------- prediction */

/* replaces GPB_SetPredictionData (include/LightGBM/c_api.h:1578; c_api.cpp). Only the settings
 * are supported: vecchia_pred_type (NULL: unchanged; supported: "order_obs_first_cond_obs_only",
 * the reference's default for Gaussian likelihoods, and "latent_order_obs_first_cond_obs_only", its
 * default for latent models, re_model_template.h:6485-6490), num_neighbors_pred (<= 0: unchanged;
 * default 2 * num_neighbors, :299) and nsim_var_pred (<= 0: unchanged; default 1000, :5374: draws of
 * the latent models' predictive-variance simulation). Prediction data must be NULL / 0 (pass it to
 * GPB_PredictREModel); cg_delta_conv_pred and rank_pred_approx_matrix_lanczos are accepted and
 * ignored (the Vecchia-Laplace draws use the model's cg_delta_conv, likelihoods.h:12043-12053). */
GPBOOST_AMD_EXPORT int GPB_SetPredictionData(REModelHandle handle,
    int32_t num_data_pred,
    const int32_t* cluster_ids_data_pred,
    const char* re_group_data_pred,
    const double* re_group_rand_coef_data_pred,
    double* gp_coords_data_pred,
    const double* gp_rand_coef_data_pred,
    const double* covariate_data_pred,
    const char* vecchia_pred_type,
    int num_neighbors_pred,
    double cg_delta_conv_pred,
    int nsim_var_pred,
    int rank_pred_approx_matrix_lanczos);

/* replaces GPB_PredictREModel (include/LightGBM/c_api.h:1617; Vecchia_utils.cpp:1634-2442,
 * re_model_template.h:3700-4071; dense CalcPred, FITC CalcPredFITC_FSA, grouped CalcPred): predictive mean
 * (out_predict[0 .. num_data_pred)) and, if predict_var, variances (out_predict[num_data_pred ..
 * 2 num_data_pred)), or, if predict_cov_mat, the num_data_pred^2 covariance (column-major).
 * gp_coords_data_pred column-major num_data_pred x dim_gp_coords. cov_pars on the original scale (NULL: those
 * of the last evaluation); y_data NULL: the response set before; use_saved_data: the data of
 * GPB_SetPredictionData. Exact Gaussian models: predict_response = false removes the nugget variance (latent
 * process). Every vecchia_pred_type is supported: order_obs_first_cond_obs_only / _cond_all, order_pred_first,
 * latent_order_obs_first_cond_obs_only / _cond_all (Gaussian and Laplace models). Latent Vecchia models
 * (PredictLaplaceApproxVecchia likelihoods.h:6576-6813): the Laplace mode at cov_pars, mean = -Bpo mode
 * (cond_all: Bp^-1 on top); with matrix_inversion_method = "iterative" predict_var / predict_cov_mat add the
 * reference's simulation term (nsim_var_pred draws; statistically equivalent, or the reference's own one-thread
 * stream with GPBOOST_AMD_PRED_DRAWS=reference), with "cholesky" the exact term ||L^-1 Bpo^T e_p||^2 on the
 * sparse Cholesky factor of Sigma^-1 + W (:6751-6811); predict_response gives the response mean / variance.
 * Deviation from the reference, by design: with vecchia_pred_type = "order_pred_first" the variances and the
 * covariance matrix are returned in prediction-point order (row p = the p-th prediction point); the
 * reference returns them in the order of its sparse factor's AMD permutation (an artefact of its
 * SimplicialLLT; the means are in prediction-point order on both sides). Unsupported inputs (clusters,
 * random coefficients, full_scale_vecchia, num_neighbors_pred > 64) return -1 with a message. */
GPBOOST_AMD_EXPORT int GPB_PredictREModel(REModelHandle handle,
    const double* y_data,
    int32_t num_data_pred,
    double* out_predict,
    bool predict_cov_mat,
    bool predict_var,
    bool predict_response,
    const int32_t* cluster_ids_data_pred,
    const char* re_group_data_pred,
    const double* re_group_rand_coef_data_pred,
    double* gp_coords_data_pred,
    const double* gp_rand_coef_data_pred,
    const double* cov_pars,
    const double* covariate_data_pred,
    bool use_saved_data,
    const double* fixed_effects,
    const double* fixed_effects_pred);

/* ---------------------------------------------------------------- EXTENSION: multi-GPU */

/* Size of the opaque communicator id (bytes). */
GPBOOST_AMD_EXPORT int GPB_CommIdSize(void);
/* Create a communicator id on one rank (to be broadcast to all ranks by the caller). */
GPBOOST_AMD_EXPORT int GPB_CommCreateId(char* id_out);
/* Join the model to an RCCL communicator. Exact Vecchia: rows (observations in Vecchia order)
 * are split into world_size contiguous blocks; this rank evaluates block `rank` and the
 * per-rank partial sums are all-reduced over RCCL (one all-reduce of 6 doubles per
 * evaluation). Latent Vecchia (iterative): every rank holds the whole factor and runs its
 * share of the num_rand_vec_trace probe columns; one all-reduce of 1 double per PCG iteration
 * (block stopping rule) and of the per-probe terms at the end (SURVEY.md §8e Option A).
 * Must be called before the first evaluation. comm_id may be NULL only at world_size 1 (no
 * communicator); a non-NULL id at world_size 1 creates a one-rank communicator (same data
 * path). */
GPBOOST_AMD_EXPORT int GPB_SetDistributed(REModelHandle handle, int rank, int world_size, const char* comm_id);
/* As GPB_SetDistributed, with the cross-rank sums done by `allreduce` on host buffers (it must
 * replace buf[0..count) by the element-wise sum over all ranks, e.g. a gloo all-reduce) instead
 * of RCCL: a transport for tests with several ranks on one GPU, where RCCL refuses to run. */
GPBOOST_AMD_EXPORT int GPB_SetDistributedHostReduce(REModelHandle handle, int rank, int world_size,
    void (*allreduce)(double* buf, int count, void* user), void* user);
/* The six per-row partial sums over Vecchia rows [row_begin, row_end) at cov_pars (original
 * scale), without any all-reduce: for callers that run their own communication. The
 * response must have been set by a previous evaluation. */
GPBOOST_AMD_EXPORT int GPB_EvalVecchiaPartials(REModelHandle handle, const double* cov_pars,
    int32_t row_begin, int32_t row_end, double* sums);
/* Host-side partition of n rows over world_size ranks (block distribution). */
GPBOOST_AMD_EXPORT int GPB_PartitionRows(int32_t num_data, int world_size, int rank, int32_t* row_begin, int32_t* row_end);
/* Host-side final assembly from all-reduced partial sums (exposed so the reduction
 * contract can be tested without a GPU): sums = [logdet, q, s1_var, s1_range, s2_var, s2_range]. */
GPBOOST_AMD_EXPORT int GPB_CombinePartials(const double* sums, int32_t num_data, double sigma2,
    int profile_sigma2, double* negll, double* grad, double* sigma2_out);

#ifdef __cplusplus
}
#endif
#endif /* GPBOOST_AMD_H_ */
