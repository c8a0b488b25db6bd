// REModelAMD: host-side model object behind the GPB_* C ABI.
//
// Mirrors the role of the reference's REModel facade + REModelTemplate
// (re_model.cpp:21-111, re_model_template.h:95-465) for the in-scope path:
// one GP component, dense ("none") or Vecchia approximation, Gaussian likelihood.
// Host code keeps configuration, the Vecchia structure (built once) and scalar
// assembly; every O(n) / O(n m^2) / O(n^3) step runs in HIP kernels on the model's
// stream. Device buffers are allocated once at construction / SetY and reused.
#pragma once

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <memory>
#include <random>
#include <string>
#include <vector>

#include "collective.h"
#include "common.h"
#include "dense.h"
#include "fitc.h"
#include "dense_laplace.h"
#include "fitc_laplace.h"
#include "vif.h"
#include "vif_laplace.h"
#include "vecchia_fisher.h"
#include "latent.h"
#include "optim.h"

namespace gpb_amd {

struct ModelConfig {
  int n = 0;
  int d = 0;
  std::string cov_fct = "exponential";
  double shape = 0.5;
  int cov_type = 0;
  std::string gp_approx = "none";
  int num_neighbors = 20;
  std::string vecchia_ordering = "random";
  std::string likelihood = "gaussian";
  std::string matrix_inversion_method = "cholesky";
  int seed = 0;
  // FITC (gp_approx = "fitc"): num_ind_points <= 0 -> 500 (re_model_template.h:319-336)
  int num_ind_points = 0;
  double cover_tree_radius = 1.;
  std::string ind_points_selection = "kmeans++";
  // derived
  bool latent = false;     // latent GP + Laplace approximation (non-Gaussian or "vecchia_latent")
  int lik = 0;             // LatentLik code when latent
};

int parse_likelihood(const std::string& name);   // LatentLik code
// cov_fcts.h:438-460: range rho -> phi on the transformed scale
// cov_fcts.h:2753-2770 ParseCovFunctionAlias (+ shape) -> kMatern05 / kMatern15 / kMatern25 / kGaussian
int parse_cov(const std::string& name, double shape);
// FindInitCovPar's initial transformed range (cov_fcts.h:1275-1450): median distance among the points X
// (host row-major n x d), at most 1000 of them drawn uniformly with rng (which continues the caller's
// generator) when n > 1000
double init_range_trafo(const std::vector<double>& X, int d, int cov_type, std::mt19937& rng);
double range_trafo(int cov_type, double rho);
// SUPPORTED_CONV_CRIT_ (re_model_template.h:756-760): true for "relative_change_in_parameters", false for
// "relative_change_in_log_likelihood"; anything else fails
bool check_convergence_criterion(const std::string& name);
// cov_fcts.h TransformBackCovPars: range transform phi -> range rho
double range_back(int cov_type, double phi);

struct EvalResult {
  double nll = 0.;
  double sigma2 = 0.;
  std::vector<double> grad;
};

class REModelAMD {
 public:
  REModelAMD(const ModelConfig& cfg, const double* coords_colmajor);
  ~REModelAMD();

  int num_cov_pars() const { return cfg_.latent ? 2 : 3; }
  int num_aux_pars() const { return (int)aux_pars_.size(); }
  const std::vector<double>& aux_pars() const { return aux_pars_; }
  std::string aux_par_name() const {
    if (!cfg_.latent) return "";
    return cfg_.lik == kLikGaussian ? "error_variance" : (cfg_.lik == kLikGamma ? "shape" : "");
  }
  void SetAuxPars(const double* aux);
  int device() const { return device_; }
  const ModelConfig& config() const { return cfg_; }

  void SetY(const double* y);
  // Stores y as the model's response (GetResponseData) and sets y - fixed_effects (nullable) as the
  // likelihood's response.
  void SetResponse(const double* y, const double* fixed_effects);
  // The response (nullable: keep) and the fixed effects F of one call: Gaussian likelihood: y - F
  // is the response; latent models: F is the offset of the location parameter (mode + F).
  void SetResponseAndOffset(const double* y, const double* fixed_effects);
  // REModel::CalcGradient (re_model.cpp:667-680 -> CalcGradientF re_model_template.h:3021-3043): the
  // gradient of the (approximate marginal) negative log-likelihood wrt F for the GPBoost algorithm,
  // written on y. Gaussian: input y (= F - label), output Psi^-1 y / sigma^2; latent models: y is
  // output only, F = fixed_effects (CalcGradNegMargLikelihoodLaplaceApproxVecchia calc_F_grad,
  // likelihoods.h:5337-5367).
  void CalcGradientF(double* y, const double* fixed_effects, bool calc_cov_factor);
  bool HasY() const { return y_set_; }

  // cov_pars on the original scale. profile: 0 -> include_error_var gradient, 1 -> L-BFGS unit.
  // Latent models: gradient wrt log(cov_pars) (+ log(aux_pars) when estimate_aux_pars).
  EvalResult Eval(const double* cov_pars_orig, bool want_grad, int profile);

  // Prediction settings (GPB_SetPredictionData; vecchia_pred_type null / num_neighbors_pred <= 0:
  // unchanged) and predictions at new coordinates (GPB_PredictREModel): exact Gaussian Vecchia,
  // "order_obs_first_cond_obs_only". coords_pred column-major n_pred x d; cov_pars on the original
  // scale (null: those of the last evaluation); y null: the response already set. out: means, then
  // variances (predict_var) or the n_pred x n_pred covariance (predict_cov_mat; diagonal here).
  void SetPredictionData(const char* vecchia_pred_type, int num_neighbors_pred, int nsim_var_pred = -1);
  // mean_add (nullable, n_pred): fixed effects / linear predictor added to the predictive mean before
  // any response transform.
  void Predict(const double* y, int n_pred, const double* coords_pred, const double* cov_pars, bool predict_cov_mat,
               bool predict_var, bool predict_response, double* out, const double* mean_add = nullptr);

  void SetDistributed(int rank, int world, const ncclUniqueId& id, bool use_comm);
  // Same partition, cross-rank sums through a host function instead of RCCL (test transport).
  void SetDistributedHost(int rank, int world, HostAllReduceFn fn, void* user);

  // Partial sums over rows [r0, r1) of this model's row block, no all-reduce (EXTENSION API).
  void EvalVecchiaPartials(const double* cov_pars_orig, int r0, int r1, double* sums);

  void GetVecchiaStructure(int* perm, int* nbr) const;
  void GetVecchiaFactor(const double* cov_pars_orig, double* Dinv, double* Bvals);
  // Latent factor with range derivatives (EXTENSION, latent models only).
  void GetLatentVecchiaFactor(const double* cov_pars_orig, double* Dinv, double* Bvals, double* dD, double* dBvals);
  // [newton iterations, mode-finding CG iterations, Lanczos steps, log|Sigma W + I|] of the last latent eval
  void GetLastIterationInfo(double* out) const { for (int k = 0; k < 4; ++k) out[k] = last_iter_info_[k]; }
  void CholeskyPlanInfo(double* out);   // GPB_GetCholeskyPlanInfo (latent Vecchia, cholesky)
  void BenchLatentOperators(int t, int reps, double* out);
  void GetLastKernelTimes(double* ms);
  // FITC inducing points (host row-major m x d; EXTENSION: GPB_GetInducingPoints)
  const std::vector<double>& InducingPoints() const;
  bool is_fitc() const { return fitc_ != nullptr; }
  bool is_vif() const { return vif_ != nullptr; }

  double last_nll() const { return last_nll_; }
  const std::vector<double>& last_cov_pars() const { return last_cov_pars_; }

  // Covariance-parameter estimation (GPB_SetOptimConfig / GPB_OptimCovPar / GPB_GetNumIt;
  // re_model.cpp:234-401, optim.cpp). Only the reference's default optimizer "lbfgs".
  void SetOptimSettings(const double* init_cov_pars, double lr, int max_iter, double delta_rel_conv,
                        const char* optimizer, int m_lbfgs);
  // called_in_boosting / reuse_lr: the GPBoost algorithm's call (REModel::OptimCovPar(..., true,
  // reuse_learning_rates_gp_model), regression_objective.hpp:164, 178): the offset is not saved for
  // prediction (re_model_template.h:1051) and the L-BFGS memory of the previous call seeds the first
  // direction when both calls estimated the covariance parameters (:880-881).
  void OptimCovPar(const double* y, const double* fixed_effects, bool called_in_boosting = false,
                   bool reuse_lr = false);
  // the latent mode of the previous objective evaluation back (ResetLaplaceApproxModeToPreviousValue,
  // optim_utils.h:350-360) after a NaN / Inf objective or gradient
  void ResetLatentModeToPrevious();
  // GPB_OptimLinRegrCoefCovPar (re_model.cpp:403-469 -> OptimLinRegrCoefCovPar
  // re_model_template.h:846-1700) for the Gaussian likelihood: covariance parameters by L-BFGS with
  // the nugget profiled out and the coefficients by generalised least squares at every objective
  // evaluation (optimizer_coef "wls", optim_utils.h:297-313; ProfileOutCoef :2427-2445).
  // X column-major n x num_covariates.
  void OptimLinRegrCoefCovPar(const double* y, const double* X, int num_covariates, const double* fixed_effects);
  // GPB_GetCoef (re_model.cpp:836-870): coefficients, then (calc_std_dev) their standard deviations
  // sqrt(diag((X^T Psi^-1 X / sigma^2)^-1)) (CalcStdDevCoef re_model_template.h:9797-9814).
  void GetCoef(double* out, bool calc_std_dev);
  int num_covariates() const { return num_covariates_; }
  bool has_covariates() const { return has_covariates_; }
  // Gaussian residual response y - offset - X beta (original order) of the stored response.
  std::vector<double> ResidualResponse(const double* y, const double* fixed_effects) const;
  // Adds X_pred beta to predictions of a model with covariates (X_pred column-major n_pred x p).
  void AddLinearPredictor(const double* X_pred, int n_pred, double* mu) const;
  // GPB_PredictREModelTrainingDataRandomEffects (re_model.cpp PredictTrainingDataRandomEffects ->
  // re_model_template.h PredictTrainingDataRandomEffects): Gaussian likelihood: mean y - Psi^-1 y and
  // variance sigma^2 (1 - diag(Psi^-1)); latent models: the posterior mode (no variances).
  void PredictTrainingDataRandomEffects(const double* cov_pars, const double* y, double* out,
                                        const double* fixed_effects, bool calc_var);
  // GPB_SetLikelihood (re_model.cpp:142-160, re_model_template.h:558-640)
  void SetLikelihood(const std::string& likelihood);
  // GPB_GetResponseData / GetCovariateData / Get- / SetOffsetData (re_model_template.h:5762-5825)
  void GetResponseData(double* y) const;
  void GetCovariateData(double* X) const;
  void GetOffsetData(double* fe) const;
  void SetOffsetData(const double* fe);
  // GPB_SetOptimConfig's init_aux_pars (re_model.cpp:264-279 -> SetAuxPars): also marks the aux
  // parameters as given (no FindInitialAuxPars at the next fit, re_model_template.h:1186)
  void SetInitAuxPars(const double* aux);
  // optimizer / preconditioner names of GPB_SetOptimConfig (NULL or "": unchanged)
  void SetOptimizerNames(const char* optimizer_cov, const char* optimizer_coef, const char* preconditioner);
  // GPB_GetInitAuxPars (re_model.cpp:1226-1238): -1 each when none were given
  void GetInitAuxPars(double* out) const;
  // GPB_GetOptimizerCovPars / GetOptimizerCoef / GetCGPreconditionerType (re_model.cpp:174-208)
  const std::string& optimizer_cov() const { return optimizer_cov_; }
  const std::string& optimizer_coef() const { return optimizer_coef_; }
  std::string cg_preconditioner_type() const;
  // CanCalculateStandardErrorsCovPars (re_model_template.h:1630-1632)
  bool CanCalculateStandardErrorsCovPars() const { return !cfg_.latent && !vif_; }
  // GLS evaluation on the transformed scale (optimizer): beta from the Gram of [X | y], then the
  // profiled L-BFGS unit on the residuals. beta_out (nullable) receives the coefficients.
  EvalResult EvalTrafoWls(const double* trafo, bool want_grad, bool fatal_on_nan, std::vector<double>* beta_out);
  // Standard deviations of the covariance parameters (original scale) at cov_pars_orig: square
  // roots of the diagonal of the inverse Fisher information (CalcStdDevCovPar,
  // re_model_template.h:9775-9789; dense, Vecchia and FITC Gaussian models).
  void StdDevCovPars(const double* cov_pars_orig, double* sd);
  // Fisher information of the log transformed parameters (Fisher scoring; dense models), 3 x 3 row-major
  std::vector<double> FisherTrafo(const double* trafo);
  // acc_rate_cov, use_nesterov_acc, nesterov_schedule_version, momentum_offset, convergence_criterion of
  // GPB_SetOptimConfig (re_model_template.h:710-761) for the internal optimizers
  // estimate_cov_par_index (re_model_template.h:806-816): a parameter with index <= 0 keeps its initial value.
  // Supported for the Gaussian likelihood with "lbfgs" (zero gradient entries, MaybeKeepVarianceConstant
  // :7104-7121, ProfileOutSigma2 :2407-2412 keeping a fixed nugget).
  void SetEstimateCovParIndex(const std::vector<int>& idx) {
    bool all = true;
    for (int v : idx) all = all && v > 0;
    est_idx_ = all ? std::vector<int>() : idx;
  }
  void SetInternalOptimSettings(double acc_rate, bool nesterov, int schedule, int momentum_offset,
                                const char* convergence_criterion) {
    isettings_.acc_rate = acc_rate;
    isettings_.nesterov = nesterov;
    isettings_.schedule = schedule;
    isettings_.momentum_offset = momentum_offset;
    if (convergence_criterion != nullptr && convergence_criterion[0] != '\0')
      isettings_.crit_params = check_convergence_criterion(convergence_criterion);
  }
  int num_it() const { return num_it_; }
  // GPB_GetInitCovPar (re_model.cpp:813-834): initial values on the original scale, or -1 each
  // when none were given or determined yet
  void GetInitCovPar(double* out) const;

  // Evaluations on the transformed scale (used by the optimizer): Gaussian trafo =
  // (sigma^2, sigma1^2 / sigma^2, phi); latent trafo = (sigma1^2, phi). fatal_on_nan = false
  // returns a NaN / Inf objective instead of failing (the line search shrinks the step).
  EvalResult EvalTrafo(const double* trafo, bool want_grad, int profile, bool fatal_on_nan = true);
  EvalResult EvalLatentTrafo(const double* trafo, bool want_grad, bool fatal_on_nan = true,
                             LatentVecchia::ModeStart start = LatentVecchia::ModeStart::kZero);

  // iterative-method settings (GPB_SetOptimConfig, re_model_template.h:686-823)
  IterativeConfig iter;
  bool estimate_aux_pars = true;   // InitializeDefaultSettings (re_model_template.h:6492-6499) for latent models
  bool aux_pars_set_ = false;      // aux_pars given by the caller (SetOptimConfig init_aux_pars / SetAuxPars)

  // REModel::InitializeCovParsIfNotDefined: init_cov_pars or FindInitCovPar on y - F (latent: the
  // stored response); current_cov_pars() = the parameters an evaluation with cov_pars == NULL uses.
  void InitCovParsIfNotDefined(const double* y, const double* fixed_effects);
  const std::vector<double>& current_cov_pars() const { return cov_pars_orig_; }

  // Latent models: the fixed effects F (location offset) of the next mode finding (NULL: none).
  void SetLatentOffset(const double* fe);
  // The offset a prediction uses: the given one, else the one saved by the last fit (re_model_template.h:3306-3312).
  const double* ResolveOffset(const double* fe) const {
    return fe != nullptr ? fe : (has_fixed_effects_ ? fixed_effects_.data() : nullptr);
  }

 private:
  void TransformCovPars(const double* orig, double* trafo) const;
  void PredictPredFirst(int n_pred, const double* coords_pred, const double* trafo, bool predict_cov_mat,
                        bool predict_var, bool predict_response, double* out, const double* mean_add);
  void PredictLatentGaussian(int n_pred, const double* coords_pred, const double* trafo, bool predict_cov_mat,
                             bool predict_var, bool predict_response, double* out, const double* mean_add);
  void PredictLatentSim(int n, int n_pred, int mp, const std::vector<int>& nb, const double* dB, const double* dDinv,
                        bool cond_all, bool predict_cov_mat, bool predict_var, bool predict_response, double* out,
                        const double* mean_add);
  void PredictDense(const double* y, int n_pred, const double* coords_pred, const double* cov_pars, bool predict_cov_mat,
                    bool predict_var, bool predict_response, double* out, const double* mean_add);
  void PredictDenseLaplace(const double* y, int n_pred, const double* coords_pred, const double* cov_pars,
                           bool predict_cov_mat, bool predict_var, bool predict_response, double* out,
                           const double* mean_add);
  void PredictVif(const double* y, int n_pred, const double* coords_pred, const double* cov_pars, bool predict_cov_mat,
                  bool predict_var, bool predict_response, double* out, const double* mean_add);
  void PredictVifLaplace(const double* y, int n_pred, const double* coords_pred, const double* cov_pars, bool predict_cov_mat,
                  bool predict_var, bool predict_response, double* out, const double* mean_add);
  void PredictFitc(const double* y, int n_pred, const double* coords_pred, const double* cov_pars, bool predict_cov_mat,
                   bool predict_var, bool predict_response, double* out, const double* mean_add);
  std::vector<int> FitcMatch(const std::vector<double>& xp_rowmajor, int n_pred) const;
  void ResponseTransform(int n_pred, double* mean, double* var, double* cov);
  void PredictFitcLaplace(const double* y, int n_pred, const double* coords_pred, const double* cov_pars,
                          bool predict_cov_mat, bool predict_var, bool predict_response, double* out,
                          const double* mean_add);
  void PredictCondAll(int n, int n_pred, int mp, const std::vector<int>& nb, const double* dB, const double* dDinv,
                      double sigma2, double nugget_sub, bool want_var, bool want_cov, std::vector<double>& h,
                      std::vector<double>& cov);
  double range_trafo_of(double rho) const { return range_trafo(cfg_.cov_type, rho); }
  void FindInitCovPar(const double* y, double* trafo) const;
  double InitialRangeTrafo() const;
  void BuildVecchiaStructure();
  void EvalVecchia(const double* trafo, double* sums);  // sums over this rank's rows, all-reduced
  void LaunchVecchiaRows(const double* trafo, int r0, int r1, double* sums_host, bool allreduce);
  void EvalDense(const double* trafo, bool want_grad, double* sums);
  // "none" and "fitc" share the Gaussian Cholesky bookkeeping (dense_ or fitc_)
  void EvalExactGaussian(const double* trafo, bool want_grad, double* sums);

  void EnsureStructure();
  void UseDevice() const;
  EvalResult EvalLatent(const double* cov_pars_orig, bool want_grad);

  ModelConfig cfg_;
  int device_ = 0;
  bool vecchia_ = false;
  bool structure_built_ = false;
  std::vector<double> coords_;       // row-major n x d, original order
  std::vector<double> coords_vo_;    // Vecchia order (Vecchia) / original (dense); latent: the unique locations
  int nu_ = 0;                       // latent dimension (unique locations of a latent model, else n)
  std::vector<int> obs_row_;         // latent models with repeated coordinates: observation (Vecchia-shuffled order) -> latent row
  bool has_dup() const { return !obs_row_.empty(); }
  std::vector<int> perm_;
  std::vector<int> nbr_;             // rows [row_begin_, row_end_) x m, or all rows when world == 1
  int nbr_row0_ = 0;
  bool y_set_ = false;

  hipStream_t stream_ = nullptr;
  hipEvent_t ev_[3] = {nullptr, nullptr, nullptr};
  DevBuf<double> d_X_, d_y_, d_block_sums_, d_sums_;
  DevBuf<int> d_nbr_;
  double* h_sums_ = nullptr;  // pinned
  double* h_sums_dev_ = nullptr;  // device address of h_sums_ (the single-rank sum kernel writes it directly)
  unsigned long long sum_seq_ = 0;  // completion flag value of the last single-rank evaluation (h_sums_[8])
  bool events_pending_ = false;   // last_kernel_ms_ of the last row launch not read from its events yet
  bool timing_ = false;           // record kernel events (set by the first GetLastKernelTimes)

  std::unique_ptr<DenseSolver> dense_;
  std::unique_ptr<FitcSolver> fitc_;   // gp_approx = "fitc"
  std::unique_ptr<FitcLaplace> fitc_lap_;   // gp_approx = "fitc", non-Gaussian likelihood (Laplace)
  std::unique_ptr<DenseLaplace> dense_lap_; // gp_approx = "none", non-Gaussian likelihood (Laplace)
  double sum_log_y_ = 0.;                   // likelihood 'gamma': sum log y (its normalizing constant)
  std::vector<int> est_idx_;                // estimate_cov_par_index (empty: all estimated)
  std::unique_ptr<VifSolver> vif_;          // gp_approx = "full_scale_vecchia"
  std::unique_ptr<VifLaplace> vif_lap_;     // gp_approx = "full_scale_vecchia", non-Gaussian likelihood (Laplace)
  std::vector<int> vif_nbr_;                // the full-scale Vecchia neighbour lists (host, model order)
  std::unique_ptr<VecchiaFisher> vfisher_;  // gp_approx = "vecchia", Gaussian: standard deviations (lazy)
  std::mt19937 fitc_rng_;              // the model's generator after the inducing-point selection
  std::mt19937 pred_ref_gen_;          // the likelihood's cg_generator_ (default seed) for reference draws
  std::mt19937* RefDraws();
  std::unique_ptr<LatentVecchia> latent_;
  // the latent solver of a Laplace model: the Vecchia (iterative) or the FITC (Cholesky) one
  LatentSolverBase* lat() const {
    if (latent_) return latent_.get();
    if (dense_lap_) return dense_lap_.get();
    if (vif_lap_) return vif_lap_.get();
    return fitc_lap_.get();
  }
  std::vector<double> y_vo_;          // host copy (Vecchia order) for the latent solver
  std::vector<double> aux_pars_;
  double loglik_const_ = 0.;          // the latent likelihood's normalizing constant at the current y
  double last_iter_info_[4] = {0., 0., 0., 0.};
  int test_nan_count_ = 0;   // latent evaluations seen by the GPBOOST_AMD_TEST_NAN_EVAL fault injection

  std::string vecchia_pred_type_ = "order_obs_first_cond_obs_only";   // re_model_template.h:6485-6490
  int num_neighbors_pred_ = 0;                                         // 2 num_neighbors (:299)
  int nsim_var_pred_ = 1000;                                           // re_model_template.h:5374
  uint64_t pred_seed_ = 1;                                             // latent variance draws (per call)

  int rank_ = 0, world_ = 1;
  int row_begin_ = 0, row_end_ = 0;
  ncclComm_t comm_ = nullptr;
  std::unique_ptr<Collective> coll_;   // RCCL (comm_) or host-callback sums; null = single rank
  void ApplyPartition(int rank, int world);

  double last_nll_ = 0.;
  std::vector<double> last_cov_pars_;
  double last_kernel_ms_[2] = {0., 0.};

  // covariates (OptimLinRegrCoefCovPar) and stored data
  void InitializeOptimizerNames();
  std::vector<double> Gram(const double* trafo);   // c x c Gram of [X | y - offset] (c = p + 1)
  void UploadCovariates();
  void EnsureTransposedLists();                     // exact Vecchia: B^T lists for the training predictions
  void PsiInvVecchia(const double* trafo, double* yaux, double* diag);
  std::vector<double> X_cov_;        // column-major n x p (original order)
  std::vector<double> coef_;
  int num_covariates_ = 0;
  bool has_covariates_ = false;
  bool coef_std_dev_valid_ = false;
  std::vector<double> coef_std_dev_;
  std::vector<double> y_raw_;        // response as last given (original order, offset not subtracted)
  std::vector<double> fixed_effects_;
  bool has_fixed_effects_ = false;
  std::vector<double> offset_vo_;     // latent models: fixed effects F of the last call (Vecchia order)
  bool has_offset_ = false;
  DevBuf<double> d_Zcov_;            // [X | y - offset], Vecchia order row-major n x c (Vecchia models)
  DevBuf<double> d_Bf_, d_Df_, d_gram_part_, d_gram_out_;
  DevBuf<int> d_tptr_, d_trow_, d_tslot_;
  std::string optimizer_cov_, optimizer_coef_;
  InternalSettings isettings_;   // "gradient_descent" / "fisher_scoring" (optimizer empty: lbfgs)
  std::string cg_preconditioner_type_;
  std::vector<double> init_aux_pars_;   // given by GPB_SetOptimConfig (original scale)

  LbfgsSettings optim_;
  std::vector<double> init_cov_pars_, cov_pars_orig_, init_used_;   // original scale
  bool cov_pars_initialized_ = false;
  int num_it_ = 0;
  InverseHessian m_bfgs_;                 // REModelTemplate::m_bfgs_ (GetMBFGS), kept across OptimCovPar calls
  bool cov_est_once_ = false;             // cov_pars_have_been_estimated_once_ (re_model_template.h:5301)
  bool cov_est_last_call_ = false;        // cov_pars_have_been_estimated_during_last_call_ (:5303)
  bool latent_evaluated_ = false;         // the latent state (factor, mode) holds a finished evaluation
};

}  // namespace gpb_amd
