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
#include <string>
#include <vector>

#include "collective.h"
#include "common.h"
#include "dense.h"
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
  // derived
  bool latent = false;     // latent GP + Laplace approximation (non-Gaussian or "vecchia_latent")
  int lik = 0;             // LatentLik code when latent
};

// cov_fcts.h:438-460: range rho -> phi on the transformed scale
double range_trafo(int cov_type, double rho);

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
  std::string aux_par_name() const { return cfg_.latent && cfg_.lik == kLikGaussian ? "error_variance" : ""; }
  void SetAuxPars(const double* aux);
  int device() const { return device_; }
  const ModelConfig& config() const { return cfg_; }

  void SetY(const double* y);
  bool HasY() const { return y_set_; }

  // cov_pars on the original scale. profile: 0 -> include_error_var gradient, 1 -> L-BFGS unit.
  // Latent models: gradient wrt log(cov_pars) (+ log(aux_pars) when estimate_aux_pars).
  EvalResult Eval(const double* cov_pars_orig, bool want_grad, int profile);

  // Prediction settings (GPB_SetPredictionData; vecchia_pred_type null / num_neighbors_pred <= 0:
  // unchanged) and predictions at new coordinates (GPB_PredictREModel): exact Gaussian Vecchia,
  // "order_obs_first_cond_obs_only". coords_pred column-major n_pred x d; cov_pars on the original
  // scale (null: those of the last evaluation); y null: the response already set. out: means, then
  // variances (predict_var) or the n_pred x n_pred covariance (predict_cov_mat; diagonal here).
  void SetPredictionData(const char* vecchia_pred_type, int num_neighbors_pred);
  void Predict(const double* y, int n_pred, const double* coords_pred, const double* cov_pars, bool predict_cov_mat,
               bool predict_var, bool predict_response, double* out);

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
  void BenchLatentOperators(int t, int reps, double* out);
  void GetLastKernelTimes(double* ms);

  double last_nll() const { return last_nll_; }
  const std::vector<double>& last_cov_pars() const { return last_cov_pars_; }

  // Covariance-parameter estimation (GPB_SetOptimConfig / GPB_OptimCovPar / GPB_GetNumIt;
  // re_model.cpp:234-401, optim.cpp). Only the reference's default optimizer "lbfgs".
  void SetOptimSettings(const double* init_cov_pars, double lr, int max_iter, double delta_rel_conv,
                        const char* optimizer, int m_lbfgs);
  void OptimCovPar(const double* y, const double* fixed_effects);
  // Standard deviations of the covariance parameters (original scale) at cov_pars_orig: square
  // roots of the diagonal of the inverse Fisher information (CalcStdDevCovPar,
  // re_model_template.h:9775-9789; dense Gaussian models only).
  void StdDevCovPars(const double* cov_pars_orig, double* sd);
  int num_it() const { return num_it_; }
  // GPB_GetInitCovPar (re_model.cpp:813-834): initial values on the original scale, or -1 each
  // when none were given or determined yet
  void GetInitCovPar(double* out) const;

  // Evaluations on the transformed scale (used by the optimizer): Gaussian trafo =
  // (sigma^2, sigma1^2 / sigma^2, phi); latent trafo = (sigma1^2, phi). fatal_on_nan = false
  // returns a NaN / Inf objective instead of failing (the line search shrinks the step).
  EvalResult EvalTrafo(const double* trafo, bool want_grad, int profile, bool fatal_on_nan = true);
  EvalResult EvalLatentTrafo(const double* trafo, bool want_grad, bool fatal_on_nan = true);

  // iterative-method settings (GPB_SetOptimConfig, re_model_template.h:686-823)
  IterativeConfig iter;
  bool estimate_aux_pars = true;   // InitializeDefaultSettings (re_model_template.h:6492-6499) for latent models
  bool aux_pars_set_ = false;      // aux_pars given by the caller (SetOptimConfig init_aux_pars / SetAuxPars)

 private:
  void TransformCovPars(const double* orig, double* trafo) const;
  double range_trafo_of(double rho) const { return range_trafo(cfg_.cov_type, rho); }
  void FindInitCovPar(const double* y, double* trafo) const;
  double InitialRangeTrafo() const;
  void BuildVecchiaStructure();
  void EvalVecchia(const double* trafo, double* sums);  // sums over this rank's rows, all-reduced
  void LaunchVecchiaRows(const double* trafo, int r0, int r1, double* sums_host, bool allreduce);
  void EvalDense(const double* trafo, bool want_grad, double* sums);

  void EnsureStructure();
  void UseDevice() const;
  EvalResult EvalLatent(const double* cov_pars_orig, bool want_grad);

  ModelConfig cfg_;
  int device_ = 0;
  bool vecchia_ = false;
  bool structure_built_ = false;
  std::vector<double> coords_;       // row-major n x d, original order
  std::vector<double> coords_vo_;    // Vecchia order (Vecchia) / original (dense)
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
  bool events_pending_ = false;   // last_kernel_ms_ of the last row launch not read from its events yet
  bool timing_ = false;           // record kernel events (set by the first GetLastKernelTimes)

  std::unique_ptr<DenseSolver> dense_;
  std::unique_ptr<LatentVecchia> latent_;
  std::vector<double> y_vo_;          // host copy (Vecchia order) for the latent solver
  std::vector<double> aux_pars_;
  double last_iter_info_[4] = {0., 0., 0., 0.};

  std::string vecchia_pred_type_ = "order_obs_first_cond_obs_only";   // re_model_template.h:6485-6490
  int num_neighbors_pred_ = 0;                                         // 2 num_neighbors (:299)

  int rank_ = 0, world_ = 1;
  int row_begin_ = 0, row_end_ = 0;
  ncclComm_t comm_ = nullptr;
  std::unique_ptr<Collective> coll_;   // RCCL (comm_) or host-callback sums; null = single rank
  void ApplyPartition(int rank, int world);

  double last_nll_ = 0.;
  std::vector<double> last_cov_pars_;
  double last_kernel_ms_[2] = {0., 0.};

  LbfgsSettings optim_;
  std::vector<double> init_cov_pars_, cov_pars_orig_, init_used_;   // original scale
  bool cov_pars_initialized_ = false;
  int num_it_ = 0;
};

}  // namespace gpb_amd
