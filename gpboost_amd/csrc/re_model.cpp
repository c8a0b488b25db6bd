// REModelAMD implementation (host orchestration; all heavy math in HIP kernels).
#include "re_model.h"

#include <algorithm>
#include <numeric>
#include <atomic>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <limits>

#include "cov.h"
#include "kernels.h"
#include "latent_kernels.h"
#include "vecchia_host.h"

namespace gpb_amd {

// likelihood names of the Laplace paths (likelihoods.h:12656 SUPPORTED_LIKELIHOODS_, the subset built here)
int parse_likelihood(const std::string& name) {
  if (name == "gaussian") return kLikGaussian;
  if (name == "bernoulli_logit") return kLikBernoulliLogit;
  if (name == "bernoulli_probit") return kLikBernoulliProbit;
  if (name == "poisson") return kLikPoisson;
  if (name == "gamma") return kLikGamma;
  Fatal("likelihood '%s' is not supported by gpboost_amd (supported: gaussian, bernoulli_logit, bernoulli_probit, poisson, "
        "gamma)", name.c_str());
  return -1;
}

int parse_cov(const std::string& name, double shape) {
  // cov_fcts.h:2753-2770 ParseCovFunctionAlias; :170-183 shape handling
  auto eq = [](double a, double b) { return std::fabs(a - b) < 1e-10; };
  if (name == "exponential" || name == "Matern") return kMatern05;
  if (name == "matern") {
    if (eq(shape, 0.5)) return kMatern05;
    if (eq(shape, 1.5)) return kMatern15;
    if (eq(shape, 2.5)) return kMatern25;
    Fatal("cov_fct 'matern' with shape %g is not supported by gpboost_amd (supported: 0.5, 1.5, 2.5)", shape);
  }
  if (name == "gaussian" || name == "Gaussian") return kGaussian;
  Fatal("cov_fct '%s' is not supported by gpboost_amd (supported: exponential, matern, gaussian)", name.c_str());
}

bool check_convergence_criterion(const std::string& name) {
  if (name == "relative_change_in_parameters") return true;
  if (name == "relative_change_in_log_likelihood") return false;
  Fatal("Convergence criterion '%s' is not supported.", name.c_str());
  return false;
}

double range_trafo(int cov_type, double rho) {
  switch (cov_type) {
    case kMatern05: return 1. / rho;
    case kMatern15: return std::sqrt(3.) / rho;
    case kMatern25: return std::sqrt(5.) / rho;
    default: return 1. / (rho * rho);
  }
}

double range_back(int cov_type, double phi) {
  switch (cov_type) {
    case kMatern05: return 1. / phi;
    case kMatern15: return std::sqrt(3.) / phi;
    case kMatern25: return std::sqrt(5.) / phi;
    default: return 1. / std::sqrt(phi);
  }
}

REModelAMD::REModelAMD(const ModelConfig& cfg, const double* coords_colmajor) : cfg_(cfg) {
  if (cfg_.n <= 0) Fatal("num_data must be > 0");
  if (cfg_.d <= 0 || cfg_.d > 3) Fatal("dim_gp_coords = %d not supported (1..3)", cfg_.d);
  cfg_.cov_type = parse_cov(cfg_.cov_fct, cfg_.shape);
  // likelihood and approximation (re_model_template.h:207-211, 563; likelihoods.h:240-257)
  cfg_.lik = parse_likelihood(cfg_.likelihood);
  if (cfg_.gp_approx == "vecchia_latent") {
    vecchia_ = true;
    cfg_.latent = true;
  } else if (cfg_.gp_approx == "vecchia") {
    vecchia_ = true;
    cfg_.latent = cfg_.lik != kLikGaussian;
  } else if (cfg_.gp_approx == "none") {
    cfg_.latent = cfg_.lik != kLikGaussian;   // Laplace approximation (DenseLaplace)
    if (cfg_.latent && cfg_.matrix_inversion_method == "iterative")   // CanUseIterative, re_model_template.h:6712-6717
      Fatal("matrix_inversion_method = 'iterative' is not supported for gp_approx = 'none' with likelihood '%s'. Use 'cholesky' ",
            cfg_.likelihood.c_str());
  } else if (cfg_.gp_approx == "fitc") {
    cfg_.latent = cfg_.lik != kLikGaussian;   // Laplace approximation (FitcLaplace)
    if (cfg_.matrix_inversion_method == "iterative")   // re_model_template.h:8774-8776
      Fatal("'iterative' methods are not implemented for gp_approx = 'fitc'. Use 'cholesky' ");
    if (cfg_.num_ind_points <= 0) cfg_.num_ind_points = 500;   // re_model_template.h:320-326
    if (!(cfg_.cover_tree_radius > 0.)) Fatal("cover_tree_radius must be > 0");
  } else if (cfg_.gp_approx == "full_scale_vecchia" || cfg_.gp_approx == "vif" || cfg_.gp_approx == "VIF") {
    cfg_.gp_approx = "full_scale_vecchia";   // re_model_template.h:204-206
    cfg_.latent = cfg_.lik != kLikGaussian;   // Laplace approximation (VifLaplace, the reference's FSVA)
    if (!cfg_.latent && cfg_.matrix_inversion_method == "iterative")   // re_model_template.h:8780-8782
      Fatal("The iterative methods are not implemented for the Full-Scale-Vecchia approximation with Gaussian "
            "likelihood. Please use Cholesky.");
    // non-Gaussian: the reference's default is "iterative" (PCG + SLQ with the FITC preconditioner,
    // re_model_template.h:6719-6723); this build runs the exact Cholesky branch for "default" and "cholesky"
    if (cfg_.latent && cfg_.matrix_inversion_method == "iterative")
      Fatal("matrix_inversion_method = 'iterative' for gp_approx = 'full_scale_vecchia' with likelihood '%s' is not "
            "supported by gpboost_amd (supported: cholesky)", cfg_.likelihood.c_str());
    if (cfg_.latent && cfg_.ind_points_selection == "random")   // the reference's FSVA component construction
      Fatal("Method 'random' is not supported for finding inducing points in the full-scale-vecchia approximation "
            "for non-Gaussian data");
    if (cfg_.num_ind_points <= 0) cfg_.num_ind_points = 200;   // re_model_template.h:320-330
    if (cfg_.num_neighbors <= 0) cfg_.num_neighbors = 30;      // :288-297
    if (!(cfg_.cover_tree_radius > 0.)) Fatal("cover_tree_radius must be > 0");
  } else {
    Fatal("gp_approx '%s' is not supported by gpboost_amd (supported: none, vecchia, vecchia_latent, fitc, "
          "full_scale_vecchia)", cfg_.gp_approx.c_str());
  }
  std::string& mim = cfg_.matrix_inversion_method;
  if (mim == "default") mim = cfg_.latent && vecchia_ ? "iterative" : "cholesky";
  if (cfg_.latent && vecchia_ && mim != "iterative" && mim != "cholesky")
    Fatal("matrix_inversion_method '%s' is not supported for latent Vecchia models in gpboost_amd (supported: iterative, "
          "cholesky)", mim.c_str());
  if (!(cfg_.latent && vecchia_) && mim != "cholesky")
    Fatal("matrix_inversion_method '%s' is not supported for likelihood 'gaussian' in gpboost_amd (supported: cholesky)", mim.c_str());
  if (cfg_.latent && (cfg_.lik == kLikGaussian || cfg_.lik == kLikGamma))
    aux_pars_ = {1.};   // likelihoods.h:241 (error_variance), :181-186 (gamma shape)
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
    Fatal("no HIP device visible: gpboost_amd has no CPU fallback");
  // The reference ABI has no device argument (c_api.h:1351 only has GPU_use): the device is
  // GPBOOST_AMD_DEVICE if set (one process per GPU), else the calling thread's current device.
  if (const char* dev = std::getenv("GPBOOST_AMD_DEVICE")) {
    device_ = std::atoi(dev);
    if (device_ < 0 || device_ >= ndev) Fatal("GPBOOST_AMD_DEVICE=%d but %d device(s) visible", device_, ndev);
  } else {
    HIP_CHECK(hipGetDevice(&device_));
  }
  UseDevice();

  const int n = cfg_.n, d = cfg_.d;
  coords_.resize((size_t)n * d);
  for (int i = 0; i < n; ++i)
    for (int q = 0; q < d; ++q) coords_[(size_t)i * d + q] = coords_colmajor[(size_t)q * n + i];

  HIP_CHECK(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));
  for (auto& e : ev_) HIP_CHECK(hipEventCreate(&e));
  // host-coherent: the single-rank block sum writes the result and a completion flag here directly
  HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&h_sums_), 16 * sizeof(double),
                          hipHostMallocMapped | hipHostMallocCoherent));
  std::fill(h_sums_, h_sums_ + 16, 0.);
  HIP_CHECK(hipHostGetDevicePointer(reinterpret_cast<void**>(&h_sums_dev_), h_sums_, 0));
  row_begin_ = 0;
  row_end_ = n;
  num_neighbors_pred_ = 2 * cfg_.num_neighbors;   // re_model_template.h:299
  nu_ = n;
  if (vecchia_) {
    perm_ = vecchia_order(n, cfg_.seed, cfg_.vecchia_ordering == "random");
    if (cfg_.vecchia_ordering != "random" && cfg_.vecchia_ordering != "none")
      Fatal("vecchia_ordering '%s' is not supported (supported: none, random)", cfg_.vecchia_ordering.c_str());
    coords_vo_.resize((size_t)n * d);
    for (int i = 0; i < n; ++i)
      for (int q = 0; q < d; ++q) coords_vo_[(size_t)i * d + q] = coords_[(size_t)perm_[i] * d + q];
    if (cfg_.latent) {
      // Latent GPs live on the UNIQUE locations (RECompGP on unique coordinates with an incidence
      // matrix, Vecchia_utils.cpp:1121-1139, re_comp.h:845-870; only_one_GP_calculations_on_RE_scale):
      // unique points in order of first appearance in the shuffled order, the Vecchia structure
      // over them, every observation mapped to its location's latent variable.
      std::vector<int> uniq, idx;
      unique_locations(coords_vo_.data(), n, d, uniq, idx);
      if ((int)uniq.size() < n) {
        nu_ = (int)uniq.size();
        obs_row_ = idx;
        std::vector<double> xu((size_t)nu_ * d);
        for (int u = 0; u < nu_; ++u)
          for (int q = 0; q < d; ++q) xu[(size_t)u * d + q] = coords_vo_[(size_t)uniq[u] * d + q];
        coords_vo_.swap(xu);
      }
      row_end_ = nu_;
    }
    if (cfg_.num_neighbors > nu_ - 1) cfg_.num_neighbors = nu_ - 1;  // Vecchia_utils.cpp:754-757
    if (cfg_.num_neighbors < 1) Fatal("num_neighbors must be >= 1");
    d_X_.alloc((size_t)nu_ * d);
    HIP_CHECK(hipMemcpyAsync(d_X_.get(), coords_vo_.data(), sizeof(double) * nu_ * d, hipMemcpyHostToDevice, stream_));
    // neighbour search is deferred to first use so a distributed model searches only its rows
  } else if (cfg_.gp_approx == "full_scale_vecchia") {
    // re_model_template.h:348-357: rng_ = mt19937(seed) shuffles the order first (random ordering), then
    // CreateREComponentsFITC_FSA selects the inducing points on the coordinates in that order with the same
    // generator; the Vecchia neighbours (Euclidean, vecchia_neighbor_selection = "nearest") follow
    if (cfg_.vecchia_ordering != "random" && cfg_.vecchia_ordering != "none")
      Fatal("vecchia_ordering '%s' is not supported (supported: none, random)", cfg_.vecchia_ordering.c_str());
    std::mt19937 rng((std::mt19937::result_type)cfg_.seed);
    perm_.resize(n);
    std::iota(perm_.begin(), perm_.end(), 0);
    if (cfg_.vecchia_ordering == "random") std::shuffle(perm_.begin(), perm_.end(), rng);
    coords_vo_.resize((size_t)n * d);
    for (int i = 0; i < n; ++i)
      for (int q = 0; q < d; ++q) coords_vo_[(size_t)i * d + q] = coords_[(size_t)perm_[i] * d + q];
    std::vector<int> uniq, idx;
    unique_locations(coords_vo_.data(), n, d, uniq, idx);
    if ((int)uniq.size() < n)
      Fatal("gp_approx = 'full_scale_vecchia' with duplicate coordinates is not supported by gpboost_amd");
    const std::vector<double> Z =
        fitc_inducing_points(coords_vo_, n, d, cfg_.num_ind_points, cfg_.ind_points_selection, rng, stream_);
    std::vector<int> zu, zi;
    unique_locations(Z.data(), cfg_.num_ind_points, d, zu, zi);
    if ((int)zu.size() < cfg_.num_ind_points) Fatal("Duplicates found in inducing points / low-dimensional knots ");
    fitc_rng_ = rng;
    if (cfg_.num_neighbors > n - 1) cfg_.num_neighbors = n - 1;   // Vecchia_utils.cpp:754-757
    if (cfg_.num_neighbors < 1) Fatal("num_neighbors must be >= 1");
    const int m = cfg_.num_neighbors;
    std::vector<int> nbr((size_t)n * m, -1);
    if (m > 64 || d > 3) vecchia_neighbors(coords_vo_.data(), n, d, m, 0, n, nbr.data());
    else vecchia_neighbors_gpu(coords_vo_.data(), n, d, m, 0, n, nbr.data(), stream_);
    d_X_.alloc((size_t)n * d);
    HIP_CHECK(hipMemcpyAsync(d_X_.get(), coords_vo_.data(), sizeof(double) * n * d, hipMemcpyHostToDevice, stream_));
    vif_.reset(new VifSolver(n, d, d_X_.get(), Z, nbr, m, stream_));
    vif_nbr_ = nbr;
    if (cfg_.latent) vif_lap_.reset(new VifLaplace(vif_.get(), nbr, coords_vo_, stream_));
  } else {
    coords_vo_ = coords_;
    d_X_.alloc((size_t)n * d);
    HIP_CHECK(hipMemcpyAsync(d_X_.get(), coords_.data(), sizeof(double) * n * d, hipMemcpyHostToDevice, stream_));
    if (cfg_.gp_approx == "fitc") {
      // inducing points on the unique locations (CreateREComponentsFITC_FSA, re_model_template.h:6946-7073);
      // with repeated coordinates the reference switches to 'full_scale_tapering' (:6963-6969), out of scope
      std::vector<int> uniq, idx;
      unique_locations(coords_.data(), n, d, uniq, idx);
      if ((int)uniq.size() < n)
        Fatal("gp_approx = 'fitc' with duplicate coordinates is not supported by gpboost_amd (the reference switches to "
              "'full_scale_tapering')");
      std::mt19937 rng((std::mt19937::result_type)cfg_.seed);   // rng_ = RNG_t(seed) (re_model_template.h:154)
      const std::vector<double> Z =
          fitc_inducing_points(coords_, n, d, cfg_.num_ind_points, cfg_.ind_points_selection, rng, stream_);
      std::vector<int> zu, zi;
      unique_locations(Z.data(), cfg_.num_ind_points, d, zu, zi);
      if ((int)zu.size() < cfg_.num_ind_points) Fatal("Duplicates found in inducing points / low-dimensional knots ");
      fitc_.reset(new FitcSolver(n, d, d_X_.get(), Z, stream_));
      fitc_rng_ = rng;
      if (cfg_.latent) {   // FindModePostRandEffCalcMLLFITC / CalcGradNegMargLikelihoodLaplaceApproxFITC
        fitc_lap_.reset(new FitcLaplace(fitc_.get(), stream_));
        perm_.resize(n);   // no reordering: the model order is the data order
        std::iota(perm_.begin(), perm_.end(), 0);
      }
    } else if (cfg_.latent) {
      // FindModePostRandEffCalcMLLStable / CalcGradNegMargLikelihoodLaplaceApproxStable on the distinct locations;
      // repeated coordinates (the reference's incidence-matrix form) are not supported here
      std::vector<int> uniq, idx;
      unique_locations(coords_.data(), n, d, uniq, idx);
      if ((int)uniq.size() < n)
        Fatal("gp_approx = 'none' with likelihood '%s' and duplicate coordinates is not supported by gpboost_amd",
              cfg_.likelihood.c_str());
      dense_lap_.reset(new DenseLaplace(n, d, d_X_.get(), stream_));
      perm_.resize(n);   // no reordering: the model order is the data order
      std::iota(perm_.begin(), perm_.end(), 0);
    } else {
      dense_.reset(new DenseSolver(n, d, d_X_.get(), stream_));
    }
  }
  d_sums_.alloc(16);
  HIP_CHECK(hipStreamSynchronize(stream_));
}

void REModelAMD::UseDevice() const { HIP_CHECK(hipSetDevice(device_)); }

// GPBOOST_AMD_PRED_DRAWS=reference: the predictive-variance simulation of Laplace models draws the
// reference's own one-thread stream (the likelihood's default-seeded cg_generator_, likelihoods.h:6668-6700)
// on the host, so results equal the reference run with one thread; default: counter-based GPU draws.
std::mt19937* REModelAMD::RefDraws() {
  const char* e = std::getenv("GPBOOST_AMD_PRED_DRAWS");
  return e != nullptr && std::string(e) == "reference" ? &pred_ref_gen_ : nullptr;
}

void REModelAMD::EnsureStructure() {
  if (vecchia_ && !structure_built_) {
    BuildVecchiaStructure();
    if (cfg_.latent) {
      latent_.reset(new LatentVecchia(nu_, cfg_.d, cfg_.num_neighbors, d_X_.get(), nbr_.data(), stream_));
      latent_->SetCholesky(cfg_.matrix_inversion_method == "cholesky");   // likelihoods.h:2935-2955 vs :2925-2934
      if (has_dup()) latent_->SetObservations(obs_row_);
      latent_->SetShard(rank_, world_, coll_.get());   // probe columns over the ranks (§8e Option A)
      latent_->SetLogLikConst(loglik_const_);
      if (y_set_) latent_->SetY(y_vo_.data());
      latent_->SetOffset(has_offset_ ? offset_vo_.data() : nullptr);
    }
    structure_built_ = true;
  }
}

void REModelAMD::SetAuxPars(const double* aux) {
  for (size_t k = 0; k < aux_pars_.size(); ++k) {
    if (!(aux[k] > 0.)) Fatal("aux_pars must be > 0");
    aux_pars_[k] = aux[k];
  }
}

REModelAMD::~REModelAMD() {
  (void)hipSetDevice(device_);
  if (stream_) (void)hipStreamSynchronize(stream_);
  dense_.reset();
  dense_lap_.reset();
  vfisher_.reset();
  vif_lap_.reset();
  vif_.reset();
  fitc_lap_.reset();
  fitc_.reset();
  latent_.reset();
  coll_.reset();
  if (comm_) ncclCommDestroy(comm_);
  if (h_sums_) (void)hipHostFree(h_sums_);
  for (auto& e : ev_) if (e) (void)hipEventDestroy(e);
  if (stream_) (void)hipStreamDestroy(stream_);
}

void REModelAMD::BuildVecchiaStructure() {
  const int n = cfg_.latent ? nu_ : cfg_.n, m = cfg_.num_neighbors;   // latent: the unique locations
  // Only this rank's rows are needed on the device (each row's neighbours are earlier points).
  nbr_.assign((size_t)(row_end_ - row_begin_) * m, -1);
  nbr_row0_ = row_begin_;
  static const bool host_knn = std::getenv("GPBOOST_AMD_HOST_KNN") != nullptr;   // A/B: host OpenMP search
  if (host_knn || m > 64 || cfg_.d > 3)
    vecchia_neighbors(coords_vo_.data(), n, cfg_.d, m, row_begin_, row_end_, nbr_.data());
  else
    vecchia_neighbors_gpu(coords_vo_.data(), n, cfg_.d, m, row_begin_, row_end_, nbr_.data(), stream_);
  // Device copy laid out by global row index (rows outside this rank's block untouched).
  d_nbr_.alloc((size_t)n * m);
  HIP_CHECK(hipMemcpyAsync(d_nbr_.get() + (size_t)row_begin_ * m, nbr_.data(), sizeof(int) * nbr_.size(),
                           hipMemcpyHostToDevice, stream_));
  if (!cfg_.latent) {   // the exact path's row kernel (m <= 64) and its block sums; latent models run their own
    const int nblocks = vecchia_rows_blocks(row_end_ - row_begin_, m);
    d_block_sums_.alloc((size_t)std::max(nblocks, 1) * kVecchiaSums);
  }
}

// Exact Vecchia: rows (Vecchia order) split into `world` contiguous blocks, one all-reduce of the
// six partial sums per evaluation. Latent Vecchia: every rank holds the whole factor and runs
// its share of the probe columns (LatentVecchia::SetShard). Dense: replicas only.
void REModelAMD::ApplyPartition(int rank, int world) {
  if (world < 1 || rank < 0 || rank >= world) Fatal("invalid rank %d / world_size %d", rank, world);
  if (!vecchia_ && world > 1) Fatal("the dense (gp_approx='none') path runs as replicas only; SetDistributed needs gp_approx='vecchia'");
  rank_ = rank;
  world_ = world;
  const int n = cfg_.n;
  if (cfg_.latent) {
    row_begin_ = 0;
    row_end_ = nu_;
  } else {
    const int base = n / world, rem = n % world;
    row_begin_ = rank * base + std::min(rank, rem);
    row_end_ = row_begin_ + base + (rank < rem ? 1 : 0);
  }
  structure_built_ = false;
  EnsureStructure();
  HIP_CHECK(hipStreamSynchronize(stream_));
}

void REModelAMD::SetDistributed(int rank, int world, const ncclUniqueId& id, bool use_comm) {
  if (world < 1 || rank < 0 || rank >= world) Fatal("invalid rank %d / world_size %d", rank, world);
  UseDevice();
  latent_.reset();   // holds a pointer to the collective
  coll_.reset();
  if (comm_) { ncclCommDestroy(comm_); comm_ = nullptr; }
  if (world > 1 || use_comm) {
    ncclResult_t r = ncclCommInitRank(&comm_, world, id, rank);
    if (r != ncclSuccess) Fatal("ncclCommInitRank failed: %s", ncclGetErrorString(r));
    coll_.reset(new RcclCollective(comm_));
  }
  ApplyPartition(rank, world);
}

void REModelAMD::SetDistributedHost(int rank, int world, HostAllReduceFn fn, void* user) {
  if (fn == nullptr) Fatal("SetDistributedHost: the all-reduce function is NULL");
  UseDevice();
  latent_.reset();
  coll_.reset();
  if (comm_) { ncclCommDestroy(comm_); comm_ = nullptr; }
  coll_.reset(new HostCallbackCollective(fn, user));
  ApplyPartition(rank, world);
}

void REModelAMD::SetPredictionData(const char* vecchia_pred_type, int num_neighbors_pred, int nsim_var_pred) {
  if (nsim_var_pred > 0) nsim_var_pred_ = nsim_var_pred;
  if (vecchia_pred_type != nullptr) {
    const std::string t(vecchia_pred_type);
    static const char* known[] = {"order_obs_first_cond_obs_only", "order_obs_first_cond_all", "order_pred_first",
                                  "latent_order_obs_first_cond_obs_only", "latent_order_obs_first_cond_all"};
    bool ok = false;
    for (const char* k : known) ok |= t == k;
    if (!ok) Fatal("Prediction type '%s' is not supported for the Veccia approximation ", t.c_str());
    std::string tt = t;
    if (cfg_.latent) {   // SetVecchiaPredType (re_model_template.h:10564-10582): latent forms for Laplace models
      if (tt == "order_obs_first_cond_obs_only") tt = "latent_order_obs_first_cond_obs_only";
      if (tt == "order_obs_first_cond_all") tt = "latent_order_obs_first_cond_all";
      if (tt == "order_pred_first")
        Fatal("Prediction type '%s' is not supported for the Veccia approximation for non-Gaussian likelihoods ", t.c_str());
    }
    vecchia_pred_type_ = tt;
  }
  if (num_neighbors_pred > 0) num_neighbors_pred_ = num_neighbors_pred;
}

// Vecchia_utils.cpp:1634-1931 (CondObsOnly = true, Gaussian, no full-scale part) and
// re_model_template.h:3787-3803, 3960-4071: neighbours of the prediction points among the
// observed points (GPU sweep, end_search_at = n - 1), the per-point rows (A, Dp) by the
// likelihood's row kernel (rows n .. n + n_pred - 1 of [observed; prediction] coordinates), then
// mean = A . y_nbr and var = (Dp - [latent: 1]) sigma2 (predict_mean_var_kernel).
namespace {
// Gauss-Hermite rule of the given order (weight exp(-x^2)) by Newton iteration on the normalised
// Hermite recurrence; returns [nodes | weights * exp(nodes^2)] (the reference's GH_nodes_ and
// adaptive_GH_weights_ tables, likelihoods.h:12891-12980, reproduced to rounding).
std::vector<double> gauss_hermite_adaptive(int order) {
  std::vector<long double> x(order), w(order);
  const long double pim4 = 0.7511255444649424828587030047762276930510L;   // pi^-1/4
  long double z = 0.;
  const int half = (order + 1) / 2;
  for (int i = 0; i < half; ++i) {
    if (i == 0) z = std::sqrt((long double)(2 * order + 1)) - 1.85575L * std::pow((long double)(2 * order + 1), -0.16667L);
    else if (i == 1) z -= 1.14L * std::pow((long double)order, 0.426L) / z;
    else if (i == 2) z = 1.86L * z - 0.86L * x[0];
    else if (i == 3) z = 1.91L * z - 0.91L * x[1];
    else z = 2.L * z - x[i - 2];
    long double pp = 1.;
    for (int it = 0; it < 100; ++it) {
      long double p1 = pim4, p2 = 0.;
      for (int j = 1; j <= order; ++j) {
        const long double p3 = p2;
        p2 = p1;
        p1 = z * std::sqrt(2.L / j) * p2 - std::sqrt((long double)(j - 1) / j) * p3;
      }
      pp = std::sqrt(2.L * order) * p2;
      const long double z1 = z;
      z = z1 - p1 / pp;
      if (std::fabs(z - z1) <= 1e-18L) break;
    }
    x[i] = z;
    x[order - 1 - i] = -z;
    w[i] = w[order - 1 - i] = 2.L / (pp * pp);
  }
  std::vector<double> out((size_t)2 * order);
  for (int j = 0; j < order; ++j) {
    out[j] = (double)x[order - 1 - j];   // ascending, as the reference's table
    out[order + j] = (double)(w[order - 1 - j] * std::exp(x[order - 1 - j] * x[order - 1 - j]));
  }
  return out;
}
}  // namespace

void REModelAMD::Predict(const double* y, int n_pred, const double* coords_pred, const double* cov_pars,
                         bool predict_cov_mat, bool predict_var, bool predict_response, double* out,
                         const double* mean_add) {
  if (vif_) {
    PredictVif(y, n_pred, coords_pred, cov_pars, predict_cov_mat, predict_var, predict_response, out, mean_add);
    return;
  }
  if (fitc_) {
    PredictFitc(y, n_pred, coords_pred, cov_pars, predict_cov_mat, predict_var, predict_response, out, mean_add);
    return;
  }
  if (dense_lap_) {
    PredictDenseLaplace(y, n_pred, coords_pred, cov_pars, predict_cov_mat, predict_var, predict_response, out, mean_add);
    return;
  }
  if (!vecchia_) {
    PredictDense(y, n_pred, coords_pred, cov_pars, predict_cov_mat, predict_var, predict_response, out, mean_add);
    return;
  }
  if (world_ > 1) Fatal("predictions are only available on single-rank models");
  if (n_pred <= 0) Fatal("num_data_pred must be > 0");
  if (coords_pred == nullptr) Fatal("gp_coords_data_pred must be provided");
  UseDevice();
  if (y != nullptr) SetY(y);
  if (!y_set_) Fatal("response variable y has not been set (pass y or evaluate the likelihood first)");
  const bool latent = cfg_.latent;
  const int ncp = latent ? 2 : 3;
  double cp[3];
  if (cov_pars != nullptr) std::copy(cov_pars, cov_pars + ncp, cp);
  else if ((int)last_cov_pars_.size() == ncp) std::copy(last_cov_pars_.begin(), last_cov_pars_.end(), cp);
  else Fatal("cov_pars must be provided (no previous evaluation)");
  if (latent) {
    if (predict_cov_mat && predict_response && cfg_.lik != kLikGaussian)
      Fatal("predictive covariance matrices of the response are not supported for likelihood '%s' by "
            "gpboost_amd (use predict_response = false or predict_var)", cfg_.likelihood.c_str());
    // the mode at these parameters, found from zero (re_model.cpp:967-977 -> CalcCovFactorOrModeAndNegLL)
    EvalLatent(cp, false);
  }
  double trafo[3];
  if (latent) {
    trafo[0] = cp[0];
    trafo[1] = range_trafo(cfg_.cov_type, cp[1]);
  } else {
    TransformCovPars(cp, trafo);
  }
  if (!latent && vecchia_pred_type_ == "order_pred_first") {
    PredictPredFirst(n_pred, coords_pred, trafo, predict_cov_mat, predict_var, predict_response, out, mean_add);
    return;
  }
  if (!latent && vecchia_pred_type_.rfind("latent_", 0) == 0) {
    PredictLatentGaussian(n_pred, coords_pred, trafo, predict_cov_mat, predict_var, predict_response, out, mean_add);
    return;
  }
  // observed points: the latent variables' locations (unique, Vecchia order) / the observations
  const int n = latent ? nu_ : cfg_.n, d = cfg_.d, na = n + n_pred;
  const int mp = std::min(num_neighbors_pred_, n);   // end_search_at + 1 (Vecchia_utils.cpp:754-757)
  if (mp > 64) Fatal("num_neighbors_pred = %d > 64 is not supported by the GPU prediction kernel", mp);
  std::vector<double> xa((size_t)na * d);
  std::copy(coords_vo_.begin(), coords_vo_.begin() + (size_t)n * d, xa.begin());
  for (int p = 0; p < n_pred; ++p)
    for (int q = 0; q < d; ++q) xa[(size_t)(n + p) * d + q] = coords_pred[(size_t)q * n_pred + p];
  std::vector<int> nb((size_t)n_pred * mp);
  // order_obs_first_cond_all: neighbours among the observed AND the earlier prediction points
  // (find_nearest_neighbors_Vecchia_fast end_search_at = -1, Vecchia_utils.cpp:1729-1737)
  const bool cond_all = vecchia_pred_type_ == "order_obs_first_cond_all" ||
                        vecchia_pred_type_ == "latent_order_obs_first_cond_all";
  const int end_at = cond_all ? -1 : n - 1;
  if (d <= 3) vecchia_neighbors_gpu(xa.data(), na, d, mp, n, na, nb.data(), stream_, end_at);
  else vecchia_neighbors(xa.data(), na, d, mp, n, na, nb.data(), end_at);
  DevBuf<double> dxa((size_t)na * d), dB((size_t)n_pred * mp), dD(n_pred), dout((size_t)2 * n_pred), dmode;
  DevBuf<int> dnb((size_t)n_pred * mp);
  HIP_CHECK(hipMemcpyAsync(dxa.get(), xa.data(), sizeof(double) * xa.size(), hipMemcpyHostToDevice, stream_));
  HIP_CHECK(hipMemcpyAsync(dnb.get(), nb.data(), sizeof(int) * nb.size(), hipMemcpyHostToDevice, stream_));
  VecchiaRowsArgs a{};
  a.X = dxa.get();
  a.Y = nullptr;              // factor rows only
  a.nbr = dnb.get();
  a.n = na;
  a.d = d;
  a.m = mp;
  a.r0 = n;
  a.r1 = na;
  if (latent) {   // no nugget: between-neighbour diagonal * JITTER_MULT_VECCHIA, Dp = sigma1^2 - A c (:1894-1898)
    a.var = trafo[0];
    a.phi = trafo[1];
    a.diag_mult = 1. + 1e-10;
    a.diag_add = 0.;
    a.d_nugget = 0.;
  } else {
    a.var = trafo[1];
    a.phi = trafo[2];
    a.diag_mult = 1.;
    a.diag_add = 1.;          // nugget on the between-neighbour covariance (Vecchia_utils.cpp:1877)
    a.d_nugget = 1.;          // Dp starts at 1 (:1797-1798)
  }
  a.B_out = dB.get();
  a.Dinv_out = dD.get();
  a.row_base = n;
  launch_vecchia_rows(cfg_.cov_type, a, stream_);
  if (latent && (cond_all || predict_cov_mat || latent_->cholesky())) {
    PredictLatentSim(n, n_pred, mp, nb, dB.get(), dD.get(), cond_all, predict_cov_mat, predict_var, predict_response,
                     out, mean_add);
    return;
  }
  if (latent) {   // mean = -Bpo mode (likelihoods.h:6609), Dp (no nugget to remove)
    std::vector<double> mode(n);
    latent_->GetMode(mode.data());
    dmode.alloc(n);
    HIP_CHECK(hipMemcpyAsync(dmode.get(), mode.data(), sizeof(double) * n, hipMemcpyHostToDevice, stream_));
    launch_predict_mean_var(n_pred, mp, dnb.get(), dB.get(), dD.get(), dmode.get(), 1., 0., dout.get(), stream_);
  } else if (!cond_all) {
    launch_predict_mean_var(n_pred, mp, dnb.get(), dB.get(), dD.get(), d_y_.get(), trafo[0],
                            predict_response ? 0. : 1., dout.get(), stream_);
  }
  std::vector<double> h((size_t)2 * n_pred);
  std::vector<double> cov_all;   // cond_all: the dense predictive covariance (predict_cov_mat)
  if (cond_all) {
    // the covariance of cond_all is assembled on the host from the rows of Bp^-1 (they fill in): bounded like the
    // latent forms (PredictLatentSim) rather than running O(n_pred^3) host work unannounced
    if (predict_cov_mat && n_pred > 20000)
      Fatal("order_obs_first_cond_all with predict_cov_mat is limited to num_data_pred <= 20000 in gpboost_amd");
    PredictCondAll(n, n_pred, mp, nb, dB.get(), dD.get(), trafo[0], predict_response ? 0. : 1., predict_var,
                   predict_cov_mat, h, cov_all);
  } else {
    HIP_CHECK(hipMemcpyAsync(h.data(), dout.get(), sizeof(double) * h.size(), hipMemcpyDeviceToHost, stream_));
    HIP_CHECK(hipStreamSynchronize(stream_));
  }
  if (mean_add != nullptr)   // external fixed effects / linear predictor on the latent mean (re_model_template.h:3929-3946)
    for (int p = 0; p < n_pred; ++p) h[p] += mean_add[p];
  std::copy(h.begin(), h.begin() + n_pred, out);
  if (latent && (predict_var || predict_response)) {
    // + the simulation term of PredictLaplaceApproxVecchia (iterative, likelihoods.h:6628-6746)
    std::vector<double> acc(n_pred);
    latent_->PredVarSim(nsim_var_pred_, iter.num_rand_vec_trace, iter.cg_delta_conv, iter.cg_max_num_it,
                        pred_seed_++, n_pred, mp, nb.data(), dB.get(), acc.data(), nullptr, RefDraws());
    for (int p = 0; p < n_pred; ++p) h[n_pred + p] += acc[p] / nsim_var_pred_;
    if (predict_response) {
      ResponseTransform(n_pred, h.data(), h.data() + n_pred, nullptr);
      std::copy(h.begin(), h.begin() + n_pred, out);
    }
  }
  if (predict_cov_mat && cond_all) {
    std::copy(cov_all.begin(), cov_all.end(), out + n_pred);
  } else if (predict_cov_mat) {   // conditioning on observed points only: the predictive covariance is diagonal
    double* c = out + n_pred;
    std::fill(c, c + (size_t)n_pred * n_pred, 0.);
    for (int p = 0; p < n_pred; ++p) c[(size_t)p * n_pred + p] = h[n_pred + p];
  } else if (predict_var) {
    std::copy(h.begin() + n_pred, h.end(), out + n_pred);
  }
}

// Latent models (Laplace, iterative) with latent_order_obs_first_cond_all or a predictive covariance
// (PredictLaplaceApproxVecchia, likelihoods.h:6576-6749): with the prediction rows' B split into Bpo
// (observed neighbours) and Bp (earlier prediction points; identity for cond_obs_only),
//   mean = -Bp^-1 Bpo mode (forward substitution in prediction order, :6610-6616)
//   var / cov = (1/nsim) sum_draws (Bp^-1 Bpo z)(.)^T + Bp^-1 diag(Dp) Bp^-T, z ~ N(0, (Sigma^-1 + W)^-1)
// with the draws of PredVarSim kept as an n_pred x nsim matrix on the device and the moments on the
// dense path (latent_pred_moments); then the response transform as in Predict.
void REModelAMD::PredictLatentSim(int n, int n_pred, int mp, const std::vector<int>& nb, const double* dB,
                                  const double* dDinv, bool cond_all, bool predict_cov_mat, bool predict_var,
                                  bool predict_response, double* out, const double* mean_add) {
  if (cond_all && n_pred > 20000)
    Fatal("latent_order_obs_first_cond_all is limited to num_data_pred <= 20000 in gpboost_amd (dense Bp^-1)");
  if (predict_cov_mat && n_pred > 40000)
    Fatal("predictive covariance matrices are limited to num_data_pred <= 40000 in gpboost_amd");
  std::vector<double> B((size_t)n_pred * mp), Dinv(n_pred), mode(n);
  HIP_CHECK(hipMemcpyAsync(B.data(), dB, sizeof(double) * B.size(), hipMemcpyDeviceToHost, stream_));
  HIP_CHECK(hipMemcpyAsync(Dinv.data(), dDinv, sizeof(double) * n_pred, hipMemcpyDeviceToHost, stream_));
  HIP_CHECK(hipStreamSynchronize(stream_));
  latent_->GetMode(mode.data());
  std::vector<double> mean(n_pred), D(n_pred), Bpo(B), Bp;
  if (cond_all) Bp.assign((size_t)n_pred * n_pred, 0.);
  for (int p = 0; p < n_pred; ++p) {
    D[p] = 1. / Dinv[p];
    double b = 0.;
    for (int r = 0; r < mp; ++r) {
      const int j = nb[(size_t)p * mp + r];
      const double v = B[(size_t)p * mp + r];
      if (j < n) {
        b += v * mode[j];
      } else {   // an earlier prediction point (cond_all)
        Bpo[(size_t)p * mp + r] = 0.;
        Bp[(size_t)(j - n) * n_pred + p] = v;
        b -= v * mean[j - n];   // mean holds x = Bp^-1 (Bpo mode) for the earlier points
      }
    }
    mean[p] = b;
    if (cond_all) Bp[(size_t)p * n_pred + p] = 1.;
  }
  for (int p = 0; p < n_pred; ++p) mean[p] = -mean[p] + (mean_add ? mean_add[p] : 0.);
  const bool want_var = predict_var || predict_response;
  std::vector<double> var(n_pred), cov(predict_cov_mat ? (size_t)n_pred * n_pred : 0);
  if (want_var || predict_cov_mat) {
    // iterative: nsim simulation draws; cholesky: the exact term through L^-1 Bpo^T (likelihoods.h:6751-6811),
    // as n "draws" whose second moment is Bpo (Sigma^-1 + W)^-1 Bpo^T
    const bool chol = latent_->cholesky();
    const int nsim = chol ? n : nsim_var_pred_;
    if (chol && (double)n_pred * n > 4e9)
      Fatal("latent Vecchia predictions with matrix_inversion_method = 'cholesky' are limited to num_data_pred * "
            "num_data <= 4e9 in gpboost_amd (predict in batches)");
    DevBuf<double> dBpo(Bpo.size()), dV((size_t)n_pred * nsim);
    HIP_CHECK(hipMemcpyAsync(dBpo.get(), Bpo.data(), sizeof(double) * Bpo.size(), hipMemcpyHostToDevice, stream_));
    if (chol)
      latent_->PredVarChol(n_pred, mp, nb.data(), dBpo.get(), dV.get());
    else
      latent_->PredVarSim(nsim, iter.num_rand_vec_trace, iter.cg_delta_conv, iter.cg_max_num_it, pred_seed_++, n_pred,
                          mp, nb.data(), dBpo.get(), nullptr, dV.get(), RefDraws());
    latent_pred_moments(stream_, n_pred, cond_all ? Bp.data() : nullptr, D.data(), dV.get(), nsim, want_var,
                        predict_cov_mat, var.data(), cov.data());
  }
  if (predict_response) ResponseTransform(n_pred, mean.data(), var.data(), predict_cov_mat ? cov.data() : nullptr);
  std::copy(mean.begin(), mean.end(), out);
  if (predict_cov_mat) std::copy(cov.begin(), cov.end(), out + n_pred);
  else if (predict_var) std::copy(var.begin(), var.end(), out + n_pred);
}

// gp_approx = "none" (CalcPred, re_model_template.h:3894-3898 -> the dense conditional Gaussian):
// mean = Sigma_po Psi^-1 y, cov = Sigma_pp - Sigma_po Psi^-1 Sigma_op (+ the nugget for the response),
// times sigma^2 (:3956, :3967), on the dense path's factor (DenseSolver::Predict).
void REModelAMD::PredictDense(const double* y, int n_pred, const double* coords_pred, const double* cov_pars,
                              bool predict_cov_mat, bool predict_var, bool predict_response, double* out,
                              const double* mean_add) {
  if (world_ > 1) Fatal("predictions are only available on single-rank models");
  if (n_pred <= 0) Fatal("num_data_pred must be > 0");
  if (coords_pred == nullptr) Fatal("gp_coords_data_pred must be provided");
  UseDevice();
  if (y != nullptr) SetY(y);
  if (!y_set_) Fatal("response variable y has not been set (pass y or evaluate the likelihood first)");
  double cp[3];
  if (cov_pars != nullptr) std::copy(cov_pars, cov_pars + 3, cp);
  else if ((int)last_cov_pars_.size() == 3) std::copy(last_cov_pars_.begin(), last_cov_pars_.end(), cp);
  else Fatal("cov_pars must be provided (no previous evaluation)");
  double trafo[3];
  TransformCovPars(cp, trafo);
  const int d = cfg_.d;
  std::vector<double> xp((size_t)n_pred * d);
  for (int p = 0; p < n_pred; ++p)
    for (int q = 0; q < d; ++q) xp[(size_t)p * d + q] = coords_pred[(size_t)q * n_pred + p];
  std::vector<double> mean(n_pred), var(predict_var ? n_pred : 0), cov(predict_cov_mat ? (size_t)n_pred * n_pred : 0);
  dense_->Predict(cfg_.cov_type, trafo[1], trafo[2], d_y_.get(), xp.data(), n_pred, predict_var && !predict_cov_mat,
                  predict_cov_mat, mean.data(), var.data(), cov.data());
  const double nug = predict_response ? 1. : 0., s2 = trafo[0];
  for (int p = 0; p < n_pred; ++p) out[p] = mean[p] + (mean_add ? mean_add[p] : 0.);
  if (predict_cov_mat) {
    for (size_t e = 0; e < cov.size(); ++e) out[n_pred + e] = cov[e] * s2;
    for (int p = 0; p < n_pred; ++p) out[n_pred + (size_t)p * n_pred + p] += nug * s2;
  } else if (predict_var) {
    for (int p = 0; p < n_pred; ++p) out[n_pred + p] = (var[p] + nug) * s2;
  }
}

// FITC: the training point whose coordinates equal prediction point p's, or -1 (CalcPredFITC_FSA,
// re_model_template.h:10643-10691: TwoNumbersAreEqual on the coordinate sums, then per coordinate,
// utils.h:52-54 with EPSILON_NUMBERS = 1e-10); candidates by sorted coordinate sums.
std::vector<int> REModelAMD::FitcMatch(const std::vector<double>& xp, int n_pred) const {
  const int n = cfg_.n, d = cfg_.d;
  auto equal = [](double a, double b) {
    return std::fabs(a - b) < 1e-10 * std::max({1.0, std::fabs(a), std::fabs(b)});
  };
  std::vector<std::pair<double, int>> sums(n);
  for (int i = 0; i < n; ++i) {
    double s = 0.;
    for (int q = 0; q < d; ++q) s += coords_[(size_t)i * d + q];
    sums[i] = {s, i};
  }
  std::sort(sums.begin(), sums.end());
  std::vector<int> match(n_pred, -1);
  for (int p = 0; p < n_pred; ++p) {
    double sp = 0.;
    for (int q = 0; q < d; ++q) sp += xp[(size_t)p * d + q];
    const double tol = 1e-10 * std::max(1.0, std::fabs(sp)) * 2. + 1e-300;
    auto it = std::lower_bound(sums.begin(), sums.end(), std::make_pair(sp - tol, -1));
    for (; it != sums.end() && it->first <= sp + tol; ++it) {
      if (!equal(sp, it->first)) continue;
      bool same = true;
      for (int q = 0; q < d; ++q) same = same && equal(xp[(size_t)p * d + q], coords_[(size_t)it->second * d + q]);
      if (same) {
        match[p] = it->second;   // training coordinates are unique (FITC requires it)
        break;
      }
    }
  }
  return match;
}

// FITC (CalcPredFITC_FSA, re_model_template.h:10600-10828 via Predict :3890-3893): means, variances or the
// covariance matrix, times sigma^2 (:3956, :3967); prediction points that coincide with a training point
// (TwoNumbersAreEqual on the coordinate sums, then per coordinate, utils.h:52-54 with
// EPSILON_NUMBERS = 1e-10) get the FITC diagonal correction.
// gp_approx = "full_scale_vecchia", Gaussian likelihood (re_model_template.h:3708-3752 ->
// CalcPredVecchiaObservedFirstOrder with the full-scale branches, Vecchia_utils.cpp:1634-1980): the prediction
// points follow the observed ones in the model order; neighbours among the observed points (cond_obs_only) or
// the observed and earlier prediction points (cond_all) by the reference's sweep; VifSolver::Predict on the
// transformed scale, then times sigma^2 with the nugget removed for the latent process (:3776-3792).
void REModelAMD::PredictVif(const double* y, int n_pred, const double* coords_pred, const double* cov_pars,
                            bool predict_cov_mat, bool predict_var, bool predict_response, double* out,
                            const double* mean_add) {
  if (world_ > 1) Fatal("predictions are only available on single-rank models");
  if (n_pred <= 0) Fatal("num_data_pred must be > 0");
  if (coords_pred == nullptr) Fatal("gp_coords_data_pred must be provided");
  if (cfg_.latent) {
    PredictVifLaplace(y, n_pred, coords_pred, cov_pars, predict_cov_mat, predict_var, predict_response, out, mean_add);
    return;
  }
  const bool cond_all = vecchia_pred_type_ == "order_obs_first_cond_all";
  if (!cond_all && vecchia_pred_type_ != "order_obs_first_cond_obs_only") {
    if (vecchia_pred_type_ == "order_pred_first")   // re_model_template.h:3748-3750
      Fatal("The full-scale Vecchia approximation is currently not implemented when prediction locations appear "
            "first in the ordering. Please use vecchia_pred_type = order_obs_first_cond_all or vecchia_pred_type = "
            "order_obs_first_cond_obs_only");
    Fatal("The full-scale Vecchia approximation for latent process(es) is currently not implemented");   // :3761-3763
  }
  UseDevice();
  if (y != nullptr) SetY(y);
  if (!y_set_) Fatal("response variable y has not been set (pass y or evaluate the likelihood first)");
  double cp[3];
  if (cov_pars != nullptr) std::copy(cov_pars, cov_pars + 3, cp);
  else if ((int)last_cov_pars_.size() == 3) std::copy(last_cov_pars_.begin(), last_cov_pars_.end(), cp);
  else Fatal("cov_pars must be provided (no previous evaluation)");
  double trafo[3];
  TransformCovPars(cp, trafo);
  const int n = cfg_.n, d = cfg_.d, na = n + n_pred;
  const int mp = std::min(num_neighbors_pred_, cond_all ? na - 1 : n);
  std::vector<double> xa((size_t)na * d);
  std::copy(coords_vo_.begin(), coords_vo_.begin() + (size_t)n * d, xa.begin());
  for (int p = 0; p < n_pred; ++p)
    for (int q = 0; q < d; ++q) xa[(size_t)(n + p) * d + q] = coords_pred[(size_t)q * n_pred + p];
  std::vector<int> nb((size_t)n_pred * mp);
  const int end_at = cond_all ? -1 : n - 1;
  if (d <= 3 && mp <= 64) vecchia_neighbors_gpu(xa.data(), na, d, mp, n, na, nb.data(), stream_, end_at);
  else vecchia_neighbors(xa.data(), na, d, mp, n, na, nb.data(), end_at);
  if (cond_all)   // the first prediction points have fewer candidates: their unused slots are -1 (no neighbour)
    for (int p = 0; p < n_pred; ++p)
      for (int r = std::min(n + p, mp); r < mp; ++r) nb[(size_t)p * mp + r] = -1;
  std::vector<double> mean(n_pred), var(predict_var ? n_pred : 0), cov(predict_cov_mat ? (size_t)n_pred * n_pred : 0);
  vif_->Predict(cfg_.cov_type, trafo[1], trafo[2], d_y_.get(), xa.data() + (size_t)n * d, n_pred, nb.data(), mp,
                cond_all, mean.data(), predict_var ? var.data() : nullptr, predict_cov_mat ? cov.data() : nullptr);
  if (mean_add != nullptr)
    for (int p = 0; p < n_pred; ++p) mean[p] += mean_add[p];
  std::copy(mean.begin(), mean.end(), out);
  const double nug = predict_response ? 0. : 1.;
  if (predict_cov_mat) {
    for (int p = 0; p < n_pred; ++p) cov[(size_t)p * n_pred + p] -= nug;
    for (size_t e = 0; e < cov.size(); ++e) out[n_pred + e] = cov[e] * trafo[0];
  } else if (predict_var) {
    for (int p = 0; p < n_pred; ++p) out[n_pred + p] = (var[p] - nug) * trafo[0];
  }
}

// gp_approx = "full_scale_vecchia" with a Laplace likelihood (re_model_template.h:3811-3846 ->
// CalcPredVecchiaObservedFirstOrder for Bpo / Bp / Dp of the latent residual and PredictLaplaceApproxFSVA,
// likelihoods.h:6060-6551): the mode at the parameters (found from zero), latent means, variances or covariance
// matrices by VifLaplace::Predict, the prediction points' fixed effects added, the response transform.
void REModelAMD::PredictVifLaplace(const double* y, int n_pred, const double* coords_pred, const double* cov_pars,
                                   bool predict_cov_mat, bool predict_var, bool predict_response, double* out,
                                   const double* mean_add) {
  const std::string& t = vecchia_pred_type_;
  const bool cond_all = t == "latent_order_obs_first_cond_all" || t == "order_obs_first_cond_all";
  if (!cond_all && t != "latent_order_obs_first_cond_obs_only" && t != "order_obs_first_cond_obs_only")
    Fatal("Prediction type '%s' is not supported for the Veccia approximation.", t.c_str());   // :3848-3850
  UseDevice();
  if (y != nullptr) SetY(y);
  if (!y_set_) Fatal("response variable y has not been set (pass y or evaluate the likelihood first)");
  double cp[2];
  if (cov_pars != nullptr) std::copy(cov_pars, cov_pars + 2, cp);
  else if ((int)last_cov_pars_.size() == 2) std::copy(last_cov_pars_.begin(), last_cov_pars_.end(), cp);
  else Fatal("cov_pars must be provided (no previous evaluation)");
  if (predict_cov_mat && predict_response)
    Fatal("predictive covariance matrices of the response are not supported for likelihood '%s' by gpboost_amd "
          "(use predict_response = false or predict_var)", cfg_.likelihood.c_str());
  EvalLatent(cp, false);   // the mode at these parameters (found from zero)
  const int n = cfg_.n, d = cfg_.d, na = n + n_pred;
  const int mp = std::min(num_neighbors_pred_, cond_all ? na - 1 : n);
  std::vector<double> xa((size_t)na * d);
  std::copy(coords_vo_.begin(), coords_vo_.begin() + (size_t)n * d, xa.begin());
  for (int p = 0; p < n_pred; ++p)
    for (int q = 0; q < d; ++q) xa[(size_t)(n + p) * d + q] = coords_pred[(size_t)q * n_pred + p];
  std::vector<int> nb((size_t)n_pred * mp);
  const int end_at = cond_all ? -1 : n - 1;
  if (d <= 3 && mp <= 64) vecchia_neighbors_gpu(xa.data(), na, d, mp, n, na, nb.data(), stream_, end_at);
  else vecchia_neighbors(xa.data(), na, d, mp, n, na, nb.data(), end_at);
  if (cond_all)
    for (int p = 0; p < n_pred; ++p)
      for (int r = std::min(n + p, mp); r < mp; ++r) nb[(size_t)p * mp + r] = -1;
  const bool want_var = predict_var || predict_response;
  std::vector<double> mean(n_pred), var(want_var ? n_pred : 0), cov(predict_cov_mat ? (size_t)n_pred * n_pred : 0);
  vif_lap_->Predict(cfg_.cov_type, cp[0], range_trafo(cfg_.cov_type, cp[1]), xa.data() + (size_t)n * d, n_pred, nb.data(),
                    mp, cond_all, mean.data(), want_var ? var.data() : nullptr, predict_cov_mat ? cov.data() : nullptr);
  if (mean_add != nullptr)
    for (int p = 0; p < n_pred; ++p) mean[p] += mean_add[p];
  if (predict_response) ResponseTransform(n_pred, mean.data(), var.data(), nullptr);
  std::copy(mean.begin(), mean.end(), out);
  if (predict_cov_mat) std::copy(cov.begin(), cov.end(), out + n_pred);
  else if (predict_var) std::copy(var.begin(), var.end(), out + n_pred);
}

void REModelAMD::PredictFitc(const double* y, int n_pred, const double* coords_pred, const double* cov_pars,
                             bool predict_cov_mat, bool predict_var, bool predict_response, double* out,
                             const double* mean_add) {
  if (n_pred <= 0) Fatal("num_data_pred must be > 0");
  if (coords_pred == nullptr) Fatal("gp_coords_data_pred must be provided");
  if (cfg_.latent) {
    PredictFitcLaplace(y, n_pred, coords_pred, cov_pars, predict_cov_mat, predict_var, predict_response, out, mean_add);
    return;
  }
  UseDevice();
  if (y != nullptr) SetY(y);
  if (!y_set_) Fatal("response variable y has not been set (pass y or evaluate the likelihood first)");
  double cp[3];
  if (cov_pars != nullptr) std::copy(cov_pars, cov_pars + 3, cp);
  else if ((int)last_cov_pars_.size() == 3) std::copy(last_cov_pars_.begin(), last_cov_pars_.end(), cp);
  else Fatal("cov_pars must be provided (no previous evaluation)");
  double trafo[3];
  TransformCovPars(cp, trafo);
  const int d = cfg_.d;
  std::vector<double> xp((size_t)n_pred * d);
  for (int p = 0; p < n_pred; ++p)
    for (int q = 0; q < d; ++q) xp[(size_t)p * d + q] = coords_pred[(size_t)q * n_pred + p];
  const std::vector<int> match = FitcMatch(xp, n_pred);
  std::vector<double> mean(n_pred), var(predict_var ? n_pred : 0);
  std::vector<double> cov(predict_cov_mat ? (size_t)n_pred * n_pred : 0);
  fitc_->Predict(cfg_.cov_type, trafo[1], trafo[2], d_y_.get(), xp.data(), n_pred, match, predict_var,
                 predict_cov_mat, predict_response, mean.data(), var.data(), cov.data());
  if (mean_add != nullptr)
    for (int p = 0; p < n_pred; ++p) mean[p] += mean_add[p];
  std::copy(mean.begin(), mean.end(), out);
  if (predict_cov_mat) {
    for (size_t e = 0; e < cov.size(); ++e) out[n_pred + e] = cov[e] * trafo[0];
  } else if (predict_var) {
    for (int p = 0; p < n_pred; ++p) out[n_pred + p] = var[p] * trafo[0];
  }
}

// PredictResponse (likelihoods.h:7526-7580) on the latent predictive mean / variance (n_pred each, in place):
// bernoulli_logit by the adaptive Gauss-Hermite rule on the GPU, bernoulli_probit / poisson in closed form,
// gaussian (vecchia_latent) + the error variance (also on the covariance diagonal, cov nullable).
void REModelAMD::ResponseTransform(int n_pred, double* mean, double* var, double* cov) {
  if (cfg_.lik == kLikBernoulliLogit) {
    static const std::vector<double> gh = gauss_hermite_adaptive(30);   // order_GH_ = 30 (likelihoods.h:12877)
    DevBuf<double> dmv((size_t)2 * n_pred), dgh(gh.size()), dout((size_t)2 * n_pred);
    HIP_CHECK(hipMemcpyAsync(dmv.get(), mean, sizeof(double) * n_pred, hipMemcpyHostToDevice, stream_));
    HIP_CHECK(hipMemcpyAsync(dmv.get() + n_pred, var, sizeof(double) * n_pred, hipMemcpyHostToDevice, stream_));
    HIP_CHECK(hipMemcpyAsync(dgh.get(), gh.data(), sizeof(double) * gh.size(), hipMemcpyHostToDevice, stream_));
    launch_resp_logit(n_pred, dmv.get(), dmv.get() + n_pred, dgh.get(), dgh.get() + 30, 30, iter.delta_conv_mode_finding,
                      dout.get(), dout.get() + n_pred, stream_);
    HIP_CHECK(hipMemcpyAsync(mean, dout.get(), sizeof(double) * n_pred, hipMemcpyDeviceToHost, stream_));
    HIP_CHECK(hipMemcpyAsync(var, dout.get() + n_pred, sizeof(double) * n_pred, hipMemcpyDeviceToHost, stream_));
    HIP_CHECK(hipStreamSynchronize(stream_));
  } else if (cfg_.lik == kLikBernoulliProbit) {   // :7531-7543
    for (int p = 0; p < n_pred; ++p) {
      mean[p] = 0.5 * std::erfc(-(mean[p] / std::sqrt(1. + var[p])) * M_SQRT1_2);
      var[p] = mean[p] * (1. - mean[p]);
    }
  } else if (cfg_.lik == kLikGamma) {   // :7571-7584
    const double a = aux_pars_.empty() ? 1. : aux_pars_[0];
    for (int p = 0; p < n_pred; ++p) {
      const double pm = std::exp(mean[p] + 0.5 * var[p]);
      var[p] = (std::exp(var[p]) - 1.) * pm * pm + std::exp(2 * mean[p] + 2 * var[p]) / a;
      mean[p] = pm;
    }
  } else if (cfg_.lik == kLikPoisson) {   // :7557-7569
    for (int p = 0; p < n_pred; ++p) {
      const double pm = std::exp(mean[p] + 0.5 * var[p]);
      var[p] = pm * ((std::exp(var[p]) - 1.) * pm + 1.);
      mean[p] = pm;
    }
  } else {   // gaussian vecchia_latent: + the error variance
    const double aux = aux_pars_.empty() ? 0. : aux_pars_[0];
    for (int p = 0; p < n_pred; ++p) var[p] += aux;
    if (cov != nullptr)
      for (int p = 0; p < n_pred; ++p) cov[(size_t)p * n_pred + p] += aux;
  }
}

// FITC with a Laplace likelihood (CalcPredFITC_FSA, re_model_template.h:10600-10760, then
// PredictLaplaceApproxFITC, likelihoods.h:7157-7232): the mode at the parameters (found from zero, as
// the Vecchia latent path), then latent means / variances / covariance (FitcLaplace::Predict), the
// fixed effects of the prediction points added to the mean, and for predict_response the bernoulli_logit
// response probabilities by the adaptive Gauss-Hermite rule (PredictResponse, likelihoods.h:7544-7556).
void REModelAMD::PredictFitcLaplace(const double* y, int n_pred, const double* coords_pred, const double* cov_pars,
                                    bool predict_cov_mat, bool predict_var, bool predict_response, double* out,
                                    const double* mean_add) {
  UseDevice();
  if (y != nullptr) SetY(y);
  if (!y_set_) Fatal("response variable y has not been set (pass y or evaluate the likelihood first)");
  double cp[2];
  if (cov_pars != nullptr) std::copy(cov_pars, cov_pars + 2, cp);
  else if ((int)last_cov_pars_.size() == 2) std::copy(last_cov_pars_.begin(), last_cov_pars_.end(), cp);
  else Fatal("cov_pars must be provided (no previous evaluation)");
  if (predict_cov_mat && predict_response)
    Fatal("predictive covariance matrices of the response are not supported for likelihood '%s' by gpboost_amd "
          "(use predict_response = false or predict_var)", cfg_.likelihood.c_str());
  EvalLatent(cp, false);   // the mode at these parameters (SetYCalcCovCalcYAuxForPred, re_model_template.h:3306-3312)
  const int d = cfg_.d;
  std::vector<double> xp((size_t)n_pred * d);
  for (int p = 0; p < n_pred; ++p)
    for (int q = 0; q < d; ++q) xp[(size_t)p * d + q] = coords_pred[(size_t)q * n_pred + p];
  const std::vector<int> match = FitcMatch(xp, n_pred);
  const bool want_var = predict_var || predict_response;
  std::vector<double> mean(n_pred), var(want_var ? n_pred : 0), cov(predict_cov_mat ? (size_t)n_pred * n_pred : 0);
  fitc_lap_->Predict(cfg_.cov_type, cp[0], range_trafo(cfg_.cov_type, cp[1]), xp.data(), n_pred, match, want_var,
                     predict_cov_mat, mean.data(), var.data(), cov.data());
  if (mean_add != nullptr)
    for (int p = 0; p < n_pred; ++p) mean[p] += mean_add[p];
  if (predict_response) ResponseTransform(n_pred, mean.data(), var.data(), nullptr);
  std::copy(mean.begin(), mean.end(), out);
  if (predict_cov_mat) std::copy(cov.begin(), cov.end(), out + n_pred);
  else if (predict_var) std::copy(var.begin(), var.end(), out + n_pred);
}

// gp_approx = "none" with a Laplace likelihood (CalcPred, re_model_template.h:10026- -> PredictLaplaceApproxStable,
// likelihoods.h:5610-5676): the mode at the parameters (found from zero), latent means Sigma_po d1 and
// (co)variances from the factor of I + W^1/2 Sigma W^1/2, the prediction points' fixed effects added to the mean,
// the response transform for predict_response.
void REModelAMD::PredictDenseLaplace(const double* y, int n_pred, const double* coords_pred, const double* cov_pars,
                                     bool predict_cov_mat, bool predict_var, bool predict_response, double* out,
                                     const double* mean_add) {
  if (n_pred <= 0) Fatal("num_data_pred must be > 0");
  if (coords_pred == nullptr) Fatal("gp_coords_data_pred must be provided");
  UseDevice();
  if (y != nullptr) SetY(y);
  if (!y_set_) Fatal("response variable y has not been set (pass y or evaluate the likelihood first)");
  double cp[2];
  if (cov_pars != nullptr) std::copy(cov_pars, cov_pars + 2, cp);
  else if ((int)last_cov_pars_.size() == 2) std::copy(last_cov_pars_.begin(), last_cov_pars_.end(), cp);
  else Fatal("cov_pars must be provided (no previous evaluation)");
  if (predict_cov_mat && predict_response)
    Fatal("predictive covariance matrices of the response are not supported for likelihood '%s' by gpboost_amd "
          "(use predict_response = false or predict_var)", cfg_.likelihood.c_str());
  EvalLatent(cp, false);   // the mode at these parameters (SetYCalcCovCalcYAuxForPred, re_model_template.h:3306-3312)
  const int d = cfg_.d;
  std::vector<double> xp((size_t)n_pred * d);
  for (int p = 0; p < n_pred; ++p)
    for (int q = 0; q < d; ++q) xp[(size_t)p * d + q] = coords_pred[(size_t)q * n_pred + p];
  const bool want_var = predict_var || predict_response;
  std::vector<double> mean(n_pred), var(want_var ? n_pred : 0), cov(predict_cov_mat ? (size_t)n_pred * n_pred : 0);
  dense_lap_->Predict(cfg_.cov_type, cp[0], range_trafo(cfg_.cov_type, cp[1]), xp.data(), n_pred, want_var,
                      predict_cov_mat, mean.data(), var.data(), cov.data());
  if (mean_add != nullptr)
    for (int p = 0; p < n_pred; ++p) mean[p] += mean_add[p];
  if (predict_response) ResponseTransform(n_pred, mean.data(), var.data(), nullptr);
  std::copy(mean.begin(), mean.end(), out);
  if (predict_cov_mat) std::copy(cov.begin(), cov.end(), out + n_pred);
  else if (predict_var) std::copy(var.begin(), var.end(), out + n_pred);
}

// order_pred_first, Gaussian likelihood (CalcPredVecchiaPredictedFirstOrder, Vecchia_utils.cpp:2018-2239):
// the prediction points first (given order), then the observations (Vecchia order); every point's
// neighbours among ALL earlier points (GPU sweep from row 0); the rows' (B, D^-1) by the row kernel.
// With Bp (prediction rows, prediction columns), Bop / Bo (observation rows, prediction /
// observation columns):
//   cond_prec = Bp^T Dp^-1 Bp + Bop^T Do^-1 Bop,  mean = -cond_prec^-1 Bop^T Do^-1 Bo y,
//   cov = cond_prec^-1 (variances its diagonal), less the nugget unless predict_response, times
// sigma^2 (re_model_template.h:3788-3815). cond_prec is assembled on the host (O((n + n_pred) m^2))
// and factorized densely on the GPU (POTRF / TRTRI / GEMM). The reference factorizes it with a
// fill-reducing (AMD) permutation and reads the variances / covariance off the inverse of the
// permuted factor, i.e. in AMD-permuted order; here they come in prediction-point order.
void REModelAMD::PredictPredFirst(int n_pred, const double* coords_pred, const double* trafo, bool predict_cov_mat,
                                  bool predict_var, bool predict_response, double* out, const double* mean_add) {
  const int n = cfg_.n, d = cfg_.d, na = n + n_pred;
  const int mp = std::min(num_neighbors_pred_, na - 1);
  if (mp > 64) Fatal("num_neighbors_pred = %d > 64 is not supported by the GPU prediction kernel", mp);
  std::vector<double> xa((size_t)na * d);
  for (int p = 0; p < n_pred; ++p)
    for (int q = 0; q < d; ++q) xa[(size_t)p * d + q] = coords_pred[(size_t)q * n_pred + p];
  std::copy(coords_vo_.begin(), coords_vo_.begin() + (size_t)n * d, xa.begin() + (size_t)n_pred * d);
  std::vector<int> nb((size_t)na * mp, -1);
  if (d <= 3) vecchia_neighbors_gpu(xa.data(), na, d, mp, 0, na, nb.data(), stream_, -1);
  else vecchia_neighbors(xa.data(), na, d, mp, 0, na, nb.data(), -1);
  DevBuf<double> dxa((size_t)na * d), dB((size_t)na * mp), dD(na);
  DevBuf<int> dnb((size_t)na * mp);
  HIP_CHECK(hipMemcpyAsync(dxa.get(), xa.data(), sizeof(double) * xa.size(), hipMemcpyHostToDevice, stream_));
  HIP_CHECK(hipMemcpyAsync(dnb.get(), nb.data(), sizeof(int) * nb.size(), hipMemcpyHostToDevice, stream_));
  VecchiaRowsArgs a{};
  a.X = dxa.get();
  a.Y = nullptr;
  a.nbr = dnb.get();
  a.n = na;
  a.d = d;
  a.m = mp;
  a.r0 = 0;
  a.r1 = na;
  a.var = trafo[1];
  a.phi = trafo[2];
  a.diag_mult = 1.;
  a.diag_add = 1.;      // nugget on the between-neighbour covariance (Vecchia_utils.cpp:2189)
  a.d_nugget = 1.;      // Dp_inv / Do_inv start at 1 (:2124-2125)
  a.B_out = dB.get();
  a.Dinv_out = dD.get();
  a.row_base = 0;
  launch_vecchia_rows(cfg_.cov_type, a, stream_);
  std::vector<double> B((size_t)na * mp), Dinv(na), y(n);
  HIP_CHECK(hipMemcpyAsync(B.data(), dB.get(), sizeof(double) * B.size(), hipMemcpyDeviceToHost, stream_));
  HIP_CHECK(hipMemcpyAsync(Dinv.data(), dD.get(), sizeof(double) * na, hipMemcpyDeviceToHost, stream_));
  HIP_CHECK(hipMemcpyAsync(y.data(), d_y_.get(), sizeof(double) * n, hipMemcpyDeviceToHost, stream_));
  HIP_CHECK(hipStreamSynchronize(stream_));
  // cond_prec (column-major n_pred x n_pred) and y_aux = Bop^T Do^-1 Bo y
  std::vector<double> P((size_t)n_pred * n_pred, 0.), yaux(n_pred, 0.);
  std::vector<int> pc;        // prediction columns of one row (incl. the diagonal of a prediction row)
  std::vector<double> pv;
  for (int i = 0; i < na; ++i) {
    const int k = std::min(i, mp);
    pc.clear();
    pv.clear();
    double boy = 0.;   // (Bo y)_i for an observation row
    if (i < n_pred) {
      pc.push_back(i);
      pv.push_back(1.);
    } else {
      boy = y[i - n_pred];
    }
    for (int r = 0; r < k; ++r) {
      const int j = nb[(size_t)i * mp + r];
      const double b = B[(size_t)i * mp + r];
      if (j < n_pred) {
        pc.push_back(j);
        pv.push_back(b);
      } else {
        boy += b * y[j - n_pred];
      }
    }
    const double w = Dinv[i];
    for (size_t u = 0; u < pc.size(); ++u) {
      for (size_t v = 0; v < pc.size(); ++v) P[(size_t)pc[v] * n_pred + pc[u]] += pv[u] * w * pv[v];
      if (i >= n_pred) yaux[pc[u]] += pv[u] * w * boy;
    }
  }
  std::vector<double> mean(n_pred), var(n_pred), cov(predict_cov_mat ? (size_t)n_pred * n_pred : 0);
  spd_solve_inverse(stream_, n_pred, P.data(), yaux.data(), mean.data(), var.data(),
                    predict_cov_mat ? cov.data() : nullptr);
  const double nug = predict_response ? 0. : 1., s2 = trafo[0];
  for (int p = 0; p < n_pred; ++p) out[p] = -mean[p] + (mean_add ? mean_add[p] : 0.);
  if (predict_cov_mat) {
    for (size_t e = 0; e < cov.size(); ++e) out[n_pred + e] = cov[e] * s2;
    for (int p = 0; p < n_pred; ++p) out[n_pred + (size_t)p * n_pred + p] -= nug * s2;
  } else if (predict_var) {
    for (int p = 0; p < n_pred; ++p) out[n_pred + p] = (var[p] - nug) * s2;
  }
}

// latent_order_obs_first_cond_obs_only / latent_order_obs_first_cond_all with the Gaussian likelihood
// (CalcPredVecchiaLatentObservedFirstOrder, Vecchia_utils.cpp:2241-2442, dispatched at
// re_model_template.h:3755-3786): a Vecchia approximation of the LATENT process over the observed
// (Vecchia order) then the prediction points, num_neighbors_pred neighbours for every point among the
// earlier observed points (cond_obs_only) or all earlier points (cond_all), no nugget (between-neighbour
// diagonal times JITTER_MULT_VECCHIA, D = sigma1^2 - A c); then Sigma = B^-1 D B^-T and the Gaussian
// conditional given y = latent + N(0, 1): mean = Sigma_po (Sigma_oo + I)^-1 y, cov = Sigma_pp -
// Sigma_po (Sigma_oo + I)^-1 Sigma_op (+ I for the response), times sigma^2. The reference forms
// B^-1 as a sparse matrix with fill; here B is dense and everything runs on the GPU's dense path, so
// the observed plus prediction points are bounded (N <= 20000).
void REModelAMD::PredictLatentGaussian(int n_pred, const double* coords_pred, const double* trafo,
                                       bool predict_cov_mat, bool predict_var, bool predict_response, double* out,
                                       const double* mean_add) {
  const int n = cfg_.n, d = cfg_.d, N = n + n_pred;
  if (N > 20000)
    Fatal("vecchia_pred_type '%s' with the Gaussian likelihood is limited to num_data + num_data_pred <= 20000 in "
          "gpboost_amd (dense latent covariance)", vecchia_pred_type_.c_str());
  const bool cond_all = vecchia_pred_type_ == "latent_order_obs_first_cond_all";
  const int mp = std::min(num_neighbors_pred_, N - 1);
  if (mp > 64) Fatal("num_neighbors_pred = %d > 64 is not supported by the GPU prediction kernel", mp);
  std::vector<double> xa((size_t)N * d);
  std::copy(coords_vo_.begin(), coords_vo_.begin() + (size_t)n * d, xa.begin());
  for (int p = 0; p < n_pred; ++p)
    for (int q = 0; q < d; ++q) xa[(size_t)(n + p) * d + q] = coords_pred[(size_t)q * n_pred + p];
  {
    std::vector<int> uniq, idx;
    unique_locations(xa.data(), N, d, uniq, idx);
    if ((int)uniq.size() < N)
      Fatal("Duplicates found among training and test coordinates. This is not supported for predictions with a "
            "Vecchia approximation for the latent process ('latent_') in gpboost_amd ");
  }
  std::vector<int> nb((size_t)N * mp, -1);
  const int end_at = cond_all ? -1 : n - 1;
  if (d <= 3) vecchia_neighbors_gpu(xa.data(), N, d, mp, 0, N, nb.data(), stream_, end_at);
  else vecchia_neighbors(xa.data(), N, d, mp, 0, N, nb.data(), end_at);
  DevBuf<double> dxa((size_t)N * d), dB((size_t)N * mp), dD(N);
  DevBuf<int> dnb((size_t)N * mp);
  HIP_CHECK(hipMemcpyAsync(dxa.get(), xa.data(), sizeof(double) * xa.size(), hipMemcpyHostToDevice, stream_));
  HIP_CHECK(hipMemcpyAsync(dnb.get(), nb.data(), sizeof(int) * nb.size(), hipMemcpyHostToDevice, stream_));
  VecchiaRowsArgs a{};
  a.X = dxa.get();
  a.Y = nullptr;
  a.nbr = dnb.get();
  a.n = N;
  a.d = d;
  a.m = mp;
  a.r0 = 0;
  a.r1 = N;
  a.var = trafo[1];
  a.phi = trafo[2];
  a.diag_mult = 1. + 1e-10;   // JITTER_MULT_VECCHIA (utils.h:36, Vecchia_utils.cpp:2382)
  a.diag_add = 0.;
  a.d_nugget = 0.;
  a.B_out = dB.get();
  a.Dinv_out = dD.get();
  a.row_base = 0;
  launch_vecchia_rows(cfg_.cov_type, a, stream_);
  std::vector<double> Bv((size_t)N * mp), Dinv(N), y(n);
  HIP_CHECK(hipMemcpyAsync(Bv.data(), dB.get(), sizeof(double) * Bv.size(), hipMemcpyDeviceToHost, stream_));
  HIP_CHECK(hipMemcpyAsync(Dinv.data(), dD.get(), sizeof(double) * N, hipMemcpyDeviceToHost, stream_));
  HIP_CHECK(hipMemcpyAsync(y.data(), d_y_.get(), sizeof(double) * n, hipMemcpyDeviceToHost, stream_));
  HIP_CHECK(hipStreamSynchronize(stream_));
  std::vector<double> Bd((size_t)N * N, 0.), D(N);
  for (int i = 0; i < N; ++i) {
    Bd[(size_t)i * N + i] = 1.;
    const int k = std::min(i, mp);
    for (int r = 0; r < k; ++r) {
      const int j = nb[(size_t)i * mp + r];
      if (j >= 0) Bd[(size_t)j * N + i] += Bv[(size_t)i * mp + r];
    }
    D[i] = 1. / Dinv[i];
  }
  std::vector<double> mean(n_pred), var(n_pred), cov(predict_cov_mat ? (size_t)n_pred * n_pred : 0);
  vecchia_latent_dense_pred(stream_, N, n, Bd.data(), D.data(), y.data(), predict_var, predict_cov_mat, mean.data(),
                            var.data(), cov.data());
  const double nug = predict_response ? 1. : 0., s2 = trafo[0];
  for (int p = 0; p < n_pred; ++p) out[p] = mean[p] + (mean_add ? mean_add[p] : 0.);
  if (predict_cov_mat) {
    for (size_t e = 0; e < cov.size(); ++e) out[n_pred + e] = cov[e] * s2;
    for (int p = 0; p < n_pred; ++p) out[n_pred + (size_t)p * n_pred + p] += nug * s2;
  } else if (predict_var) {
    for (int p = 0; p < n_pred; ++p) out[n_pred + p] = (var[p] + nug) * s2;
  }
}

// order_obs_first_cond_all, Gaussian likelihood (Vecchia_utils.cpp:1776-1803 the B rows split into
// Bpo (observed neighbours) and Bp (earlier prediction points), :1977-2006 the moments): the rows
// (A = -B, Dp) come from the row kernel like the obs-only type; then on the host
//   mean = -Bp^-1 Bpo y                         (sp_L_solve: forward substitution in prediction order)
//   cov  = Bp^-1 diag(Dp) Bp^-T, var its diagonal (rows of Bp^-1 by the same recursion)
// less the nugget unless predict_response, times sigma^2 (re_model_template.h:3789-3815).
void REModelAMD::PredictCondAll(int n, int n_pred, int mp, const std::vector<int>& nb, const double* dB,
                                const double* dDinv, double sigma2, double nugget_sub, bool want_var, bool want_cov,
                                std::vector<double>& h, std::vector<double>& cov) {
  std::vector<double> B((size_t)n_pred * mp), Dinv(n_pred), y(n);
  HIP_CHECK(hipMemcpyAsync(B.data(), dB, sizeof(double) * B.size(), hipMemcpyDeviceToHost, stream_));
  HIP_CHECK(hipMemcpyAsync(Dinv.data(), dDinv, sizeof(double) * n_pred, hipMemcpyDeviceToHost, stream_));
  HIP_CHECK(hipMemcpyAsync(y.data(), d_y_.get(), sizeof(double) * n, hipMemcpyDeviceToHost, stream_));
  HIP_CHECK(hipStreamSynchronize(stream_));
  h.assign((size_t)2 * n_pred, 0.);
  double* mu = h.data();
  for (int p = 0; p < n_pred; ++p) {   // -Bpo y
    double s = 0.;
    for (int r = 0; r < mp; ++r) {
      const int j = nb[(size_t)p * mp + r];
      if (j < n) s -= B[(size_t)p * mp + r] * y[j];
    }
    mu[p] = s;
  }
  for (int p = 0; p < n_pred; ++p)   // Bp mu = -Bpo y, unit lower triangular in prediction order
    for (int r = 0; r < mp; ++r) {
      const int j = nb[(size_t)p * mp + r];
      if (j >= n) mu[p] -= B[(size_t)p * mp + r] * mu[j - n];
    }
  if (!want_var && !want_cov) return;
  // rows of Bp^-1: R_p = e_p - sum_{j in pred nbrs(p)} B_pj R_j (sparse, column indices ascending)
  std::vector<std::vector<std::pair<int, double>>> R(n_pred);
  std::vector<double> acc(n_pred, 0.);
  std::vector<int> touched;
  std::vector<char> on(n_pred, 0);
  for (int p = 0; p < n_pred; ++p) {
    touched.clear();
    acc[p] = 1.;
    on[p] = 1;
    touched.push_back(p);
    for (int r = 0; r < mp; ++r) {
      const int j = nb[(size_t)p * mp + r];
      if (j < n) continue;
      const double b = B[(size_t)p * mp + r];
      for (const auto& e : R[j - n]) {
        if (!on[e.first]) { on[e.first] = 1; acc[e.first] = 0.; touched.push_back(e.first); }
        acc[e.first] -= b * e.second;
      }
    }
    std::sort(touched.begin(), touched.end());
    R[p].reserve(touched.size());
    for (int k : touched) {
      R[p].emplace_back(k, acc[k]);
      on[k] = 0;
    }
  }
  std::vector<double> Dp(n_pred);
  for (int p = 0; p < n_pred; ++p) Dp[p] = 1. / Dinv[p];
  for (int p = 0; p < n_pred; ++p) {
    double v = 0.;
    for (const auto& e : R[p]) v += e.second * e.second * Dp[e.first];
    h[n_pred + p] = (v - nugget_sub) * sigma2;
  }
  if (!want_cov) return;
  // cov = Bp^-1 diag(Dp) Bp^-T on the dense path (unit-lower inverse + MFMA GEMM; the host product of
  // the filled-in rows was O(n_pred^3)); Bp column-major with its unit diagonal, as PredictLatentSim
  std::vector<double> Bp((size_t)n_pred * n_pred, 0.);
  for (int p = 0; p < n_pred; ++p) {
    Bp[(size_t)p * n_pred + p] = 1.;
    for (int r = 0; r < mp; ++r) {
      const int j = nb[(size_t)p * mp + r];
      if (j >= n) Bp[(size_t)(j - n) * n_pred + p] = B[(size_t)p * mp + r];
    }
  }
  cov.assign((size_t)n_pred * n_pred, 0.);
  latent_pred_moments(stream_, n_pred, Bp.data(), Dp.data(), nullptr, 0, false, true, nullptr, cov.data());
  for (double& c : cov) c *= sigma2;
  for (int p = 0; p < n_pred; ++p) cov[(size_t)p * n_pred + p] -= nugget_sub * sigma2;
}

void REModelAMD::TransformCovPars(const double* orig, double* trafo) const {
  // re_model_template.h:7189-7213 -> cov_fcts.h:438-460
  if (!(orig[0] > 0. && orig[1] > 0. && orig[2] > 0.)) Fatal("covariance parameters must be > 0");
  trafo[0] = orig[0];
  trafo[1] = orig[1] / orig[0];
  trafo[2] = range_trafo(cfg_.cov_type, orig[2]);
}

void REModelAMD::SetY(const double* y) {
  // re_model_template.h:5689-5726: y is copied (and permuted into Vecchia order)
  UseDevice();
  const int n = cfg_.n;
  std::vector<double> yv(n);
  if (vecchia_ || vif_) for (int i = 0; i < n; ++i) yv[i] = y[perm_[i]];
  else std::copy(y, y + n, yv.begin());
  if (cfg_.latent) {
    double lognorm = 0.;   // CheckY (likelihoods.h:637-737), CalculateLogNormalizingConstant (:8290-8310)
    if (cfg_.lik == kLikBernoulliLogit || cfg_.lik == kLikBernoulliProbit) {
      for (int i = 0; i < n; ++i)
        if (yv[i] != 0. && yv[i] != 1.)
          Fatal("The response variable ('y') needs to be 0 or 1 for likelihood = '%s' ", cfg_.likelihood.c_str());
    } else if (cfg_.lik == kLikGamma) {   // :668-673; sum log y for the normalizing constant (:8181-8191)
      sum_log_y_ = 0.;
      for (int i = 0; i < n; ++i) {
        if (yv[i] <= 0.)
          Fatal(" Must have y > 0 for the response variable ('y') for likelihood = '%s', found %g ", cfg_.likelihood.c_str(), yv[i]);
        sum_log_y_ += std::log(yv[i]);
      }
    } else if (cfg_.lik == kLikPoisson) {
      for (int i = 0; i < n; ++i) {
        if (yv[i] < 0.) Fatal(" Must have y >= 0 for the response variable ('y') for likelihood = 'poisson', found %g ", yv[i]);
        double ip;
        if (std::modf(yv[i], &ip) != 0.)
          Fatal("Found non-integer response variable ('y'). Response variable can only be integer valued for likelihood = 'poisson' ");
        for (int k = 2; k <= (int)yv[i]; ++k) lognorm -= std::log((double)k);   // LogNormalizingConstantPoissonOneSample
      }
    }
    loglik_const_ = lognorm;
    y_vo_ = yv;
    if (lat()) {
      lat()->SetLogLikConst(loglik_const_);
      lat()->SetY(y_vo_.data());
    }
  }
  d_y_.alloc(n);
  HIP_CHECK(hipMemcpyAsync(d_y_.get(), yv.data(), sizeof(double) * n, hipMemcpyHostToDevice, stream_));
  HIP_CHECK(hipStreamSynchronize(stream_));
  y_set_ = true;
}

void REModelAMD::LaunchVecchiaRows(const double* trafo, int r0, int r1, double* sums, bool allreduce) {
  VecchiaRowsArgs a{};
  a.X = d_X_.get();
  a.Y = d_y_.get();
  a.nbr = d_nbr_.get();
  a.n = cfg_.n;
  a.d = cfg_.d;
  a.m = cfg_.num_neighbors;
  a.r0 = r0;
  a.r1 = r1;
  a.var = trafo[1];
  a.phi = trafo[2];
  a.diag_mult = 1.;   // Gaussian likelihood: nugget 1 on the transformed scale (Vecchia_utils.cpp:1540)
  a.diag_add = 1.;
  a.d_nugget = 1.;
  if (d_block_sums_.size() == 0)   // built as a latent model and switched to the Gaussian likelihood
    d_block_sums_.alloc((size_t)std::max(vecchia_rows_blocks(row_end_ - row_begin_, a.m), 1) * kVecchiaSums);
  a.block_sums = d_block_sums_.get();
  static const int sched = [] {   // A/B of the partial-round schedule (kernels.h VecchiaRowsArgs::sched)
    const char* e = std::getenv("GPBOOST_AMD_ROWS16_SCHED");
    return e ? std::atoi(e) : 0;
  }();
  a.sched = sched;
  int nblocks = 0;   // the launch's grid (<= vecchia_rows_blocks, the buffer size)
  // HIP events cost ~10 us of host time per evaluation (a quarter of the host overhead): recorded
  // only once GetLastKernelTimes has been called
  const bool timing = timing_;
  if (timing) HIP_CHECK(hipEventRecord(ev_[0], stream_));
  nblocks = launch_vecchia_rows(cfg_.cov_type, a, stream_);
  if (timing) HIP_CHECK(hipEventRecord(ev_[1], stream_));
  static const bool sync_wait = std::getenv("GPBOOST_AMD_EVAL_SYNC") != nullptr;   // A/B: stream sync
  if (sync_wait && !(allreduce && coll_ != nullptr)) {
    launch_sum_blocks(d_block_sums_.get(), nblocks, kVecchiaSums, h_sums_dev_, stream_);
    if (timing) HIP_CHECK(hipEventRecord(ev_[2], stream_));
    HIP_CHECK(hipStreamSynchronize(stream_));
  } else {
    // the fixed-order block sum writes the host-coherent buffer directly and then a sequence flag
    // (after a system-scope release); the host spins on the flag instead of synchronising the
    // stream: 0.2448 vs 0.2500 ms per evaluation at one rank (profiles/r03/rows_env_ab_r03k.log).
    // Several ranks: the block sum goes to the device, is all-reduced on the stream, and a one-block
    // pass of the same kernel publishes the reduced sums and the flag.
    unsigned long long* flag = reinterpret_cast<unsigned long long*>(h_sums_dev_ + 8);
    const unsigned long long seq = ++sum_seq_;
    if (allreduce && coll_ != nullptr) {
      launch_sum_blocks(d_block_sums_.get(), nblocks, kVecchiaSums, d_sums_.get(), stream_);
      coll_->AllReduceSum(d_sums_.get(), kVecchiaSums, stream_);
      launch_sum_blocks(d_sums_.get(), 1, kVecchiaSums, h_sums_dev_, stream_, flag, seq);
    } else {
      launch_sum_blocks(d_block_sums_.get(), nblocks, kVecchiaSums, h_sums_dev_, stream_, flag, seq);
    }
    if (timing) HIP_CHECK(hipEventRecord(ev_[2], stream_));
    volatile unsigned long long* hf = reinterpret_cast<volatile unsigned long long*>(h_sums_ + 8);
    for (long spins = 1; *hf != seq; ++spins) {
      if ((spins & ((1 << 16) - 1)) == 0) {   // a failed launch never writes the flag: surface the error
        const hipError_t e = hipStreamQuery(stream_);
        if (e != hipSuccess && e != hipErrorNotReady) HIP_CHECK(e);
        if (e == hipSuccess && *hf != seq) Fatal("row-kernel block sum did not report");
      }
      __builtin_ia32_pause();
    }
    std::atomic_thread_fence(std::memory_order_acquire);
  }
  events_pending_ = timing;   // kernel times are read from the events only when asked for
  std::copy(h_sums_, h_sums_ + kVecchiaSums, sums);
}

void REModelAMD::GetLastKernelTimes(double* ms) {
  timing_ = true;   // evaluations from now on record their kernel events
  if (events_pending_) {
    UseDevice();
    HIP_CHECK(hipEventSynchronize(ev_[2]));   // the evaluation returned on the sum flag, not a stream sync
    float ms0 = 0.f, ms1 = 0.f;
    HIP_CHECK(hipEventElapsedTime(&ms0, ev_[0], ev_[1]));
    HIP_CHECK(hipEventElapsedTime(&ms1, ev_[0], ev_[2]));
    last_kernel_ms_[0] = ms0;
    last_kernel_ms_[1] = ms1;
    events_pending_ = false;
  }
  ms[0] = last_kernel_ms_[0];
  ms[1] = last_kernel_ms_[1];
}

void REModelAMD::EvalVecchia(const double* trafo, double* sums) {
  LaunchVecchiaRows(trafo, row_begin_, row_end_, sums, true);
}

void REModelAMD::EvalVecchiaPartials(const double* cov_pars_orig, int r0, int r1, double* sums) {
  if (!vecchia_) Fatal("model does not use the Vecchia approximation");
  if (cfg_.latent) Fatal("row-range partial sums exist only for the exact Gaussian Vecchia likelihood");
  if (!y_set_) Fatal("response variable y has not been set");
  if (r0 < row_begin_ || r1 > row_end_ || r0 > r1) Fatal("row range [%d, %d) outside this model's rows [%d, %d)", r0, r1, row_begin_, row_end_);
  UseDevice();
  EnsureStructure();
  double trafo[3];
  TransformCovPars(cov_pars_orig, trafo);
  LaunchVecchiaRows(trafo, r0, r1, sums, false);
}

void REModelAMD::EvalExactGaussian(const double* trafo, bool want_grad, double* sums) {
  if (vif_) {
    events_pending_ = false;
    vif_->Eval(cfg_.cov_type, trafo[1], trafo[2], d_y_.get(), want_grad, sums, last_kernel_ms_);
    return;
  }
  if (fitc_) {
    events_pending_ = false;
    fitc_->Eval(cfg_.cov_type, trafo[1], trafo[2], d_y_.get(), want_grad, sums, last_kernel_ms_);
    return;
  }
  EvalDense(trafo, want_grad, sums);
}

const std::vector<double>& REModelAMD::InducingPoints() const {
  if (vif_) return vif_->inducing_points();
  if (!fitc_) Fatal("model does not use gp_approx = 'fitc' or 'full_scale_vecchia'");
  return fitc_->inducing_points();
}

void REModelAMD::EvalDense(const double* trafo, bool want_grad, double* sums) {
  events_pending_ = false;
  dense_->Eval(cfg_.cov_type, trafo[1], trafo[2], d_y_.get(), want_grad, sums, last_kernel_ms_);
}

EvalResult REModelAMD::EvalLatent(const double* cov_pars_orig, bool want_grad) {
  if (!(cov_pars_orig[0] > 0. && cov_pars_orig[1] > 0.)) Fatal("covariance parameters must be > 0");
  // TransformCovPars for non-Gaussian likelihoods: no division by a nugget (cov_fcts.h:438-460)
  const double trafo[2] = {cov_pars_orig[0], range_trafo(cfg_.cov_type, cov_pars_orig[1])};
  EvalResult res = EvalLatentTrafo(trafo, want_grad);
  last_cov_pars_.assign(cov_pars_orig, cov_pars_orig + 2);
  return res;
}

void REModelAMD::ResetLatentModeToPrevious() {
  if (lat()) lat()->ResetModeToPrevious();
}

EvalResult REModelAMD::EvalLatentTrafo(const double* trafo, bool want_grad, bool fatal_on_nan,
                                       LatentVecchia::ModeStart start) {
  if (!y_set_) Fatal("response variable y has not been set");
  UseDevice();
  EnsureStructure();
  lat()->ClearModePrevious();
  const double aux = aux_pars_.empty() ? 1. : aux_pars_[0];
  const bool aux_grad = estimate_aux_pars && !aux_pars_.empty();
  if (cfg_.lik == kLikGamma) {   // LogNormalizingConstantGamma (likelihoods.h:8431-8440): 0 at shape 1 (TwoNumbersAreEqual)
    const double c = std::fabs(aux - 1.) < 1e-10 * std::max({1., std::fabs(aux), 1.})
                         ? 0.
                         : (aux - 1.) * sum_log_y_ + cfg_.n * (aux * std::log(aux) - std::lgamma(aux));
    lat()->SetLogLikConst(c);
  }
  LatentResult r;
  try {
    // fault injection for the tests: the k-th latent evaluation of this model reports NaN
    if (const char* e = std::getenv("GPBOOST_AMD_TEST_NAN_EVAL"))
      if (++test_nan_count_ == std::atoi(e)) throw LatentNan("NaN or Inf occurred (injected by GPBOOST_AMD_TEST_NAN_EVAL)");
    r = lat()->Eval(cfg_.cov_type, cfg_.lik, trafo, aux, iter, want_grad, aux_grad, nullptr, start);
    latent_evaluated_ = true;
  } catch (const LatentNan& e) {
    HIP_CHECK(hipStreamSynchronize(stream_));   // drain what the interrupted evaluation had queued
    if (fatal_on_nan) Fatal("%s", e.what());
    r = LatentResult();   // the line search shrinks the step (LineSearchBacktracking.h:78)
    r.nll = std::numeric_limits<double>::quiet_NaN();
    r.grad.assign(want_grad ? (aux_grad ? 3 : 2) : 0, std::numeric_limits<double>::quiet_NaN());
  }
  if (fatal_on_nan && !std::isfinite(r.nll)) Fatal("NaN or Inf occurred in the approximate negative marginal log-likelihood");
  EvalResult res;
  res.nll = r.nll;
  res.grad = r.grad;
  res.sigma2 = aux;
  last_iter_info_[0] = r.newton_its;
  last_iter_info_[1] = r.cg_its;
  last_iter_info_[2] = r.lanczos_steps;
  last_iter_info_[3] = r.logdet;
  events_pending_ = false;
  last_kernel_ms_[0] = last_kernel_ms_[1] = r.ms_total;
  last_nll_ = res.nll;
  return res;
}

void REModelAMD::BenchLatentOperators(int t, int reps, double* out) {
  if (!cfg_.latent || !latent_) Fatal("BenchLatentOperators needs an evaluated latent Vecchia (iterative) model");
  UseDevice();
  latent_->BenchOperators(t, reps, out);
}

EvalResult REModelAMD::Eval(const double* cov_pars_orig, bool want_grad, int profile) {
  if (!y_set_) Fatal("response variable y has not been set");
  if (cfg_.latent) {
    if (profile) Fatal("profile_sigma2 is only defined for the Gaussian likelihood without 'vecchia_latent'");
    return EvalLatent(cov_pars_orig, want_grad);
  }
  double trafo[3];
  TransformCovPars(cov_pars_orig, trafo);
  EvalResult res = EvalTrafo(trafo, want_grad, profile);
  last_cov_pars_.assign(cov_pars_orig, cov_pars_orig + 3);
  if (profile) last_cov_pars_[0] = res.sigma2;
  return res;
}

EvalResult REModelAMD::EvalTrafo(const double* trafo, bool want_grad, int profile, bool fatal_on_nan) {
  if (!y_set_) Fatal("response variable y has not been set");
  UseDevice();
  EnsureStructure();
  double sums[kVecchiaSums];
  if (vecchia_) EvalVecchia(trafo, sums);
  else EvalExactGaussian(trafo, want_grad, sums);
  if (fatal_on_nan && (!std::isfinite(sums[0]) || !std::isfinite(sums[1])))
    Fatal("NaN or Inf occurred in the negative log-likelihood (non-positive-definite covariance?)");
  EvalResult res;
  res.grad.resize(profile ? 2 : 3);
  combine_partials(sums, cfg_.n, trafo[0], profile, &res.nll, res.grad.data(), &res.sigma2);
  if (!std::isfinite(sums[0]) || !std::isfinite(sums[1])) res.nll = std::numeric_limits<double>::quiet_NaN();
  last_nll_ = res.nll;
  return res;
}

void REModelAMD::GetVecchiaStructure(int* perm, int* nbr) const {
  if (!vecchia_) Fatal("model does not use the Vecchia approximation");
  if (has_dup()) Fatal("GetVecchiaStructure is not available for latent models with repeated coordinates");
  if (world_ > 1) Fatal("GetVecchiaStructure is only available on single-rank models");
  const_cast<REModelAMD*>(this)->UseDevice();
  const_cast<REModelAMD*>(this)->EnsureStructure();
  std::copy(perm_.begin(), perm_.end(), perm);
  std::copy(nbr_.begin(), nbr_.end(), nbr);
}

void REModelAMD::GetLatentVecchiaFactor(const double* cov_pars_orig, double* Dinv, double* Bvals, double* dD,
                                        double* dBvals) {
  if (!cfg_.latent) Fatal("model does not use a latent Vecchia approximation");
  if (world_ > 1) Fatal("GetLatentVecchiaFactor is only available on single-rank models");
  if (has_dup()) Fatal("GetLatentVecchiaFactor is not available for latent models with repeated coordinates");
  if (!(cov_pars_orig[0] > 0. && cov_pars_orig[1] > 0.)) Fatal("covariance parameters must be > 0");
  UseDevice();
  EnsureStructure();
  const int n = cfg_.n, m = cfg_.num_neighbors;
  DevBuf<double> a(n), b((size_t)n * m), c(n), e((size_t)n * m);
  LatentFactorArgs fa{};
  fa.X = d_X_.get(); fa.nbr = d_nbr_.get(); fa.n = n; fa.d = cfg_.d; fa.m = m;
  fa.var = cov_pars_orig[0];
  fa.phi = range_trafo(cfg_.cov_type, cov_pars_orig[1]);
  fa.jitter = 1. + 1e-10;
  fa.Bv = b.get(); fa.dBv = e.get(); fa.Dinv = a.get(); fa.dD = c.get();
  launch_latent_factor(cfg_.cov_type, fa, stream_);
  HIP_CHECK(hipMemcpyAsync(Dinv, a.get(), sizeof(double) * n, hipMemcpyDeviceToHost, stream_));
  HIP_CHECK(hipMemcpyAsync(Bvals, b.get(), sizeof(double) * n * m, hipMemcpyDeviceToHost, stream_));
  HIP_CHECK(hipMemcpyAsync(dD, c.get(), sizeof(double) * n, hipMemcpyDeviceToHost, stream_));
  HIP_CHECK(hipMemcpyAsync(dBvals, e.get(), sizeof(double) * n * m, hipMemcpyDeviceToHost, stream_));
  HIP_CHECK(hipStreamSynchronize(stream_));
}

void REModelAMD::GetVecchiaFactor(const double* cov_pars_orig, double* Dinv, double* Bvals) {
  if (!vecchia_) Fatal("model does not use the Vecchia approximation");
  if (cfg_.latent) Fatal("latent Vecchia model: use GPB_GetLatentVecchiaFactor");
  if (world_ > 1) Fatal("GetVecchiaFactor is only available on single-rank models");
  UseDevice();
  EnsureStructure();
  double trafo[3];
  TransformCovPars(cov_pars_orig, trafo);
  const int n = cfg_.n, m = cfg_.num_neighbors;
  DevBuf<double> dD(n), dB((size_t)n * m);
  VecchiaRowsArgs a{};
  a.X = d_X_.get();
  a.Y = nullptr;
  a.nbr = d_nbr_.get();
  a.n = n; a.d = cfg_.d; a.m = m; a.r0 = 0; a.r1 = n;
  a.var = trafo[1]; a.phi = trafo[2];
  a.diag_mult = 1.; a.diag_add = 1.; a.d_nugget = 1.;
  a.Dinv_out = dD.get();
  a.B_out = dB.get();
  launch_vecchia_rows(cfg_.cov_type, a, stream_);
  HIP_CHECK(hipMemcpyAsync(Dinv, dD.get(), sizeof(double) * n, hipMemcpyDeviceToHost, stream_));
  HIP_CHECK(hipMemcpyAsync(Bvals, dB.get(), sizeof(double) * n * m, hipMemcpyDeviceToHost, stream_));
  HIP_CHECK(hipStreamSynchronize(stream_));
}

void combine_partials(const double* s, int n, double sigma2_in, int profile, double* nll, double* grad,
                      double* sigma2_out) {
  // s = [logdet, q, s1_var, s1_range, s2_var, s2_range]
  const double logdet = s[0], q = s[1];
  const double sigma2 = profile ? q / n : sigma2_in;          // ProfileOutSigma2 (re_model_template.h:2407)
  *nll = q / 2. / sigma2 + logdet / 2. + n / 2. * (std::log(sigma2) + std::log(2 * M_PI));  // :2880, :2890
  int off = 0;
  if (!profile) { grad[0] = -q / sigma2 / 2. + n / 2.; off = 1; }  // :1774 / :1806
  grad[off + 0] = s[2] / sigma2 + 0.5 * s[4];                    // :1786-1787 / :1813-1814
  grad[off + 1] = s[3] / sigma2 + 0.5 * s[5];
  if (sigma2_out) *sigma2_out = sigma2;
}

void REModelAMD::CholeskyPlanInfo(double* out) {
  if (!vif_lap_ && (!(cfg_.latent && vecchia_) || cfg_.matrix_inversion_method != "cholesky"))
    Fatal("GPB_GetCholeskyPlanInfo needs a latent Vecchia or full-scale Vecchia model with matrix_inversion_method = "
          "'cholesky'");
  UseDevice();
  EnsureStructure();
  const CholPlan* p = vif_lap_ ? &vif_lap_->plan() : latent_->CholPlanInfo();
  out[0] = p->nsup;
  out[1] = (double)p->lvl_ptr.size() - 1;
  out[2] = (double)p->nnz_l;
  out[3] = (double)p->front_doubles;
  out[4] = p->flops;
  out[5] = p->max_fs;
  out[6] = p->max_ns;
  out[7] = p->ms_analyze;
  out[8] = vif_lap_ ? vif_lap_->last_factor_ms() : latent_->CholLastFactorMs();
}

}  // namespace gpb_amd
