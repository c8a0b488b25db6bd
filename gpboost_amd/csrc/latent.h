// LatentVecchia: the latent-GP Vecchia likelihood with iterative methods on one GPU.
//
// Replaces, for one GP component in Vecchia order, the reference's
//   FindModePostRandEffCalcMLLVecchia      likelihoods.h:2765-3076   (Newton + PCG + Armijo)
//   CalcLogDetStochVecchia (vadu)          likelihoods.h:12069-12212 (SLQ log-determinant)
//   CalcGradNegMargLikelihoodLaplaceApproxVecchia (iterative, vadu)
//                                          likelihoods.h:4951-5206, 12225-12546
//   CGVecchiaLaplaceVec / CGTridiagVecchiaLaplace / GenRandVecNormalParallel
//                                          CG_utils.cpp:21-217, 930-1041
// for likelihood "gaussian" under gp_approx = "vecchia_latent" (aux par = error variance)
// and "bernoulli_logit". Every O(n) / O(n m) / O(n m t) step is a HIP kernel on the
// model's stream; the host runs the iteration logic (stopping tests, line search) and
// the O(t k^2) tridiagonal eigenproblems, exactly where the reference branches.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <map>
#include <memory>
#include <cmath>
#include <stdexcept>
#include <random>
#include <vector>

#include "common.h"
#include "collective.h"
#include "latent_kernels.h"
#include "vadu_precond.h"
#include "sparse_chol.h"

namespace gpb_amd {

struct IterativeConfig {
  int cg_max_num_it = 1000;                // re_model_template.h:5364
  int cg_max_num_it_tridiag = 1000;        // :5366
  double cg_delta_conv = 1e-2;             // :5368
  int num_rand_vec_trace = 50;             // :5376
  int seed_rand_vec_trace = 1;             // :5380
  bool reuse_rand_vec_trace = true;
  double delta_conv_mode_finding = 1e-8;   // likelihoods.h:12723
};

// NaN / Inf in the mode finding or a CG solve of an evaluation. The reference sets the approximate
// marginal log-likelihood to NaN and returns (likelihoods.h:2929-2933, 2997-3000), so an L-BFGS line
// search shrinks the step (LineSearchBacktracking.h:78); REModelAMD turns this into nll = NaN when
// its caller tolerates it and into a fatal error otherwise.
// digamma by the asymptotic expansion after recurrence to x >= 8.5 (Bernardo 1976, Algorithm AS 103; the form the
// reference's GPBoost::digamma uses, DF_utils.cpp:82-123)
inline double digamma_asa103(double x) {
  if (x <= 0.000001) return -0.57721566490153286060 - 1.0 / x + 1.6449340668482264365 * x;
  double value = 0., x2 = x;
  while (x2 < 8.5) {
    value = value - 1.0 / x2;
    x2 = x2 + 1.0;
  }
  double r = 1.0 / x2;
  value = value + std::log(x2) - 0.5 * r;
  r = r * r;
  return value - r * (1.0 / 12.0 - r * (1.0 / 120.0 - r * (1.0 / 252.0 - r * (1.0 / 240.0 - r * (1.0 / 132.0)))));
}

struct LatentNan : std::runtime_error {
  using std::runtime_error::runtime_error;
};

struct LatentResult {
  double nll = 0.;
  std::vector<double> grad;   // [d/dlog sigma1^2, d/dlog phi, (gaussian, if requested) d/dlog aux]
  int newton_its = 0, cg_its = 0, lanczos_steps = 0;
  double logdet = 0.;         // log|Sigma W + I|
  double ms_total = 0.;       // device time of the whole evaluation (HIP events)
};

// What REModelAMD needs from a latent (Laplace) solver, whatever the approximation: LatentVecchia
// (gp_approx = "vecchia", iterative) and FitcLaplace (gp_approx = "fitc", Cholesky; fitc_laplace.h).
// Host vectors are in the model's internal order (Vecchia order / the original order for FITC).
class LatentSolverBase {
 public:
  // start: where the Newton iterations begin (FindModePostRandEffCalcMLL*, likelihoods.h):
  //   kZero  the mode re-initialised to 0 (InitializeModeAvec: GPB_EvalNegLogLikelihood, predictions);
  //   kWarm  from the previous evaluation (the L-BFGS objective: mode_initialized_ stays true), kept for
  //          ResetModeToPrevious;
  //   kKeep  no mode finding: the factor, W and log-determinant at the current mode (CalcGradientF with
  //          calc_cov_factor = false, re_model_template.h:3021-3043).
  enum class ModeStart { kZero, kWarm, kKeep };
  virtual ~LatentSolverBase() = default;
  virtual void SetY(const double* y) = 0;
  virtual void SetOffset(const double* off) = 0;   // NULL: none
  virtual void GetMode(double* mode) = 0;
  virtual LatentResult Eval(int cov_type, int lik, const double* trafo, double aux, const IterativeConfig& cfg,
                            bool want_grad, bool want_aux_grad, double* grad_f = nullptr,
                            ModeStart start = ModeStart::kZero) = 0;
  virtual void ResetModeToPrevious() = 0;
  virtual void ClearModePrevious() = 0;
  // the log-likelihood's normalizing constant (e.g. -sum log y! for poisson, CalculateLogNormalizingConstant
  // likelihoods.h:8290-8310), part of the mode-finding objective and of the marginal likelihood
  void SetLogLikConst(double c) { loglik_const_ = c; }

 protected:
  double loglik_const_ = 0.;
};

class LatentVecchia : public LatentSolverBase {
 public:
  // d_X: coordinates (Vecchia order, row-major n x d) on the device, owned by the caller.
  // nbr: host n x m neighbour table (row i holds min(i, m) entries).
  LatentVecchia(int n, int d, int m, const double* d_X, const int* nbr, hipStream_t stream);
  ~LatentVecchia();

  // Repeated coordinates (the reference's unique-location form, Vecchia_utils.cpp:1121-1139): the
  // latent variables are the n unique locations and obs_row[i] is the latent Vecchia row of
  // observation i (observations in the model's Vecchia-shuffled order). SetY / SetOffset then take
  // one value per observation (that order); the likelihood terms of a latent variable are sums over
  // its observations.
  void SetObservations(const std::vector<int>& obs_row);
  void SetY(const double* y_vo) override;   // host, Vecchia order (per observation after SetObservations)
  // Posterior mode of the last evaluation (host, Vecchia order).
  void GetMode(double* mode_vo) override;
  // Fixed effects F of the location parameter (host, Vecchia order; NULL: none). The likelihood is
  // evaluated at mode + F (InitializeLocationPar, likelihoods.h).
  void SetOffset(const double* off_vo) override;

  // trafo = (sigma1^2, phi). aux = gaussian error variance (ignored for bernoulli_logit).
  // grad_f_vo (host, Vecchia order, nullable; needs want_grad): gradient wrt the fixed effects F
  // (CalcGradNegMargLikelihoodLaplaceApproxVecchia calc_F_grad, likelihoods.h:5337-5367).
  // start (LatentSolverBase::ModeStart; FindModePostRandEffCalcMLLVecchia, likelihoods.h:2782-2789): kWarm
  // continues from the previous mode (mode_previous_value_ = mode_). The Gaussian likelihood's single
  // Newton step does not depend on the start.
  LatentResult Eval(int cov_type, int lik, const double* trafo, double aux, const IterativeConfig& cfg,
                    bool want_grad, bool want_aux_grad, double* grad_f_vo = nullptr,
                    ModeStart start = ModeStart::kZero) override;
  // Likelihood::ResetModeToPreviousValue (likelihoods.h:528-535): the mode at the start of the last
  // kWarm evaluation back (no-op when no such evaluation started since ClearModePrevious).
  void ResetModeToPrevious() override;
  void ClearModePrevious() override { mode_prev_valid_ = false; }

  // Operator costs on the factor of the last evaluation (benchmark roofline): out[0] = ms per
  // A = B^T D^-1 B + W application, out[1] = ms per VADU preconditioner application (both on
  // t columns, averaged over reps, HIP events on the model's stream), out[2] = nnz(B) incl.
  // the unit diagonal, out[3] = dependent launches per preconditioner application.
  void BenchOperators(int t, int reps, double* out);

  // Predictive-variance simulation of PredictLaplaceApproxVecchia (likelihoods.h:6628-6746,
  // iterative): nsim draws z ~ N(0, (Sigma^-1 + W)^-1), each the solution of (Sigma^-1 + W) z =
  // B^T D^-1/2 e1 + W^1/2 e2 by the VADU-preconditioned CG (own stopping rule ||r|| < delta per draw,
  // as CGVecchiaLaplaceVec), t draws per block of independent columns; returns acc[p] = sum over the
  // draws of (Bpo z)_p^2 (host, n_pred). Uses the factor, W and preconditioner of the last Eval.
  // nbr_vo: host n_pred x mp neighbour indices (latent Vecchia rows), d_Bpo: device n_pred x mp.
  // d_V (nullable, device n_pred x nsim column-major): the draws Bpo z themselves (predictive
  // covariance, cond_all); acc (nullable) as before. ref_gen (nullable): draw the reference's one-thread
  // stream from this generator on the host instead of the counter-based GPU draws.
  void PredVarSim(int nsim, int t, double delta, int cg_max, uint64_t seed, int n_pred, int mp, const int* nbr_vo,
                  const double* d_Bpo, double* acc, double* d_V = nullptr, std::mt19937* ref_gen = nullptr);

  // Probe-column sharding (SURVEY.md §8e Option A): rank r of `world` runs the probe columns
  // [t r / world, t (r+1) / world) of every SLQ block — padded to ceil(t / world) columns, so
  // every rank's blocks have the same width and the replicated Newton / mode columns are
  // computed bitwise alike on every rank — with one all-reduce per PCG iteration (the block
  // stopping rule's norm sum) and the per-column log-determinant / trace terms and the
  // mode-derivative row moments all-reduced at the end. coll: owned by the caller; null at
  // world 1.
  void SetShard(int rank, int world, Collective* coll);

  // matrix_inversion_method = "cholesky" (latent_chol.cpp): Eval runs the reference's exact Laplace-Vecchia
  // branch on the GPU sparse Cholesky of Sigma^-1 + W (sparse_chol.h) instead of PCG / SLQ. The plan is
  // built at the first evaluation; CholPlanInfo builds it on demand (statistics).
  void SetCholesky(bool on);
  bool cholesky() const { return use_chol_; }
  const CholPlan* CholPlanInfo();
  float CholLastFactorMs() { return chol_ ? chol_->last_factor_ms() : 0.f; }
  // Cholesky predictive-variance terms (likelihoods.h:6751-6811) on the factor of the last evaluation:
  // d_V (device n_pred x n column-major) = sqrt(n) (L^-1 P Bpo^T)^T, for latent_pred_moments with nsim = n.
  // nbr_vo: host n_pred x mp neighbour indices (latent Vecchia rows; >= n: none), d_Bpo device n_pred x mp.
  void PredVarChol(int n_pred, int mp, const int* nbr_vo, const double* d_Bpo, double* d_V);

 private:
  // Device work space of a t-column PCG (t = 1 for the Newton solves, t probes for SLQ).
  struct Block {
    int t = 0;
    DevBuf<double> R, Z, H, V, G, Xt;     // n x t
    DevBuf<double> small;                 // rz, rz_new, hv, rr, a, b: 6 x t
    DevBuf<double> a_hist, b_hist;        // pmax x t (CG coefficients per iteration)
    DevBuf<int> act;                      // per-column activity mask
    DevBuf<int> ctl;                      // PcgCtl (device side of the stopping rule)
    double* rz() const { return small.get(); }
    double* rz_new() const { return small.get() + t; }
    double* hv() const { return small.get() + 2 * t; }
    double* rr() const { return small.get() + 3 * t; }
    double* a() const { return small.get() + 4 * t; }
    double* b() const { return small.get() + 5 * t; }
  };

  LatentResult EvalChol(int cov_type, int lik, const double* trafo, double aux, const IterativeConfig& cfg,
                        bool want_grad, bool want_aux_grad, double* grad_f_vo, ModeStart start);
  void EnsureChol();
  bool use_chol_ = false;
  std::unique_ptr<SparseChol> chol_;
  DevBuf<double> d_diagS_;
  std::vector<int> obs_cnt_;   // observations per storage row (repeated coordinates)
  void Relabel(const int* nbr, std::vector<int>& nbr_p);   // storage order for locality
  void BuildStructure(const int* nbr);
  Block& GetBlock(int which, int t, int pmax);
  void EnsureProbes(const IterativeConfig& cfg);
  void ApplyA(const double* H, double* V, double* G, int t);
  void Precond(const double* R, double* Z, double* Xt, int t);
  void SetDiag();   // the preconditioner's D^-1 + W changed (after every newton_prep writing dw)
  // PCG on the b.t columns of RHS sharing every operator application. Columns [0, n_single)
  // are independent single-vector CGs (CG_utils.cpp:21-108: own ||r|| < delta, warm start
  // allowed when t == 1); columns [n_single, t) are the block of CGTridiagVecchiaLaplace
  // (:110-217: mean ||r|| < delta). Stopped columns are frozen (a = b = 0). The per-
  // iteration coefficients land in b.a_hist / b.b_hist (Lanczos tridiagonals). The stopping
  // rule runs on the device (pcg_check); the host reads its verdict one preconditioner
  // application behind, so the queue never drains between iterations.
  struct PcgResult {
    int its_single = 0, its_block = 0;
    bool nan = false, zero_rhs = false;
  };
  // n_valid: columns >= n_valid are padding (never active); nblock_all: the block's column count
  // over all ranks (> 0 with a collective: the block rule uses the all-reduced norm sum).
  PcgResult Pcg(Block& b, const double* RHS, double* U, int n_single, bool init_zero, bool u_is_zero,
                int pmax_single, int pmax_block, double delta, int n_valid = -1, int nblock_all = 0);
  // Sum of a host vector over ranks (identity at world 1).
  void AllReduceHost(double* v, int count);
  int probe_cols() const { return world_ > 1 ? (t_all_ + world_ - 1) / world_ : t_all_; }
  void Scalars(const ScalarArgs& a, double* out);
  double Dot1(const double* x, const double* y);   // single-vector dot, synchronous
  void WaitCtl(int seq, int* out);

  int n_, d_, m_;
  const double* d_X_;
  hipStream_t s_;
  std::vector<int> vo_, lab_;   // storage row p holds Vecchia row vo_[p]; lab_ = inverse
  DevBuf<double> d_Xp_;         // coordinates in storage order
  DevBuf<double> d_tval_;       // B values in transposed-list order (refreshed per evaluation)
  int tnnz_ = 0;
  SparseB sp_{};
  DevBuf<int> d_nbr_, d_tptr_, d_trow_, d_tslot_, d_longr_;
  DevBuf<int> d_ell_idx_, d_ell_slot_, d_seg_rb_;
  DevBuf<uint32_t> d_seg_pk_;
  DevBuf<int4> d_seg_info_;
  DevBuf<uint32_t> d_seg_pk2_;
  DevBuf<int> d_seg_slot2_;
  DevBuf<double> d_seg_val2_;
  int seg2_n_ = 0;
  struct TileDev {   // device arrays of a TileOp
    DevBuf<int> r0, uoff, urow, fb;
    DevBuf<uint16_t> lidx;
    DevBuf<unsigned char> isfb;
    TileOp op{};
  };
  TileDev tile_b_, tile_bt_;
  DevBuf<double> d_ell_val_;
  int dense_rows_ = 0, head_rows_ = 0;   // VADU plan split (VaduPrecond)
  std::unique_ptr<VaduPrecond> pre_;
  DevBuf<double> d_y_, d_Bv_, d_dBv_, d_Dinv_, d_dD_, d_W_, d_dw_, d_sdw_, d_d1_;
  double sum_log_y_ = 0.;   // likelihood 'gamma
  DevBuf<double> d_mode_, d_mode_upd_, d_mode_new_, d_rhs_, d_dir_, d_Adir_, d_vS_, d_dmll_;
  DevBuf<double> d_mode_prev_;   // mode_previous_value_ (kWarm evaluations)
  bool mode_prev_valid_ = false;
  DevBuf<double> d_probes_, d_Zp_, d_U_, d_P_;   // n x t
  DevBuf<double> d_rhsf_, d_Uf_;                 // n x (1 + t): mode column fused with the probes (gaussian)
  int probes_t_ = 0;
  uint64_t probe_run_id_ = 0;                    // cg_generator_counter_ (likelihoods.h:12800)
  bool probes_saved_ = false;
  DevBuf<double> d_partials_, d_out_;
  double* h_out_ = nullptr;                      // pinned
  std::unique_ptr<Block> blk1_, blkt_, blkb_;   // blkb_: BenchOperators
  int* h_ctl_ = nullptr;                         // host-coherent verdict words written by pcg_check (2 x 64 bit)
  int* d_hctl_ = nullptr;                        // their device address
  int pcg_seq_ = 0;
  hipEvent_t ev0_ = nullptr, ev1_ = nullptr;
  int rank_ = 0, world_ = 1;
  Collective* coll_ = nullptr;
  int t_all_ = 0, c0_ = 0, c1_ = 0;              // probes of all ranks; this rank's [c0_, c1_)
  DevBuf<double> d_gsum_, d_red_, d_mom_, d_mom2_;
  bool y_set_ = false;
  bool factor_ready_ = false;
  DevBuf<double> d_off_, d_gradf_;   // fixed effects (storage order), gradient wrt F
  bool has_off_ = false;
  // observations of the latent variables (repeated coordinates): storage-row-major lists
  bool has_obs_ = false;
  int n_obs_ = 0;
  std::vector<int> obs_order_;        // position e of the lists -> observation index
  DevBuf<int> d_optr_;                // n + 1
  DevBuf<double> d_yo_, d_offo_;      // n_obs
  ObsMap Obs() const;
};

}  // namespace gpb_amd
