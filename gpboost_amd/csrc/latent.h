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
#include <vector>

#include "common.h"
#include "latent_kernels.h"

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

struct LatentResult {
  double nll = 0.;
  std::vector<double> grad;   // [d/dlog sigma1^2, d/dlog phi, (gaussian, if requested) d/dlog aux]
  int newton_its = 0, cg_its = 0, lanczos_steps = 0;
  double logdet = 0.;         // log|Sigma W + I|
  double ms_total = 0.;       // device time of the whole evaluation (HIP events)
};

class LatentVecchia {
 public:
  // d_X: coordinates (Vecchia order, row-major n x d) on the device, owned by the caller.
  // nbr: host n x m neighbour table (row i holds min(i, m) entries).
  LatentVecchia(int n, int d, int m, const double* d_X, const int* nbr, hipStream_t stream);
  ~LatentVecchia();

  void SetY(const double* y_vo);   // host, Vecchia order

  // trafo = (sigma1^2, phi). aux = gaussian error variance (ignored for bernoulli_logit).
  LatentResult Eval(int cov_type, int lik, const double* trafo, double aux, const IterativeConfig& cfg,
                    bool want_grad, bool want_aux_grad);

  // Operator costs on the factor of the last evaluation (benchmark roofline): out[0] = ms per
  // A = B^T D^-1 B + W application, out[1] = ms per VADU preconditioner application (both on
  // t columns, averaged over reps, HIP events on the model's stream), out[2] = nnz(B) incl.
  // the unit diagonal, out[3] = level sets of the two triangular solves.
  void BenchOperators(int t, int reps, double* out);
  int num_levels_fwd() const { return (int)fptr_.size() - 1; }
  int num_levels_bwd() const { return (int)bptr_.size() - 1; }

 private:
  // Device work space of a t-column PCG (t = 1 for the Newton solves, t probes for SLQ).
  struct Block {
    int t = 0;
    DevBuf<double> R, Z, H, V, G, Xt;     // n x t
    DevBuf<double> small;                 // rz, rz_new, hv, rr, a, b: 6 x t
    DevBuf<double> a_hist, b_hist;        // pmax x t (CG coefficients per iteration)
    DevBuf<int> act;                      // per-column activity mask
    double* rz() const { return small.get(); }
    double* rz_new() const { return small.get() + t; }
    double* hv() const { return small.get() + 2 * t; }
    double* rr() const { return small.get() + 3 * t; }
    double* a() const { return small.get() + 4 * t; }
    double* b() const { return small.get() + 5 * t; }
  };

  void Relabel(const int* nbr, std::vector<int>& nbr_p);   // storage order for locality
  void BuildStructure(const int* nbr);
  Block& GetBlock(int which, int t, int pmax);
  void EnsureProbes(const IterativeConfig& cfg);
  void ApplyA(const double* H, double* V, double* G, int t);
  void Precond(const double* R, double* Z, double* Xt, int t);
  void PrecondImpl(const double* R, double* Z, double* Xt, int t);
  // PCG on the b.t columns of RHS sharing every operator application. Columns [0, n_single)
  // are independent single-vector CGs (CG_utils.cpp:21-108: own ||r|| < delta, warm start
  // allowed when t == 1); columns [n_single, t) are the block of CGTridiagVecchiaLaplace
  // (:110-217: mean ||r|| < delta). Stopped columns are frozen (a = b = 0). The per-
  // iteration coefficients land in b.a_hist / b.b_hist (Lanczos tridiagonals).
  struct PcgResult {
    int its_single = 0, its_block = 0;
    bool nan = false, zero_rhs = false;
  };
  PcgResult Pcg(Block& b, const double* RHS, double* U, int n_single, bool init_zero, bool u_is_zero,
                int pmax_single, int pmax_block, double delta);
  void Scalars(const ScalarArgs& a, double* out);
  double Dot1(const double* x, const double* y);   // single-vector dot, synchronous
  void CheckSolveError();

  int n_, d_, m_;
  const double* d_X_;
  hipStream_t s_;
  std::vector<int> vo_, lab_;   // storage row p holds Vecchia row vo_[p]; lab_ = inverse
  DevBuf<double> d_Xp_;         // coordinates in storage order
  DevBuf<double> d_tval_;       // B values in transposed-list order (refreshed per evaluation)
  int tnnz_ = 0;
  SparseB sp_{};
  DevBuf<int> d_nbr_, d_tptr_, d_trow_, d_tslot_, d_longr_;
  // step plan of the two VADU triangular solves (see SweepPlan)
  std::vector<int> fptr_, bptr_;           // level pointers (host, diagnostics)
  SweepPlan plan_{};
  DevBuf<int> d_blob_, d_vpos_, d_eslot_;
  int plan_entries_ = 0;
  // level-by-level form replayed as hipGraphs (one per (R, Y, Z, t) buffer set)
  LevelPlan lplan_{};
  DevBuf<int> d_crit_;
  std::vector<int> h_crit_;
  unsigned long long* prof_ = nullptr;   // diagnostics: flow-kernel timestamps
  DevBuf<int> d_lrows_, d_beoff_, d_beidx_, d_fidx_, d_lslot_;
  DevBuf<double> d_lval_;
  int lplan_entries_ = 0;
  struct GraphEntry { const void* key[3]; int t; hipGraphExec_t exec; };
  std::vector<GraphEntry> graphs_;
  bool use_graph_ = true;
  // 0 = sync-free flow kernels, 1 = level graphs, 2 = sweep, 3 = sync-free resident waves,
  // 4 = head/tail split (head kernels + tail level graphs)
  int precond_mode_ = 4;
  // head/tail plan (BuildHeadPlan): tail level plan, the two head solves, the B^T partial
  LevelPlan tplan_{};
  HeadSolve hlow_{}, hbt_{};
  HeadPartial hpart_{};
  DevBuf<int> d_hint_, d_hslot_;
  DevBuf<double> d_hval_;
  int hslot_count_ = 0, head_K_ = 0, head_passes_ = 0;
  std::vector<GraphEntry> hgraphs_;
  // tile-blocked tail (launch_vadu_tile): superstep -> item ranges of the two solves
  bool tail_tiles_ = false;
  std::vector<int> sup_b_, sup_f_;
  const int* d_items_ = nullptr;   // inside d_hint_
  void TailSolve(bool lower, const double* R, double* Xt, double* Z, int t);
  void BuildHeadPlan(const int* nbr, const std::vector<int>& tptr, const std::vector<int>& trow,
                     const std::vector<int>& tslot, const std::vector<int>& lb);
  int max_flow_blocks_ = 512;
  int sf_grid_ = 256;                            // precond_mode_ 3: resident single-wave workgroups
  DevBuf<int> d_err_;
  void BuildSweepPlan(const int* nbr, const std::vector<int>& tptr, const std::vector<int>& trow,
                      const std::vector<int>& tslot, const std::vector<int>& lf, const std::vector<int>& lb);
  DevBuf<double> d_y_, d_Bv_, d_dBv_, d_Dinv_, d_dD_, d_W_, d_dw_, d_sdw_, d_d1_;
  DevBuf<double> d_mode_, d_mode_upd_, d_mode_new_, d_rhs_, d_dir_, d_Adir_, d_vS_, d_dmll_;
  DevBuf<double> d_probes_, d_Zp_, d_U_, d_P_;   // n x t
  DevBuf<double> d_rhsf_, d_Uf_;                 // n x (1 + t): mode column fused with the probes (gaussian)
  int probes_t_ = 0;
  uint64_t probe_run_id_ = 0;                    // cg_generator_counter_ (likelihoods.h:12800)
  bool probes_saved_ = false;
  DevBuf<double> d_partials_, d_out_;
  double* h_out_ = nullptr;                      // pinned
  std::vector<double> h_rr_;
  std::unique_ptr<Block> blk1_, blkt_, blkb_;   // blkb_: BenchOperators
  hipEvent_t ev0_ = nullptr, ev1_ = nullptr;
  bool y_set_ = false;
  bool factor_ready_ = false;
};

}  // namespace gpb_amd
