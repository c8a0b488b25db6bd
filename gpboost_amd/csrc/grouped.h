// GroupedRE: Gaussian likelihood with grouped (crossed) random effects on one GPU — BASELINE
// config 4's engine (the reference's expressible proxy is crossed grouped random
// effects with iterative methods).
//
// Model (transformed scale, sigma^2 factored out): Psi = Z Sigma Z^T + I, Sigma = diag(tau_k I_{m_k})
// for K grouping variables with m_k levels, tau_k = sigma_k^2 / sigma^2. Woodbury form of the
// reference (re_model_template.h:8560-8598, 2780-2872, 8985-9003, 2242-2391):
//   A = Sigma^-1 + Z^T Z (M x M, M = sum m_k), y^T Psi^-1 y = y^T y - (Z^T y)^T A^-1 Z^T y,
//   log|Psi| = log|A| + sum_k m_k log tau_k.
// K >= 2 ("iterative", the reference's default there): A^-1 Z^T y by PCG with the SSOR
// preconditioner P = L D^-1 L^T (L = lower triangle of A, D = diag(A); CGRandomEffectsVec,
// CG_utils.cpp:1100-1230), log|A| by stochastic Lanczos quadrature on t probe vectors drawn from
// N(0, P) (CGTridiagRandomEffects :1232-1400, LogDetStochTridiag :988-1004) plus log|P| = sum log D,
// and the gradient by stochastic traces with the SSOR variance reduction (CalcOptimalC :1006).
// K == 1: A is diagonal and everything is closed-form (the reference's Cholesky branch).
// K >= 2 "cholesky" (:8571-8598, the reference's sparse SimplicialLLT): A assembled DENSE in HBM
// (M x M column-major; the integer counts of Z^T Z are exact in any order) and factored on the
// dense path's MFMA POTRF / TRTRI (chol_lower / trtri_lower): log|A| = 2 sum log L_ii, u = A^-1 Z^T y
// by the two triangular products of the inverse factor, and the traces from diag(A^-1):
// tr(Psi^-1 dPsi_k) = m_k - tr(A^-1_kk) / tau_k (the reference's tau_k (||Z_k||^2 - ||L^-1 Z^T Z_k||^2),
// :2279-2296, without its cancellation). Posterior variances of the levels: diag(A^-1).
//
// Data layout in HBM: Z^T Z as its diagonal `cnt` (M) and its off-diagonal part in CSR over RE rows
// (columns ascending: the entries of lower effects first, `split` marks the first entry of a
// higher effect); observation lists per RE level (for Z^T y). Every per-iteration vector is M-long
// (t columns row-major M x t): after Z^T y the n observations never enter an iteration.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <map>
#include <memory>
#include <vector>

#include "common.h"
#include "grouped_kernels.h"
#include "latent.h"

namespace gpb_amd {

struct GroupedParts {
  double yTPsiInvy = 0.;          // y^T Psi^-1 y (transformed scale)
  double logdet = 0.;             // log|Psi|
  std::vector<double> quad;       // per effect: tau_k ||Z_k^T (y - Z A^-1 Z^T y)||^2 (= y^T Psi^-1 dPsi_k Psi^-1 y)
  std::vector<double> trace;      // per effect: tr(Psi^-1 dPsi_k) (stochastic for K >= 2)
  int cg_its = 0, lanczos_steps = 0;
};

class GroupedRE {
 public:
  // levels: K x n, levels[k][i] = level index (0 .. m_k - 1, order of first appearance) of
  // observation i for effect k.
  GroupedRE(int n, const std::vector<std::vector<int>>& levels, hipStream_t s);
  ~GroupedRE();
  GroupedRE(const GroupedRE&) = delete;
  GroupedRE& operator=(const GroupedRE&) = delete;

  int K() const { return K_; }
  int M() const { return M_; }
  const std::vector<int>& levels_per_effect() const { return m_; }
  void SetY(const double* y);   // host, observation order
  // tau: K transformed variances. iterative: SSOR-PCG + SLQ (K >= 2), else closed form (K == 1).
  // warm: start the A^-1 Z^T y solve from the previous solution (the reference does so once the
  // optimizer's iteration counter is > 0, re_model_template.h:8975-8981).
  void Eval(const double* tau, bool want_grad, bool iterative, bool warm, const IterativeConfig& cfg,
            GroupedParts& out);
  bool has_solution() const { return u_valid_; }
  // Posterior means of the M random effects (host, effect-major): tau_k Z_k^T Psi^-1 y; var
  // (nullable, K == 1 only): their posterior variances on the transformed scale.
  void Blup(const double* tau, bool iterative, bool warm, const IterativeConfig& cfg, double* b, double* var);
  // After Blup (cholesky): the e_p^T A^-1 e_q part of the predictive (co)variances on the transformed scale,
  // e_p the indicator vector of prediction point p's seen levels (idx: np x K global level indices, -1 for
  // a level not in the training data). want_cov: out = np x np column-major, else out = np variances.
  // Derivation: Cov = U - Ztilde Sigma Z^T Z Sigma Ztilde^T + Ztilde Sigma Z^T Z A^-1 Z^T Z Sigma Ztilde^T
  // (re_model_template.h:10350-10358, 10510-10522) with Z^T Z = A - Sigma^-1 collapses to
  // U - sum_k tau_k [same seen level] + e_p^T A^-1 e_q. K >= 2: E = Li [e_p] on the device (one wave per
  // point), variances ||E_p||^2, covariances E^T E on the MFMA GEMM; K == 1: A^-1 = diag(1/D).
  void PredCov(int np, const std::vector<int>& idx, bool want_cov, double* out);
  // Fisher information of the original-scale parameters [sigma^2, sigma_1^2 .. sigma_K^2] (cholesky;
  // CalcFisherInformation_Only_Grouped_REs_Woodbury re_model_template.h:9559-9651 with transf_scale =
  // false): with B = S^1/2 A^-1 S^1/2 (S = Sigma^-1 on the transformed scale), F_jk = ||B_jk||_F^2 and
  // t_j = tr(B_jj), Z_j^T Psi^-1 Z_k = S^1/2 (delta_jk I - B_jk) S^1/2 and Psi^-1 Z = Z A^-1 S give
  //   2 sigma^4 FI_00 = n - M + sum_jk F_jk,  2 sigma^4 FI_0j = (t_j - sum_k F_jk) / tau_j,
  //   2 sigma^4 FI_jk = (F_jk + delta_jk (m_j - 2 t_j)) / (tau_j tau_k).
  // Factors A at tau first. FI: (1 + K)^2 row-major.
  void Fisher(const double* tau, double sigma2, double* FI);
  // the pieces of both forms: F (K x K, F_jk = ||B_jk||_F^2) and t_j = tr(B_jj)
  void FisherParts(const double* tau, std::vector<double>& F, std::vector<double>& tr);

 private:
  struct Block {   // work space of a t-column PCG
    int t = 0;
    DevBuf<double> R, Z, H, V, U, S;   // M x t
    DevBuf<double> small;              // rz, rz_new, hv, rr, a, b: 6 x t
    DevBuf<double> a_hist, b_hist;
  };
  Block& GetBlock(int which, int t, int pmax);
  void CheckMethod(const double* tau, bool iterative) const;
  int SolveU(bool iterative, bool warm, const IterativeConfig& cfg, double* single_sums);
  // Chunk plans of the off-diagonal entries for one lane split tc (grouped_kernels.h)
  struct ChunkPlan {
    DevBuf<int> e0[3], e1[3], ptr[3];   // full, lower, upper
    int n[3] = {0, 0, 0};
    std::vector<int> lower_q, upper_q;  // K + 1 chunk boundaries of each effect's rows
  };
  const ChunkPlan& Plan(int tc);
  GroupedOp Op(int t);
  void Diag(const double* tau);                              // D, sqrt(D), per-effect sums of log D and 1/D
  // K >= 2 cholesky: A dense, its Cholesky factor, log|A| (dense_logdet_), the inverse factor Li (dW_)
  // and its transpose (dLiT_), diag(A^-1) (d_invdiag_); u = A^-1 Z^T y
  void DenseFactor();
  int ldM_ = 0;
  double dense_logdet_ = 0.;
  DevBuf<double> dA_, dW_, dLiT_, dX_, d_invdiag_, d_tmpM_;
  DevBuf<int> d_info_;
  void ApplyA(const double* X, double* Y, int t, bool with_sigma_inv);
  void Precond(const double* R, double* Z, double* S, int t); // Z = P^-1 R (S: scratch)
  // Reference PCG forms: single column (stop on ||r|| < delta) or block (stop on the mean column
  // norm, Lanczos coefficients recorded). Returns the iterations run; nan -> Fatal.
  // warm (single column only): U holds the initial guess, R = RHS - A U.
  int Pcg(Block& b, const double* RHS, double* U, bool block, int pmax, double delta, bool warm = false);

  DevBuf<double> d_sums3_;   // 3 t K column sums of the trace terms
  int n_, K_, M_;
  hipStream_t s_;
  std::vector<int> m_, cum_;
  std::vector<int> rowptr_h_, split_h_;
  std::map<int, std::unique_ptr<ChunkPlan>> plans_;
  DevBuf<double> d_chunk_partials_;
  DevBuf<int> d_rowptr_, d_split_, d_col_, d_blk_, d_obs_ptr_, d_obs_, d_cum_;
  DevBuf<double> d_val_, d_cnt_, d_D_, d_sqrtD_, d_tau_, d_dsum_;
  DevBuf<double> d_zty_, d_y_, d_yty_, d_u_, d_ztzu_, d_partials_, d_out_;
  DevBuf<double> d_probes_, d_probesP_, d_PI_, d_DI_;
  double* h_out_ = nullptr;   // pinned
  std::unique_ptr<Block> b1_, bt_;
  int probes_t_ = 0;
  uint64_t probe_run_id_ = 0;
  bool probes_saved_ = false;
  bool y_set_ = false;
  bool u_valid_ = false;   // d_u_ holds a solution of a previous evaluation
};

}  // namespace gpb_amd
