// Sparse Cholesky of Sigma^-1 + W = B^T D^-1 B + diag(W) for the Vecchia-Laplace path with
// matrix_inversion_method = "cholesky" (the reference's exact Laplace-Vecchia branch):
//   FindModePostRandEffCalcMLLVecchia     likelihoods.h:2935-2955 (factorize per Newton step, solve),
//                                         :3052-3070 (log-determinant 2 sum log L_ii)
//   CalcGradNegMargLikelihoodLaplaceApproxVecchia, Cholesky branch
//                                         likelihoods.h:5207-5336 (L^-1, (Sigma^-1 + W)^-1 at the
//                                         non-zeros of SigmaI_deriv, its diagonal)
//   PredictLaplaceApproxVecchia, Cholesky likelihoods.h:6751-6811 (L \ (Bpo^T Bp^-T))
// The reference factors with Eigen's simplicial LLT (chol_sp_mat_t, AMD ordering, one column at a
// time on the host). Here:
//   * symbolic analysis once per model on the host (CholPlan): a nested-dissection ordering of the
//     graph of A (each Vecchia row's clique {i} U N(i)) from coordinate bisections with a graph vertex
//     separator, the elimination tree, column counts, fundamental supernodes with relaxed amalgamation,
//     each supernode's row structure and the level schedule of the supernodal tree;
//   * numeric multifrontal factorization on the GPU (sparse_chol.hip): one dense fs x fs front per
//     supernode (fs = ns columns + |R_s| rows below), A's entries assembled from per-entry lists of
//     clique contributions, children's update matrices pulled in by extend-add, the partial dense
//     Cholesky of the first ns columns in LDS (small fronts) or on the fp64 MFMA GEMM (large fronts);
//     all supernodes of one tree level per launch;
//   * solves, 2 sum log L_ii, and the selected inverse S = (Sigma^-1 + W)^-1 on the pattern of L
//     (Takahashi recursion over the same fronts, root first), which gives the gradient's traces
//     tr(dA S) exactly (the reference forms L^-1 with a sparse triangular solve of the identity and
//     then L^-T L^-1 at the non-zeros: CalcLtLGivenSparsityPattern).
// The factor does not depend on the ordering beyond rounding: log-determinant, solves and traces equal
// the reference's to ~1e-12 relative.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <memory>
#include <vector>

#include "common.h"

namespace gpb_amd {

// ---- work items of the numeric phases (host-built once per plan, executed by sparse_chol.hip)
// Buffers a task can address (bits of CholGemmTask::flags): the fronts F (factor + update blocks), the
// selected inverse S (same layout), the diagonal-block inverses Wd (64 x 64 per block), a scratch Y.
// P holds split-K partial products (reduced by CholReduceTask).
enum CholBuf { kCbF = 0, kCbS = 1, kCbW = 2, kCbY = 3, kCbP = 4 };
// One output tile (M, N <= 64): C = alpha op(A) op(B) + beta C, column-major, element offsets into the
// flagged buffers. flags: bit 0 transA, bit 1 transB, bit 2 lower-only output (write when
// i - j + doff >= 0, tile-local i, j), bits 4-6 / 7-9 / 10-12 the buffers of A / B / C.
struct CholGemmTask {
  int64_t a, b, c;
  int lda, ldb, ldc;
  int M, N, K;
  int flags, doff;
  double alpha, beta;
};
constexpr int kCgTA = 1, kCgTB = 2, kCgLower = 4;
inline int cg_bufs(int a, int b, int c) { return (a << 4) | (b << 7) | (c << 10); }
// C (M x N <= 64 x 64, ld ldc, buffer bufc) = beta C + alpha sum_{q < nslices} P[p + q pstride] (slices M x N, ld M)
struct CholReduceTask {
  int64_t c, p, pstride;
  int ldc, M, N, nslices, bufc, pad;
  double alpha, beta;
};
// Diagonal block (j0, j0) of a front: ib x ib Cholesky in place + its inverse to Wd[w] (ld 64).
struct CholDiagTask {
  int64_t c, w;
  int ld, ib;
};
// Columns [c0, c1) of supernode s's front (assembly / gather / mirror ranges).
struct CholColTask {
  int s, c0, c1, pad;
};
enum CholOpType {
  kOpAsmTile = 0,        // CholColTask {s, row tile, column tile}: front tile = sum of the children's update blocks
  kOpAsmEntries,     // CholColTask {s, j0, j1}: A's entries of front columns [j0, j1) (+ W on the diagonal) added
  kOpReduce,         // CholReduceTask
  kOpDiag,           // CholDiagTask
  kOpGemm,           // CholGemmTask
  kOpGatherS,        // CholColTask over the R x R block: S_RR of s from its parent's front (both triangles)
  kOpMirror,         // CholColTask: S[j, i] = S[i, j] for front columns [c0, c1), rows [pad, pad + 64) below
  kOpAsmV,           // CholColTask (c0 = 0, c1 = fs): V_s = [P b at the columns; 0] + children's parts
  kOpGatherX,        // CholColTask: V_s[ns:fs] = X[R_s]
  kOpScatterX,       // CholColTask: X[cols(s)] = V_s[0:ns]
  kOpFSolve1,        // t = 1, a level of small supernodes: one workgroup per supernode runs its whole forward
  kOpBSolve1,        //   / backward panel sweep; ntask = the level's supernodes, task0 = its first lvl_sup index
  kOpLoadV,          // CholColTask: V_s[0:ns] = X[cols(s)] (a backward-only sweep's input)
  kOpFwdVec,         // t = 1, CholColTask {s, block k, row tile rt}: x_b = W_b v_b (to the side buffer XS when rt is
                     //   the first row tile) and v[rt:rt+64] -= L[rt:rt+64, b] x_b, one wave per task (one launch per
                     //   block step instead of two)
  kOpCopyXS,         // CholColTask: V_s[c0:c1] = XS_s[c0:c1] (the forward results of a fused level)
  kOpBwdVecPart,     // t = 1, CholColTask {s, block k, row chunk kc, slot}: P[slot] = L[chunk, b]^T v[chunk] (256 rows)
  kOpBwdVecFin,      // t = 1, CholColTask {s, block k, nch, slot0}: x_b = W_b^T (v_b - sum_kc P[slot0 + kc]) in place
};
struct CholOp {
  int type, ntask;
  int64_t task0;   // first task in the array of its type
};
struct CholSchedule {
  std::vector<CholOp> ops;
  std::vector<CholGemmTask> gemm;
  std::vector<CholDiagTask> diag;
  std::vector<CholColTask> col;
  std::vector<CholReduceTask> red;
  int64_t y_doubles = 0;   // scratch the schedule needs
  int64_t p_doubles = 0;   // split-K partials
};

// Host symbolic analysis.
struct CholPlan {
  int n = 0;
  std::vector<int> perm, iperm;   // perm[k] = matrix index eliminated k-th; iperm = inverse
  int nsup = 0;
  std::vector<int> sfirst;        // nsup + 1: supernode s = elimination positions [sfirst[s], sfirst[s+1])
  std::vector<int> sparent;       // -1 for a root
  std::vector<int64_t> rptr;      // nsup + 1
  std::vector<int> rows;          // R_s = rows[rptr[s] .. rptr[s+1]): positions > the last column, ascending
  std::vector<int64_t> foff;      // nsup + 1: offset of s's fs x fs front (column-major, ld = fs)
  std::vector<int> lvl_ptr, lvl_sup;   // supernodes of tree level l (height): lvl_sup[lvl_ptr[l] ..)
  std::vector<int> col_sup;       // position -> supernode
  // statistics
  int64_t nnz_l = 0;              // entries of L (incl. the amalgamation zeros, diagonal blocks lower)
  int64_t front_doubles = 0;      // sum fs^2
  double flops = 0.;              // factorization flops (POTRF + TRSM + SYRK per front)
  int max_fs = 0, max_ns = 0;
  double ms_analyze = 0.;
  // extend-add maps: rel[rptr[s] + a] = position of R_s[a] in the parent's front; children CSR
  std::vector<int> rel;
  std::vector<int> cptr, child;
  // cinv[cinv_off[c] + p] = index in R_c of the parent's front position p (-1: none), for the tile assembly
  std::vector<int64_t> cinv_off;
  std::vector<int> cinv;
  std::vector<int64_t> woff;      // nsup + 1: offset of s's diagonal-block inverses (64 x 64 per block)
  // schedules
  CholSchedule factor, selinv;
  int nblk(int s) const { return (ns(s) + 63) / 64; }
  int ns(int s) const { return sfirst[s + 1] - sfirst[s]; }
  int nr(int s) const { return (int)(rptr[s + 1] - rptr[s]); }
  int fs(int s) const { return ns(s) + nr(s); }
};

// Graph of A: vertex i's clique is {i} U nbr[i*m + r] for r < kcount(i) = min(i, m) (entries < 0
// skipped). X: host coordinates row-major n x d (geometric bisection of the nested dissection).
// leaf: largest subgraph left undivided.
void chol_analyze(int n, int m, const int* nbr, int d, const double* X, int leaf, CholPlan& plan);
// Schedule of a forward + backward solve with t right-hand sides (front vectors fs x t per supernode
// in the scratch, ld fs; the global X is n x t, ld n, in elimination positions). vofs: per supernode
// scratch offsets (nsup + 1). forward_only: stop after the forward sweep (L^-1 b left in the fronts,
// scattered to X). backward_only: the backward sweep alone, its input (the layout a forward-only sweep
// leaves in X) loaded into the fronts first.
void chol_solve_schedule(const CholPlan& P, int t, bool forward_only, CholSchedule& S, std::vector<int64_t>& vofs,
                         bool backward_only = false);

// A's lower entries in the front layout and their clique contributions (host, once per plan):
//   column g (elimination position) holds entries [ecol[g], ecol[g+1]) (rows ascending, the diagonal
//   first) at front offsets eoff[e]; entry e sums ctr[cptr[e] .. cptr[e+1]) = row r << 16 | a << 8 | b:
//   D^-1_r B(r, q_a) B(r, q_b) with q_0 = r, q_{a} = nbr[r m + a - 1] (a, b <= 255, so m <= 254);
//   dpos[g] = front offset of the diagonal of column g.
struct CholEntries {
  std::vector<int64_t> ecol, eoff, cptr, dpos;
  std::vector<uint64_t> ctr;
};
void chol_entry_lists(const CholPlan& P, int m, const int* nbr, CholEntries& E);

// Numeric factorization, solves and selected inverse on the device (sparse_chol.hip). All work is
// queued on the stream given at construction; the matrix labels are those of nbr / X.
struct SparseCholDev;
class SparseChol {
 public:
  // nbr: host n x m neighbour table of the Vecchia factor (row i holds min(i, m) entries); X: host
  // coordinates row-major n x d. Builds the plan and the entry lists (host), uploads them.
  SparseChol(int n, int m, const int* nbr, int d, const double* X, hipStream_t s);
  ~SparseChol();
  SparseChol(const SparseChol&) = delete;
  SparseChol& operator=(const SparseChol&) = delete;
  const CholPlan& plan() const { return plan_; }

  // A = B^T D^-1 B: the clique sums of A's lower entries and, if dBv != null, of the derivative
  // dA = dB^T D^-1 B + B^T D^-1 dB - B^T D^-1 dD D^-1 B (range parameter). Bv, dBv device n x m
  // (B(i, nbr) values, unit diagonal implicit), Dinv, dD device n.
  void SetB(const double* Bv, const double* Dinv, const double* dBv, const double* dD);
  // Factor A + diag(W) (W device n, nullable = 0; read at launch). Non-positive pivots: Info() > 0.
  void Factor(const double* W);
  // x = A^-1 b (device n vectors, matrix labels; x may alias b).
  void Solve(const double* b, double* x);
  // X = L^-1 P B for nrhs columns (device column-major n x nrhs, ld n, matrix labels; the result in
  // elimination positions mapped back to the labels): the reference's TriangularSolveGivenCholesky(L, Maux)
  // for predictive variances (likelihoods.h:6765); column norms are label-invariant.
  void ForwardCols(const double* B, double* X, int nrhs);
  // X = A^-1 B for nrhs columns (device column-major n x nrhs, ld n, matrix labels; X may alias B)
  void SolveMulti(const double* B, double* X, int nrhs);
  // X = P^T L^-T B for nrhs columns, B in the layout ForwardCols returns (so BackwardCols(ForwardCols(b)) = A^-1 b;
  // X may alias B)
  void BackwardCols(const double* B, double* X, int nrhs);
  // 2 sum log L_ii (synchronises)
  double LogDet();
  // non-positive pivots of the last factorization (synchronises)
  int Info();
  // Selected inverse S = A^-1 on the structure of L (fronts' layout), then tr(S B^T D^-1 B) and, after a
  // SetB with derivatives, tr(S dA); diag(S) to diagS (device n, matrix labels; nullable). Synchronises.
  void SelectedInverse(double* tr_bdb, double* tr_da, double* diagS);
  // device time of the last Factor (ms; HIP events; synchronises)
  float last_factor_ms();

 private:
  void Run(const SparseCholDev& sch, double* ybuf, const void* solve_args);
  void SolveCols(const double* b, double* x, int t, int mode);   // mode 0: full, 1: forward only, 2: backward only
  struct Impl;
  CholPlan plan_;
  hipStream_t s_;
  int n_ = 0, m_ = 0;
  std::unique_ptr<Impl> impl_;
  DevBuf<int> d_perm_, d_sfirst_, d_rows_, d_rel_, d_cptr_, d_child_, d_sparent_, d_cinv_;
  DevBuf<int64_t> d_cinv_off_, d_woff_, d_vofs1_;
  DevBuf<int> d_lvl_sup_;
  int64_t vofs1_total_ = 0;
  DevBuf<int64_t> d_rptr_, d_foff_;
  DevBuf<int64_t> d_ecol_, d_eoff_, d_ecptr_, d_dpos_;
  DevBuf<uint64_t> d_ctr_;
  int64_t nent_ = 0;
  DevBuf<double> d_aval_, d_daval_;     // values of A's entries (B^T D^-1 B) and of dA
  DevBuf<double> d_F_, d_S_, d_Wd_, d_Y_, d_P_;
  DevBuf<int> d_info_;
  DevBuf<double> d_red_;
  const double* cur_W_ = nullptr;
  bool has_dA_ = false, factored_ = false, timed_ = false;
  hipEvent_t ev0_ = nullptr, ev1_ = nullptr;
};

// Helpers of the Cholesky Laplace path (sparse_chol.hip).
struct ObsMap;
// dmll_i = 0.5 diagS_i dW_i/dloc (the information's derivative at loc + offset; with obs: the sum over the
// row's observations): d_mll_d_mode of the Cholesky branch (likelihoods.h:5259).
void launch_chol_dmll(int n, int lik, double aux, const double* y, const double* loc, const double* offset,
                      const ObsMap& obs, const double* diagS, double* dmll, hipStream_t s);
// cols (n x np, ld n) = Bpo^T: column p holds Bpo[p][r] at row nb[p mp + r] (rows < 0 skipped)
void launch_chol_pred_cols(int n, int np, int mp, const int* nb, const double* Bpo, double* cols, hipStream_t s);
// V[p + k ldv] = scale * M[k + p n] for k < n, p < np
void launch_chol_transpose_scale(int n, int np, const double* M, double scale, double* V, int ldv, hipStream_t s);

}  // namespace gpb_amd
