// Launchers for the latent-Vecchia iterative path (latent_factor.hip, sparse_kernels.hip).
//
// Data layout in HBM (all in Vecchia order):
//   nbr    int32 n x m        neighbour j of row i at nbr[i*m + r], r < k_i = min(i, m)
//   Bv     fp64  n x m        B(i, nbr[i*m+r]) = -A_i[r]; B has a unit diagonal (implicit)
//   dBv    fp64  n x m        dB / dlog(phi), same sparsity (zero diagonal)
//   Dinv, dD fp64 n           D^-1 and dD / dlog(phi)
//   tptr/trow/tslot           transposed lists for B^T: column j -> entries e in
//                             [tptr[j], tptr[j+1]) with row trow[e] and value slot tslot[e]
//                             (= trow*m + r), rows ascending (deterministic sums)
//   blocks of t vectors       row-major n x t ("probe-interleaved"): X[i*t + c], so one
//                             neighbour gather reads t contiguous doubles
#pragma once

#include <hip/hip_runtime.h>

#include <vector>

namespace gpb_amd {

struct LatentFactorArgs {
  const double* X;   // coords row-major n x d (Vecchia order)
  const int* nbr;
  int n, d, m;
  double var, phi;   // sigma1^2, range transform
  double jitter;     // between-neighbour diagonal multiplier (JITTER_MULT_VECCHIA)
  double* Bv;
  double* dBv;       // nullable (no gradient)
  double* Dinv;
  double* dD;        // nullable
};
void launch_latent_factor(int cov_type, const LatentFactorArgs& a, hipStream_t s);

struct SparseB {
  int n, m;
  const int* nbr;
  const int* tptr;
  const int* trow;
  const int* tslot;
  // nullable: tval[e] = tval_of[tslot[e]], the values array in transposed-list order
  // (refreshed per evaluation); launch_bt_apply reads it when vals == tval_of
  const double* tval;
  const double* tval_of;
  // rows j whose transposed list is longer than kLongRow (early Vecchia rows are the
  // neighbours of hundreds of later rows): the t = 1 operator gives each a whole wave
  const int* longr;
  int nlong;
};
constexpr int kLongRow = 64;

// Y = diag(scale) (unit*X + V X)   with V = vals on the B pattern (rows list optional)
void launch_b_apply(const SparseB& B, const double* vals, bool unit, const double* X, int t, const double* scale,
                    double* Y, hipStream_t s);
// Y = unit*pre.*X + V^T (pre.*X) + W.*H  (pre, W/H nullable)
void launch_bt_apply(const SparseB& B, const double* vals, bool unit, const double* X, int t, const double* pre,
                     const double* W, const double* H, double* Y, hipStream_t s);
// VADU preconditioner Z = P^-1 R = (diag(dw) B)^-1 B^-T R for t columns in one launch
// (vadu_sweep.hip): one workgroup per column walks the level sets of both triangular
// solves with a workgroup barrier between "steps" (a level, or a slice of a large one),
// while the next step's structure is copied into LDS asynchronously.
// Step s is a contiguous blob of 32-bit words (blobs back to back, 16-byte aligned):
//   [0, kSweepHdr)        header: R rows, E entries, v0, own size, next blob's size, phase
//   [H, H + R)            row indices (original Vecchia index) of the step    (H = kSweepHdr)
//   [H + R, H + 2R + 1)   entry offsets (relative, eoff[0] = 0)
//   [v0, v0 + 2E)         entry values (fp64, 8-byte aligned)
//   [v0 + 2E, +E)         entry column indices
// B^T solve entries of row j: (child i, B(i, j)); lower solve entries of row i:
// (nbr[i][r], B(i, nbr[i][r])); phase 0 = B^T solve, 1 = lower solve.
constexpr int kSweepRows = 512;      // rows per step (= threads per workgroup)
constexpr int kSweepEnts = 6144;     // entries per step (two staged blobs fill ~156 KB of LDS)
constexpr int kSweepHdr = 8;
struct SweepPlan {
  int nsteps;
  int max_words;                     // largest blob (LDS buffer size, words)
  int first_words;                   // size of the first blob
  int* blob;                         // values refreshed per evaluation (launch_sweep_values)
};
void launch_vadu_sweep(const SweepPlan& plan, const double* dw, const double* R, double* Y, double* Z, int t,
                       hipStream_t s);
// Level-by-level form of the same preconditioner (one kernel per level, replayed as a
// hipGraph; rows of a level spread over all CUs, T lanes per row = the t columns).
// Rows in level order p: B^T solve rows p in [0, n) (levels [0, nlev_b)), lower solve rows
// p in [n, 2n). B^T solve: entries [beoff[p], beoff[p+1]) of (beidx, beval) = (child, B(child, row)).
// Lower solve: fixed stride m, entries (fidx, fval)[(p - n) * m + r] = (nbr, B(row, nbr)),
// zero-value padding, so a row's structure is one dependency-free load.
struct LevelPlan {
  int n, m;
  int nlev_b, nlev;
  std::vector<int> lptr;             // host, nlev + 1 (row positions p)
  const int* lrows;                  // 2n
  const int* beoff;                  // n + 1
  const int* beidx;
  const double* beval;
  const int* fidx;                   // n x m
  const double* fval;                // n x m
};
void launch_vadu_level(const LevelPlan& lp, int l, const double* dw, const double* R, double* Y, double* Z, int t,
                       hipStream_t s);
// Sync-free form of one of the two solves (vadu_flow.hip): one launch runs the whole DAG,
// each solved value doubling as its readiness flag. Positions q in [0, n) follow the solve's
// level order (row lrows[q]); B^T solve: entries [eoff[q], eoff[q+1]) of (eidx, eval);
// lower solve (eoff null): entries q*m + r, r < min(row, m), and the input is divided by dw.
// X (n x t) is filled with the sentinel by the launcher; err is set if a spin gives up.
struct FlowArgs {
  const int* lrows;
  const int* crit;     // per position: the dependency of highest level (-1: none), polled first
  const int* eoff;
  const int* eidx;
  const double* eval;
  const double* dw;
  const double* in;
  double* X;
  int* err;
  unsigned long long* prof;   // diagnostics (nullable): per position {setup, crit seen, published} timestamps
  int n, m, t, shift;
};
void launch_vadu_flow(const FlowArgs& a, bool lower, int max_blocks, hipStream_t s);
// Sync-free form with a fixed grid of resident single-wave workgroups (vadu_sf.hip): position
// q in [0, n) of the solve's level order is owned by workgroup q mod grid. Same structure
// arrays as FlowArgs; X is filled with the sentinel by the launcher.
struct SfArgs {
  const int* lrows;
  const int* crit;     // per position: the dependency of highest level (-1: none)
  const int* eoff;     // B^T solve: entry offsets per position (null for the lower solve)
  const int* eidx;
  const double* eval;
  const double* dw;    // lower solve: input divided by dw
  const double* in;
  double* X;
  int* err;
  int n, m, t;
};
void launch_vadu_sf(const SfArgs& a, bool lower, int grid, hipStream_t s);
// Head/tail split of the two solves (precond mode 4, vadu_head.hip). Head = the first K rows
// in Vecchia order (a thin, deep part of the DAG), solved by ONE workgroup per column with the
// column's head values in LDS (slot = Vecchia index < K); tail = the other rows, by the level
// kernels on a LevelPlan of the tail rows only. Lower solve: head, then tail levels. B^T
// solve: tail levels, then launch_vadu_head_partial (tail contributions to head rows), then
// the head.
// One solve's head rows in level order are cut into passes of at most kHeadRowsPerPass rows
// of ONE level. A pass has kHeadRowsPerPass slots of kHeadG lanes; a row takes 1, 2 or 4
// consecutive slots (aligned; by its entry count), so its group has GL = kHeadG << lg lanes.
// Record r = q * kHeadRowsPerPass + slot: bits 0-15 the row's LDS slot (K = padding), bits
// 16-17 lg, bits 18-19 the slot's index within the row, bit 31 set when the row has overflow
// entries [ooff[r0], ooff[r0 + 1]) (r0 = the row's first slot). Entries (head dependencies
// only) in a fixed lane-major layout: entry e < GL * EPL of the row sits at group lane
// gl = e % GL, k = e / GL, i.e. slot r0 + gl / kHeadG, position ((r * EPL + k) * kHeadG + gl %
// kHeadG) (zero value = padding); entries beyond GL * EPL go to the overflow lists.
constexpr int kHeadRowsPerPass = 64;
constexpr int kHeadMaxRows = 16384;  // K limit: 128 KB of LDS per column workgroup
constexpr int kHeadG = 16;            // lanes per slot
constexpr int kHeadEpl = 2;           // fixed-layout entries per lane
struct HeadSolve {
  int K;              // head rows = LDS slots (+ 1 scratch slot)
  int npass;
  const int* hrow;    // K: storage row of head slot v (Vecchia index v)
  const int* rec;     // npass * kHeadRowsPerPass records
  const int* eidx;    // fixed layout: LDS slot of the dependency
  const double* eval; // fixed layout: B value (refreshed per evaluation)
  const int* ooff;    // npass * kHeadRowsPerPass + 1
  const int* pend;    // npass: 1 = the pass ends its level (the next pass reads its results)
  const int* oidx;    // overflow entries
  const double* oval;
};
struct HeadPartial {  // B^T solve: tail rows' contributions to the head rows
  int rows;
  const int* row;     // storage row of head row w
  const int* eoff;    // entries [eoff[w], eoff[w+1])
  const int* eidx;    // storage row of the (tail) dependency
  const double* eval;
};
void launch_vadu_head(const HeadSolve& h, bool lower, const double* dw, const double* in, double* X, int t,
                      hipStream_t s);
void launch_vadu_head_partial(const HeadPartial& h, const double* R, double* X, int t, hipStream_t s);
void set_vadu_head_lds_limit(int K);
// Tile-blocked schedule of the tail solves (precond mode 4, GPBOOST_AMD_TAIL_TILES): tail rows
// are grouped into spatial tiles (blocks of TS consecutive storage rows, Morton order) and each
// row gets (superstep s, local level lam): the lexicographic max over its tail dependencies of
// (s_d, lam_d + 1) for a dependency in the same tile (wrapping to (s_d + 1, 0) at lam = L) and
// (s_d + 1, 0) for one in another tile. One launch per superstep, one workgroup per (s, tile)
// item, which runs its local levels with a workgroup barrier between them (a dependency on
// another workgroup's row was finished by an earlier launch). Positions of `lp` follow
// (s, tile, lam); item i covers local level l at positions [item_off[i*(L+1)+l], ...[l+1]).
constexpr int kTailLocalLevels = 8;
void launch_vadu_tile(const LevelPlan& lp, bool lower, const int* item_off, int L, int item0, int nitems,
                      const double* dw, const double* in, double* X, int t, hipStream_t s);
// blob_f64[vpos[e]] = Bv[eslot[e]] for all count entries (per-evaluation value refresh)
void launch_sweep_values(int count, const int* vpos, const int* eslot, const double* Bv, int* blob, hipStream_t s);
// dst[p*m + r] = src[rows[p]*m + r]  (n x m, level order)  |  dst[e] = idx[e] >= 0 ? src[idx[e]] : 0
void launch_gather_rows(int n, int m, const int* rows, const double* src, double* dst, hipStream_t s);
void launch_gather(int count, const int* idx, const double* src, double* dst, hipStream_t s);

// Per-column dot products: out[q*t + c] = sum_i A_q[i,c] * B_q[i,c], q < np (np <= 3).
// Deterministic two-pass reduction through `partials` (>= kMaxRedBlocks * np * t doubles).
constexpr int kMaxRedBlocks = 512;
void launch_coldots(int n, int t, int np, const double* const* A, const double* const* Bm, double* partials,
                    double* out, hipStream_t s);
// U += a .* H ; R -= a .* V ; rr[c] = sum_i R[i,c]^2 (per-column a from device memory)
void launch_cg_update(int n, int t, const double* a, const double* H, const double* V, double* U, double* R,
                      double* partials, double* rr, hipStream_t s);
// H = Z + b .* H
void launch_h_update(int n, int t, const double* b, const double* Z, double* H, hipStream_t s);
// a = rz / hv (hist[it*t + c] = a)  |  b = rz_new / rz, rz = rz_new (hist[it*t + c] = b);
// act (nullable): per-column activity mask, inactive columns get a = b = 0 (frozen)
void launch_cg_alpha(int t, const double* rz, const double* hv, const int* act, double* a, double* hist,
                     hipStream_t s);
void launch_cg_beta(int t, const double* rz_new, double* rz, const int* act, double* b, double* hist,
                    hipStream_t s);
// dst[i*ld_dst + c_dst + c] = src[i*ld_src + c_src + c], c < ncols (row-major column blocks)
void launch_pack_columns(int n, int ncols, const double* src, int ld_src, int c_src, double* dst, int ld_dst,
                         int c_dst, hipStream_t s);
// Y = X (n x t copy)
void launch_copy(size_t count, const double* X, double* Y, hipStream_t s);
// Z = alpha X + beta Y (elementwise, count entries; Z may alias X or Y)
void launch_axpby(size_t count, double alpha, const double* X, double beta, const double* Y, double* Z,
                  hipStream_t s);

// ---- likelihood-specific elementwise and reductions
enum LatentLik : int { kLikGaussian = 0, kLikBernoulliLogit = 1 };

struct NewtonPrepArgs {
  int n, lik;
  double aux;           // gaussian error variance
  const double* y;
  const double* loc;    // mode (+ offset)
  const double* mode;
  const double* Dinv;
  double* d1;           // first derivative of the log-likelihood
  double* W;            // information (read; rewritten when W_update)
  int W_update;
  double* rhs;          // W*mode + d1 (nullable)
  double* dw;           // D^-1 + W (nullable)
  double* sdw;          // sqrt(dw) (nullable)
};
void launch_newton_prep(const NewtonPrepArgs& a, hipStream_t s);

// Scalar row sums (one thread per row), fixed order -> out[kLatentScalars].
enum LatentScalar : int {
  kSqQuad = 0,     // (Bm)^T D^-1 (Bm)
  kSqLogLik,       // sum log p(y | loc)
  kSqLogDinv,      // sum log D^-1
  kSqLogDw,        // sum log(D^-1 + W)
  kSqRss,          // sum (y - loc)^2 (gaussian)
  kSqDQuadRng,     // (dB m)^T D^-1 (Bm)
  kSqDDQuad,       // (Bm)^T D^-1 dD D^-1 (Bm)
  kSqTrVar,        // sum dw^-1 D^-1
  kSqTrRng,        // sum dw^-1 D^-2 dD
  kSqDinvDD,       // sum D^-1 dD
  kSqTrDw,         // sum dw^-1  (aux trace, times dW/dlog aux)
  kSqImpVar,       // (B vS)^T D^-1 (Bm)
  kSqImpRng,       // (dB vS)^T D^-1 Bm + (B vS)^T D^-1 dB m - (B vS)^T D^-1 dD D^-1 Bm
  kLatentScalars
};
struct ScalarArgs {
  int n, m, lik;
  double aux;
  const int* nbr;
  const double* Bv;
  const double* dBv;    // nullable -> gradient terms skipped
  const double* Dinv;
  const double* dD;
  const double* dw;     // nullable -> log/trace terms skipped
  const double* y;
  const double* mode;
  const double* vS;     // nullable -> implicit terms skipped
};
void launch_latent_scalars(const ScalarArgs& a, double* partials, double* out, hipStream_t s);

// Per-column stochastic-trace sums for the gradient (U = (Sigma^-1+W)^-1 Z, P = P^-1 Z):
// out[q*t + c], q = 0 zt1_var, 1 ztP_var, 2 zt1_rng, 3 ztP_rng, 4 zt1_aux, 5 ztP_aux
// (aux terms use the constant dW/dlog aux = daux).
constexpr int kGradCols = 6;
struct GradColsArgs {
  int n, m, t;
  const int* nbr;
  const double* Bv;
  const double* dBv;
  const double* Dinv;
  const double* dD;
  const double* W;
  double daux;
  const double* U;
  const double* P;
};
void launch_grad_cols(const GradColsArgs& a, double* partials, double* out, hipStream_t s);

// Row-wise (per-observation) stochastic estimate of d log|Sigma W + I| / d mode with
// per-row control variates (likelihoods.h:12320-12341, CG_utils.cpp:1026-1041):
// dmll[i] = 0.5 * ( tr1_i + c_i * dW_i / dw_i - c_i * trP_i ).
struct ModeDerivArgs {
  int n, m, t, lik;
  const int* nbr;
  const double* Bv;
  const double* dw;
  const double* loc;
  const double* U;
  const double* P;
  double* dmll;
};
void launch_mode_deriv(const ModeDerivArgs& a, hipStream_t s);

}  // namespace gpb_amd
