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

#include <cstdint>
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
  // Gaussian form (transformed scale, VecchiaFisher): nugget 1 on the between-neighbour diagonal and in
  // D (Vecchia_utils.cpp:1351-1353, 1540); 0 = the latent form above
  double nugget;
  // nullable: dB / dlog(var) and dD / dlog(var) (the nugget form's variance derivative,
  // Vecchia_utils.cpp:1512, 1573-1580: dA = C^-1 a, dD = var - a.c - a.a)
  double* dBv_var;
  double* dD_var;
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
  // t = 1 default form of B: ELL stored column-major (entry r of row i at r n + i), so a wave's
  // loads of entry r of 64 rows are coalesced and its gathers are the r-th neighbours of 64
  // spatially close rows (Morton storage). Values refreshed per factor (vals_of = their source).
  const int* ell_idx;
  const double* ell_val;
  const double* vals_of;
  // t = 1 default form of B^T (n < 2^24; else null): nseg runs of consecutive storage rows
  // [seg_rb[w], seg_rb[w + 1]) with <= kSegEntries entries (or one longer row) and <= kSegRows rows;
  // seg_pk[e] = trow[e] | run-row index << 24 | (last entry of its row) << 31. One wave per run
  // sums its entries 64 at a time with a segmented wave scan.
  const int* seg_rb;
  const uint32_t* seg_pk;
  const int4* seg_info;   // per run {row begin, row end, entry begin, entry end} in the paired layout
  const uint32_t* seg_pk2; // paired layout: seg_pk with every run starting at an even position
  const double* seg_val2;  // values in the paired layout (refreshed with tval)
  int nseg;
};
constexpr int kLongRow = 64;
#ifndef GPB_SEG_ENTRIES
#define GPB_SEG_ENTRIES 512
#endif
constexpr int kSegEntries = GPB_SEG_ENTRIES;   // (A/B builds override)
constexpr int kSegRows = 127;                  // run-row index in 7 bits (127 = padding lanes)

// LDS-tiled form of the t >= 2 operator (opt-in, GPBOOST_AMD_SPMV_TILED=1; slower than the
// global-gather wave kernels, see sparse_kernels.hip) (one workgroup per tile of consecutive storage rows): the
// union of the tile's dependency rows is staged once into LDS (a Morton tile of 64 rows has ~270
// distinct neighbours for its ~1900 entries at m = 30), then every entry reads its row from LDS.
// Entry e of the op's lists (B: row i's r-th neighbour at i m + r; B^T: the tptr/trow order)
// carries its union-local index lidx[e]. Rows whose own list exceeds kTileUnion (early Vecchia
// rows of B^T) are not in any tile: rows fb[...] take the global-gather wave path.
struct TileOp {
  int ntile, nfb;
  const int* r0;        // ntile + 1: tile k = storage rows [r0[k], r0[k+1]) minus fallback rows
  const int* uoff;      // ntile + 1
  const int* urow;      // union rows (storage)
  const uint16_t* lidx; // per entry
  const int* fb;        // fallback rows
  const unsigned char* isfb;   // n: row is a fallback row
  int umax;             // largest union of a tile
};
#ifndef GPB_TILE_UNION
#define GPB_TILE_UNION 176
#endif
constexpr int kTileRows = 64, kTileUnion = GPB_TILE_UNION;

// tiled forms (t >= 2, vals = B's values in the op's entry order: B n x m / B^T tval)
void launch_b_apply_tiled(const SparseB& B, const TileOp& op, const double* vals, const double* X, int t,
                          const double* scale, double* Y, hipStream_t s);
void launch_bt_apply_tiled(const SparseB& B, const TileOp& op, const double* tval, const double* X, int t,
                           const double* W, const double* H, double* Y, hipStream_t s);
// Y = diag(scale) (unit*X + V X)   with V = vals on the B pattern (rows list optional)
void launch_b_apply(const SparseB& B, const double* vals, bool unit, const double* X, int t, const double* scale,
                    double* Y, hipStream_t s);
// Y = unit*pre.*X + V^T (pre.*X) + W.*H  (pre, W/H nullable)
void launch_bt_apply(const SparseB& B, const double* vals, bool unit, const double* X, int t, const double* pre,
                     const double* W, const double* H, double* Y, hipStream_t s);
// ---- VADU preconditioner Z = P^-1 R = B^-1 diag(1/dw) B^-T R (CG_utils.cpp:56-60); the plan that
// strings these kernels together is VaduPrecond (vadu_precond.h).
//
// Tail solves (vadu_level.hip): the wide part of the DAG, one launch per MERGED level. Rows of
// g consecutive dependency levels are solved in one launch: a row's dependencies inside its own
// merged level are substituted recursively by their own expressions, so every row reads only
// values of earlier merged levels (X entries) and inputs (IN entries):
//   x_i = sum_{IN e} c_e in[idx_e] (/ dw[idx_e], lower solve) + sum_{X e} c_e X[idx_e].
// In a random Vecchia ordering a row depends on ~1 row of the level just before it and the
// substituted rows' neighbourhoods overlap, so the fill is small (n = 100k, m = 30: g = 4 turns
// 103 launches per solve into 26 for +53% entries). g = 1 is the plain level schedule
// (x_i = in_i (/ dw_i) - sum_j b_ij x_j). The coefficients c are products of B values, computed
// per factor by launch_merged_numeric (one launch per level offset inside a merged level).
struct MergedSolve {
  int npos;                          // tail rows (positions in level order)
  std::vector<int> lptr;             // host: merged level boundaries (positions)
  const int* rows;                   // npos: storage row of position p
  const int* eoff;                   // npos + 1: entries [eoff[p], eoff[p+1])
  const int* xoff;                   // npos: [eoff[p], xoff[p]) IN entries, [xoff[p], eoff[p+1]) X entries
  const int* eidx;                   // storage row of the entry
  double* eval;                      // coefficients (launch_merged_numeric)
  // numeric plan: per position ops [opoff[p], opoff[p+1]): w = -Bv[op_slot]; op_map < 0: c[op_a] += w
  // (op_a a position in p's list); else c[map[op_map + q]] += w * c_{op_a}[q] for every entry q of
  // position op_a's list (a substituted dependency). c[0] = 1 is the row's own input.
  const int* opoff;
  const int* op_a;
  const int* op_slot;
  const int* op_map;
  const int* map;
  const int* offpos;                 // positions grouped by level offset inside their merged level
  std::vector<int> offptr;           // host: offset o -> offpos[offptr[o], offptr[o+1])
};
void launch_merged_numeric(const MergedSolve& ms, const double* Bv, hipStream_t s);
// coef = eval with 1/dw of the IN entry's row folded in (the lower solve's coefficients, per system)
void launch_merged_scale(const MergedSolve& ms, const double* dw, double* coef, hipStream_t s);
// merged level L of one solve: X[rows] = sum coef * (in for IN entries, earlier X for X entries);
// coef = ms.eval for the B^T solve, the launch_merged_scale output for the lower solve
void launch_merged_level(const MergedSolve& ms, int L, const double* coef, const double* in, double* X, int t,
                         hipStream_t s);
// Persistent form of one whole tail solve (vadu_level.hip, GPBOOST_AMD_TAIL_FORM=persist): ONE launch
// runs every merged level, with a grid barrier between merged levels instead of a kernel boundary, so
// the rows a level writes stay in its XCD's L2 for the later levels that gather them (a kernel
// boundary invalidates L2). Workgroup b belongs to XCD group b % 8 (the dispatch order), and group x
// solves the x-th eighth of every merged level's positions (Morton-sorted: one compact region of the
// domain), so most gathers stay inside one XCD. Tail values go to a padded copy Tp (row stride 64
// doubles = four whole cache lines: a line has one writer and is never read before it is written)
// and to the caller's X.
constexpr int kTailBit = 1 << 30;   // eidx_p: an X entry on a tail row (read from Tp)
constexpr int kTailPad = 64;        // Tp row stride (doubles); t <= kTailPad
struct TailPersist {
  const int* lptr;    // nL + 1 merged level boundaries (device copy of MergedSolve::lptr)
  int nL;
  const int* eidx_p;  // MergedSolve::eidx with kTailBit on X entries whose row is a tail row
  int W;              // workgroups per XCD group (grid 8 W; all resident at once)
  int diag;           // timing diagnostics only (TimeParts): 1 = no barriers, 2 = no gathers
};
// counters: nL x 9 unsigned, zeroed by the call before the launch (stream order)
void launch_tail_persist(const MergedSolve& ms, const TailPersist& tp, unsigned* counters, const double* coef,
                         const double* in, const double* Xr, double* Tp, double* X, int t, hipStream_t s);
// workgroups per XCD group the persistent tail kernel can keep resident (0: not available)
int tail_persist_max_w();
// LDS segment kernel (vadu_head.hip): ONE workgroup per column solves a segment of K rows with
// the column's segment values resident in LDS (slot = position in the segment); a level costs an
// LDS gather + a workgroup barrier instead of a launch. Dependencies outside the segment were
// folded into `in` by launch_vadu_partial, so the kernel serves both solves:
//   x_v = in[hrow[v]] (/ dw) - sum_{e} val_e x_{slot_e}   in pass order.
// The segment's rows in level order are cut into passes of at most kHeadRowsPerPass rows of ONE
// level. A pass has kHeadRowsPerPass slots of kHeadG lanes; a row takes 1, 2 or 4 consecutive
// slots (aligned; by its entry count), so its group has GL = kHeadG << lg lanes.
// Record r = q * kHeadRowsPerPass + slot: bits 0-15 the row's LDS slot (K = padding), bits
// 16-17 lg, bits 18-19 the slot's index within the row, bit 31 set when the row has overflow
// entries [ooff[r0], ooff[r0 + 1]) (r0 = the row's first slot). Entries (segment dependencies
// only) in a fixed lane-major layout: entry e < GL * EPL of the row sits at group lane
// gl = e % GL, k = e / GL, i.e. slot r0 + gl / kHeadG, position ((r * EPL + k) * kHeadG + gl %
// kHeadG) (zero value = padding); entries beyond GL * EPL go to the overflow lists.
// 64 slots of 16 lanes (2 entries each). (128 slots of 8 lanes x 4 entries: 40% fewer passes at
// n = 100k but each pass slower, 0.318 vs 0.297 ms for the two segment solves at t = 51.)
constexpr int kHeadRowsPerPass = 64;
constexpr int kHeadMaxRows = 16384;  // segment limit: 128 KB of LDS per column workgroup
constexpr int kHeadG = 16;            // lanes per slot
constexpr int kHeadEpl = 2;           // fixed-layout entries per lane
struct HeadSolve {
  int K;              // segment rows = LDS slots (+ 1 scratch slot)
  int npass;
  const int* hrow;    // K: storage row of slot v
  const int* rec;     // npass * kHeadRowsPerPass records
  const int* eidx;    // fixed layout: LDS slot of the dependency
  const double* eval; // fixed layout: B value (refreshed per evaluation)
  const int* ooff;    // npass * kHeadRowsPerPass + 1
  const int* pend;    // npass: 1 = the pass ends its level (the next pass reads its results)
  const int* oidx;    // overflow entries
  const double* oval;
};
void launch_vadu_head(const HeadSolve& h, const double* in, const double* dw, double* X, int t, hipStream_t s);
void set_vadu_head_lds_limit(int K);
// One-wave form of the same segment solve (the default): the passes are run by ONE wave per column
// (the workgroup's other waves only load the segment into LDS and write it back), so a pass is one
// wave's instruction stream with no workgroup barrier — LDS operations of one wave complete in
// order, which orders every pass's writes before the next pass's reads. A pass holds up to 64 >> lg
// rows of one level, each on a group of G = 2^lg lanes (rows with more than kSegSteps entries take
// G > 1); lane l of a pass takes the entries j = l % G, j + G, ... of its row over L <= kSegSteps
// steps, lanes reduce over G by DPP, and the group's first lane writes x = -acc. A row's first
// entry is its own input with coefficient -1 (value slot -2 -> -1 in the per-factor gather), so
// acc = sum_e c_e x_e - in and the pass needs no read-modify-write. Entries are LDS byte offsets.
constexpr int kSegSteps = 32;
struct SegWave {
  int K;               // segment rows (LDS slot K = a zero, the padding entries' target)
  int npass;
  const int* hrow;     // K: storage row of slot v
  const int4* meta;    // npass: {entry offset (units of 64 entries), steps L, lg, 0}
  const int* rec;      // npass x 64: the output slot of the lane's row (first lane of the group), -1 otherwise
  const int* eidx;     // (sum of L) x 64: LDS byte offset of the entry's value
  const double* eval;  // same layout: coefficient (the row's own input: -1; padding: 0)
};
void launch_vadu_seg_wave(const SegWave& w, const double* in, const double* dw, double* X, int t, hipStream_t s);
// Partial sums of dependencies outside a step, for each listed row r (storage rows):
//   out[r] = (in ? in[r] / (dw ? dw[r] : 1) : out[r]) - sum_{e in [eoff[w], eoff[w+1])} eval[e] src[eidx[e]]
struct PartialList {
  int rows;
  const int* row;     // storage row of list row w
  const int* eoff;
  const int* eidx;    // storage row of the dependency
  const double* eval;
};
// compact (nullable): list rows w < ncompact are also stored at compact[w * t + c].
void launch_vadu_partial(const PartialList& p, const double* in, const double* dw, const double* src, double* out,
                         int t, hipStream_t s, double* compact = nullptr, int ncompact = 0);
// Dense head block (vadu_dense.hip), K0 x K0 column-major with leading dimension ld (K0 rounded
// up to 64, identity padding): per factor Bd = B_00, G = Bd^-1 and GT = G^T (T: ld x (ld/2 + 64)
// scratch); per application, with X the head-0 rows of the B^T solve's result in Vecchia order
// (compact row-major K0 x t, written by the last partial sum that touches them), S = diag(1/dw_0)
// G^T X (S: 2 ld x t scratch, X may be its first half), then Y[rows] = G S (Y: the storage-order
// t-column block, head-0 rows reached through DenseHead::row).
struct DenseHead {
  int K0, ld, m;
  const int* row;      // K0: storage row of Vecchia row v < K0
  const int* col;      // K0 x m: Vecchia index of entry (v, r) (-1: padding)
  const double* val;   // K0 x m: B value of entry (v, r) (refreshed per factor)
};
void dense_head_factor(const DenseHead& d, double* Bd, double* G, double* GT, double* T, hipStream_t s);
void launch_dense_head_apply(const DenseHead& d, const double* G, const double* GT, const double* dw, const double* X,
                             double* S, double* Y, int t, hipStream_t s);
// dst[e] = idx[e] >= 0 ? src[idx[e]] : (idx[e] == -2 ? -1 : 0)
void launch_gather(int count, const int* idx, const double* src, double* dst, hipStream_t s);

// Per-column dot products: out[q*t + c] = sum_i A_q[i,c] * B_q[i,c], q < np (np <= 3).
// Deterministic two-pass reduction through `partials` (>= kMaxRedBlocks * np * t doubles).
constexpr int kMaxRedBlocks = 512;
void launch_coldots(int n, int t, int np, const double* const* A, const double* const* Bm, double* partials,
                    double* out, hipStream_t s);
// U += a .* H ; R -= a .* V ; rr[c] = sum_i R[i,c]^2 (per-column a from device memory)
void launch_cg_update(int n, int t, const double* a, const double* H, const double* V, double* U, double* R,
                      double* partials, double* rr, hipStream_t s);
// Device side of the PCG stopping rules (LatentVecchia::Pcg). ctl[kCtlActS]: single-vector
// columns [0, n_single) still running; ctl[kCtlActB]: block columns [n_single, t) running;
// ctl[kCtlItsS] / [kCtlItsB]: iterations done; ctl[kCtlNan]: NaN/Inf met in a residual norm.
enum PcgCtlField : int { kCtlActS = 0, kCtlActB, kCtlItsS, kCtlItsB, kCtlNan, kPcgCtl = 8 };
// Host copy of a verdict: one 64-bit word, bits 0-15 the check's sequence number, 16 / 17 / 18
// the single / block / NaN flags, 19-39 its_single, 40-60 its_block.
__host__ __device__ inline unsigned long long pcg_pack(int seq, int act_s, int act_b, int nan, int its_s, int its_b) {
  return (unsigned long long)(seq & 0xFFFF) | (unsigned long long)(act_s & 1) << 16 |
         (unsigned long long)(act_b & 1) << 17 | (unsigned long long)(nan & 1) << 18 |
         (unsigned long long)(its_s & 0x1FFFFF) << 19 | (unsigned long long)(its_b & 0x1FFFFF) << 40;
}
__host__ __device__ inline void pcg_unpack(unsigned long long v, int* ctl) {
  ctl[kCtlActS] = (int)(v >> 16) & 1;
  ctl[kCtlActB] = (int)(v >> 17) & 1;
  ctl[kCtlNan] = (int)(v >> 18) & 1;
  ctl[kCtlItsS] = (int)(v >> 19) & 0x1FFFFF;
  ctl[kCtlItsB] = (int)(v >> 40) & 0x1FFFFF;
}
// act[c] = 1, except single columns whose right-hand side is zero (rr0[c] < zero_sq: the
// reference returns u = 0 without iterating, CG_utils.cpp:42-45).
void launch_pcg_init(int t, int n_valid, int n_single, int pmax_single, int pmax_block, double zero_sq,
                     const double* rr0, int* act, int* ctl, hipStream_t s);
// out[0] = sum of the block columns' norms [n_single, n_valid) of this rank
void launch_pcg_block_sum(int n_valid, int n_single, const double* rr, double* out, hipStream_t s);
// After iteration j's update (rr[c] = ||r_c||^2): single columns stop on their own norm
// (CG_utils.cpp:80-90), the block on the mean column norm (:172-178), both at their pmax.
// host_ctl (nullable, 8-byte aligned host-coherent memory mapped for the device): receives
// pcg_pack(seq, ...) by one store.
// gsum != null: the block norm sum over all ranks, nblock its column count (probe-sharded blocks)
void launch_pcg_check(int j, int t, int n_single, int pmax_single, int pmax_block, double delta, const double* rr,
                      const double* gsum, int nblock, int* act, int* ctl, int* host_ctl, int seq, hipStream_t s);
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
// the Newton trial mode's change capped at log(100) per entry (CapChangeModeUpdateNewton, likelihoods.h:11800-11810;
// cap_change_mode_newton_ for poisson / gamma, :481-490)
void launch_cap_mode_change(size_t count, const double* mode, double* mnew, hipStream_t s);

// ---- likelihood-specific elementwise and reductions
enum LatentLik : int { kLikGaussian = 0, kLikBernoulliLogit = 1, kLikBernoulliProbit = 2, kLikPoisson = 3, kLikGamma = 4 };

// Observations of the latent variables when coordinates repeat (the reference's unique-location
// form: Z maps n observations to the n_u latent variables, Vecchia_utils.cpp:1121-1139,
// re_comp.h:845-870): the observations of storage row i are [ptr[i], ptr[i+1]) of y / offset
// (latent-variable-major). ptr == nullptr: one observation per row, y / offset indexed by row.
// The likelihood's per-row quantities are then sums over the row's observations (Z^T d1, Z^T W Z,
// Z^T dW), evaluated at mode_i + offset_e.
struct ObsMap {
  const int* ptr = nullptr;
  const double* y = nullptr;
  const double* offset = nullptr;
};

struct NewtonPrepArgs {
  int n, lik;
  double aux;           // gaussian error variance
  const double* y;
  const double* loc;    // mode
  const double* offset; // fixed effects F (nullable): the likelihood is evaluated at loc + F
  const double* mode;
  const double* Dinv;
  double* d1;           // first derivative of the log-likelihood
  double* W;            // information (read; rewritten when W_update)
  int W_update;
  double* rhs;          // W*mode + d1 (nullable)
  double* dw;           // D^-1 + W (nullable)
  double* sdw;          // sqrt(dw) (nullable)
  ObsMap obs;           // several observations per latent variable (repeated coordinates), optional
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
  const double* offset; // fixed effects F (nullable): log-likelihood at mode + F
  const double* vS;     // nullable -> implicit terms skipped
  ObsMap obs;
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
  const int* obs_ptr;   // nullable: dW/dlog aux of row i = daux x its number of observations
  const double* U;
  const double* P;
};
void launch_grad_cols(const GradColsArgs& a, double* partials, double* out, hipStream_t s);

// Row-wise (per-observation) stochastic estimate of d log|Sigma W + I| / d mode with
// per-row control variates (likelihoods.h:12320-12341, CG_utils.cpp:1026-1041):
// dmll[i] = 0.5 * ( tr1_i + c_i * dW_i / dw_i - c_i * trP_i ).
struct ModeDerivArgs {
  int n, m, t, lik;
  double aux;                  // the likelihood's auxiliary parameter (gamma: shape)
  int t_valid, t_all, stage;   // see mode_deriv_kernel; single rank: t_valid = t_all = t, stage 0
  double* mom;                 // stages 1-3: n x 2 row sums (all-reduced between stages)
  double* mom2;
  const int* nbr;
  const double* Bv;
  const double* dw;
  const double* loc;
  const double* offset;        // nullable: third derivative at loc + F
  const double* y;             // response (the probit information depends on it)
  ObsMap obs;
  const double* U;
  const double* P;
  double* dmll;
};
void launch_mode_deriv(const ModeDerivArgs& a, hipStream_t s);

// Gradient of the approximate negative marginal log-likelihood wrt the fixed effects F
// (likelihoods.h:5360-5366, no duplicate locations): out = -d1 + dmll - W .* vS (dmll / vS
// nullable: the likelihood's information does not depend on the mode -> out = -d1).
void launch_grad_f(int n, const double* d1, const double* dmll, const double* W, const double* vS, double* out,
                   hipStream_t s);
// likelihood 'gamma': per-observation records [l + y e^-l, W diag((Sigma^-1 + W)^-1), d1 (Sigma^-1 + W)^-1 dmll] of
// the shape gradient (n x 3; no duplicate locations)
void launch_gamma_aux_rec(int n, double aux, const double* y, const double* off, const double* loc, const double* W,
                          const double* dmll, const double* d1, const double* vS, double* rec, hipStream_t s);

// ---- latent predictions (latent_pred.hip)
// out (n x t row-major) ~ N(0, 1): counter-based, a function of (seed, stream, column c0 + c, row)
void launch_gen_normal(int n, int t, uint64_t seed, int stream, long c0, double* out, hipStream_t s);
void launch_sqrt_vec(int n, const double* x, double* y, hipStream_t s);
// acc[p] += sum_c (sum_r B[p, r] Z[nbr[p, r], c])^2 for the t <= 64 columns of Z (n x t row-major)
// bernoulli_logit response means (adaptive Gauss-Hermite, likelihoods.h:7857-7889) at latent N(mean, var);
// out_var (nullable) = p (1 - p). nodes / aw: the order-point rule, aw = w exp(x^2) (device).
void launch_resp_logit(int n, const double* mean, const double* var, const double* nodes, const double* aw, int order,
                       double delta, double* out_mean, double* out_var, hipStream_t s);
void launch_pred_sq_acc(int n_pred, int mp, int t, const int* nbr, const double* B, const double* Z, double* acc,
                        hipStream_t s);
// V[p + (col0 + c) ldv] = sum_r B[p, r] Z[nbr[p, r], c] for columns c < tc of the t-column block
void launch_pred_samples(int n_pred, int mp, int t, int tc, const int* nbr, const double* B, const double* Z, double* V,
                         int ldv, int col0, hipStream_t s);

}  // namespace gpb_amd
