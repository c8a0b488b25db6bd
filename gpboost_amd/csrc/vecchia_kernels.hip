// Vecchia factor + likelihood/gradient row kernel for gfx950 (CDNA4, wave64).
//
// Reference path replaced: CalcCovFactorGradientVecchia (Vecchia_utils.cpp:1307-1632,
// per-row loop :1405-1617) fused with CalcYAux / CalcYTPsiIInvY
// (re_model_template.h:8885-9120) and the Vecchia branch of CalcGradPars (:1768-1791).
//
// Mapping: one Vecchia row i (k_i = min(i, m) neighbours) is owned by a group of K
// lanes of one wavefront (K = 16/32/64 -> 4/2/1 rows per wave); lane r owns row r of
// the k x k between-neighbour covariance C_i (rows >= k_i are identity padding, which
// leaves every solution unchanged). All synchronisation inside a row is wave-local.
//
//  1. covariance pairs: the k(k-1)/2 exp-heavy entries are computed ONCE, split evenly
//     over the K lanes (lane l takes half of rows {l mod K/2, K-1-l mod K/2}), and
//     written to a packed lower triangle in LDS (K(K+1)/2 doubles per row);
//  2. lane r loads row r of [C | c | y_nbr] into registers and runs symmetric
//     Gauss-Jordan elimination: step j broadcasts column j of the current matrix and
//     the two augmented entries of row j through three K-double LDS slots (the trailing
//     block stays symmetric, so row j's entries are column j's). After K steps the
//     matrix is diagonal and lane r holds a_r = (C^-1 c)_r and v_r = (C^-1 y_nbr)_r:
//     no separate forward/backward substitution chains;
//  3. t = dC_range a, with dC_rc = h(phi r_rc) C_rc recomputed from the packed C and the
//     neighbour coordinates (no second exp, no second matrix image).
// Measured (MI355X, n=100k, m=30, 2 waves/SIMD): pair phase unrolled by 8 and branch-free plus
// the dC a sum unrolled with four partials: 0.455 -> 0.41 ms per launch; publishing the next
// pivot's reciprocal with the column (reciprocal chain off the step chain) needs ~290 registers
// (occupancy 1): 0.63 ms, rejected (re-measured with the bordered form: 0.319 vs 0.3145 ms).
// The row then emits six partial sums (logD, (By)^2/D, and per parameter
// s1 = uk u - u^2 dD/2, s2 = dD/D; DESIGN.md "reduction contract"). Blocks stride over
// row groups and keep per-lane accumulators, so one launch writes few block partials.
// Optional outputs D^-1 and B(i, nbr) = -a are written for the factor API.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <type_traits>

#include "common.h"
#include "cov.h"
#include "kernels.h"

namespace gpb_amd {
namespace {

constexpr int kDMax = 3;
#ifndef GPB_ROWS_MAXBLOCKS
#define GPB_ROWS_MAXBLOCKS 1024
#endif
// Row-kernel grid cap: 1024 blocks = exactly the resident capacity at 2 waves/SIMD (4 two-wave
// blocks per CU), every block striding over ~25 row groups: 0.3775 ms vs 0.383 (4096 blocks, 4
// rounds) and 0.405 (2048), and a quarter of the block partials for the sum kernel.
constexpr int kMaxBlocks = GPB_ROWS_MAXBLOCKS;   // (A/B builds override)
#ifndef GPB_PAIR_UNROLL
#define GPB_PAIR_UNROLL 8
#endif
constexpr int kPairUnroll = GPB_PAIR_UNROLL;   // pair-phase unroll (A/B builds override)

// Orders a wave's own LDS writes before its subsequent LDS reads.
__device__ __forceinline__ void wave_lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
// Compiler-only ordering (write-after-read on LDS within one wave is ordered by hardware).
__device__ __forceinline__ void compiler_fence() { asm volatile("" ::: "memory"); }

// Sum over a K-lane group (K = 16, 32, 64; smaller K by shuffles), result in every lane: the 16-lane DPP-row part by
// VALU data movement (quad swaps, half-row and row mirrors), only the cross-row steps through
// the LDS crossbar. Fixed order -> bitwise repeatable.
// Every control used here has a source lane for every lane, so bound_ctrl (read 0 for a missing
// source) never fires; it lets the move write all lanes without an initialised old value (the
// update_dpp(0, ...) form costs two extra v_mov per double).
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v) {
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), CTRL, 0xF, 0xF, true);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), CTRL, 0xF, 0xF, true);
  return __hiloint2double(hi, lo);
}
#ifndef GPB_PERMLANE_SWAP
#define GPB_PERMLANE_SWAP 1
#endif
#if GPB_PERMLANE_SWAP
template <bool ROW32>
__device__ __forceinline__ double swap_sum(double v) {
  const unsigned lo = __double2loint(v), hi = __double2hiint(v);
  if constexpr (ROW32) {
    const auto pl = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
    const auto ph = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
    return __hiloint2double(ph[0], pl[0]) + __hiloint2double(ph[1], pl[1]);
  } else {
    const auto pl = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
    const auto ph = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
    return __hiloint2double(ph[0], pl[0]) + __hiloint2double(ph[1], pl[1]);
  }
}
#endif

// ---- lane broadcasts without LDS (Gauss-Jordan pivot column)
template <int B, int E, class F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    static_for<B + 1, E>(f);
  }
}

// Value of lane L of each 16-lane DPP row, broadcast to that whole row (row_newbcast: one 64-bit
// DPP move on gfx950).
template <int L>
__device__ __forceinline__ double row_bcast(double v) {
  const long b = __builtin_amdgcn_mov_dpp(__builtin_bit_cast(long, v), 0x150 + L, 0xF, 0xF, true);
  return __builtin_bit_cast(double, b);
}

// 32-lane groups: lo = the value of group lane CP, hi = that of group lane 16 + CP, in every lane
// of the group. One row_newbcast per dword, then the gfx950 row-swap permute of the broadcast with
// itself: its first output holds the even DPP row's value in both rows of each pair, its second
// the odd row's (V_PERMLANE16_SWAP exchanges rows 1/3 of VDST with rows 0/2 of VSRC).
template <int CP>
__device__ __forceinline__ void group_bcast_pair(double v, double& lo, double& hi) {
  const double b = row_bcast<CP>(v);
  const unsigned bl = __double2loint(b), bh = __double2hiint(b);
  const auto pl = __builtin_amdgcn_permlane16_swap(bl, bl, false, false);
  const auto ph = __builtin_amdgcn_permlane16_swap(bh, bh, false, false);
  lo = __hiloint2double(ph[0], pl[0]);
  hi = __hiloint2double(ph[1], pl[1]);
}

template <int K>
__device__ __forceinline__ double group_sum(double v) {
  if constexpr (K < 16) {   // sub-row groups (the two-rows-per-lane variant): plain shuffles
#pragma unroll
    for (int off = K / 2; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
  }
  v += dpp_f64<0xB1>(v);    // quad_perm [1,0,3,2]
  v += dpp_f64<0x4E>(v);    // quad_perm [2,3,0,1]
  v += dpp_f64<0x141>(v);   // row_half_mirror
  v += dpp_f64<0x140>(v);   // row_mirror
#if GPB_PERMLANE_SWAP
  // cross-row steps by the gfx950 row-swap permutes (VALU, no LDS): the two outputs of a swap
  // of v with itself are {own, partner} in some order, and own + partner is order-independent
  if (K >= 32) v = swap_sum<false>(v);
  if (K >= 64) v = swap_sum<true>(v);
#else
  if (K >= 32) v += __shfl_xor(v, 16, 64);
  if (K >= 64) v += __shfl_xor(v, 32, 64);
#endif
  return v;
}

// Eight sums over a 32-lane group (two DPP rows) at once. The cross-row step goes first and is
// transposed: one row-swap permute of the pair (v[i], v[i + 4]) leaves the row-0 lanes holding
// v[i] of both rows and the row-1 lanes v[i + 4] of both rows, so one add per pair halves the
// values to four before the four in-row DPP steps (3 VALU per step per double instead of 5 per
// step per sum). Result: lanes of row 0 hold the sums of v[0..3] in s[0..3], lanes of row 1 those
// of v[4..7]. Every sum adds (row-0 part) + (row-1 part), then fixed DPP pairings: bitwise
// repeatable.
__device__ __forceinline__ void group_sum8_rows(const double v[8], double s[4]) {
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const auto pl = __builtin_amdgcn_permlane16_swap(__double2loint(v[q]), __double2loint(v[q + 4]), false, false);
    const auto ph = __builtin_amdgcn_permlane16_swap(__double2hiint(v[q]), __double2hiint(v[q + 4]), false, false);
    s[q] = __hiloint2double(ph[0], pl[0]) + __hiloint2double(ph[1], pl[1]);
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    double x = s[q];
    x += dpp_f64<0xB1>(x);    // quad_perm [1,0,3,2]
    x += dpp_f64<0x4E>(x);    // quad_perm [2,3,0,1]
    x += dpp_f64<0x141>(x);   // row_half_mirror
    x += dpp_f64<0x140>(x);   // row_mirror
    s[q] = x;
  }
}

// The odd DPP row's value of v in every lane of each row pair (row 1 -> rows 0 and 1).
__device__ __forceinline__ double odd_row_value(double v) {
  const unsigned lo = __double2loint(v), hi = __double2hiint(v);
  const auto pl = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
  const auto ph = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
  return __hiloint2double(ph[1], pl[1]);   // [0]: the even row's value, [1]: the odd row's
}

template <int K>
constexpr int block_threads() { return K == 64 ? 64 : 128; }

template <int K, bool BORDER = false>
constexpr int group_lds_doubles() {
  // packed C + packed dC + neighbour coords + 3 broadcast slots; bordered: packed C (dC in its
  // circulant layout over it after the row load) + two coordinate copies (the slots alias them)
  return BORDER ? K * (K + 1) / 2 + 2 * kDMax * K : K * (K + 1) + kDMax * K + 3 * K;
}

__device__ __forceinline__ int packed(int r, int c) {  // r >= c
  return r * (r + 1) / 2 + c;
}

// Diagnostics (GPBOOST_AMD_ROWS_PROF): per-phase s_memtime cycles of wave 0 of block 0, summed
// over its row groups: [gather, pairs, gj, dca, reduce, iterations].
__device__ unsigned long long g_rows_prof[8];

// MK <= K: matrix rows (= elimination steps); lanes r >= MK of a group only take part in the
// wave-level operations (m <= 30 with K = 32: the two identity-padding steps are not run).
// DPPBC (K = 16 / 32, A/B form, see rows_dpp): the Gauss-Jordan steps broadcast the pivot column
// by DPP row broadcasts and row-swap permutes (VALU) instead of LDS slots. Same values in the same
// FMA order: bitwise identical results.
#ifndef GPB_ROWS_WAVES
#define GPB_ROWS_WAVES 0
#endif
#if GPB_ROWS_WAVES > 0
#define GPB_ROWS_WAVES_ATTR __attribute__((amdgpu_waves_per_eu(GPB_ROWS_WAVES, GPB_ROWS_WAVES)))
#else
#define GPB_ROWS_WAVES_ATTR
#endif
// BORDER (MK + 2 <= K): the augmented columns ride as two extra matrix rows held by the idle lanes
// MK and MK + 1 (the bordered symmetric matrix [[C, c, y_nbr], [c^T ...], [y_nbr^T ...]]): a step
// broadcasts ONE column (row j of the trailing block incl. the pivot row's augmented entries
// M[j][MK] = M[MK][j]) by one LDS store, and the lanes read it back as 16-byte pairs.
// DIM > 0: the coordinate dimension is known at compile time (DIM == a.d), else loops run to kDMax
// over zero-padded coordinates.
template <int K, int COV, bool PROF = false, int MK = K, bool DPPBC = false, bool BORDER = false, int DIM = 0>
__global__ void __launch_bounds__(block_threads<K>()) GPB_ROWS_WAVES_ATTR vecchia_rows_kernel(VecchiaRowsArgs a) {
  static_assert(!DPPBC || K == 16 || K == 32, "DPP broadcasts need 16- or 32-lane groups");
  static_assert(!BORDER || (!DPPBC && MK + 2 <= K && (MK & 1) == 0), "bordered form: two spare lanes, even width");
  constexpr int NC = BORDER ? MK + 2 : MK;   // register columns per lane
  extern __shared__ __attribute__((aligned(16))) double smem[];
  constexpr int BT = block_threads<K>();
  constexpr int G = 64 / K;                 // rows per wave
  constexpr int rows_per_block = (BT / 64) * G;
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int g = lane / K;
  const int r_lane = lane - g * K;
  const int group_id = wave * G + g;
  static_assert(DIM == 0 || (BORDER && DIM <= kDMax), "compile-time dimension: bordered form only");
  constexpr int ND = DIM > 0 ? DIM : kDMax;   // coordinates per point in the distance loops
  constexpr int CS = BORDER ? ND : kDMax;     // coordinate stride of the LDS copy (2: 16-byte reads)
  const int d = DIM > 0 ? DIM : a.d;
  const double var = a.var, phi = a.phi;
  const double cdiag = var * a.diag_mult + a.diag_add;
  const double delta = cdiag - var;         // C - C_nonugget on the diagonal
  const bool want_like = a.Y != nullptr;

  double* Cp = smem + group_id * group_lds_doubles<K, BORDER>();   // packed lower triangle of C (incl. diag)
  // packed lower triangle of dC/dlog(phi); bordered: dC lives in registers through the row load,
  // then in the circulant layout W[(delta - 1) K + r] over the packed C
  double* dCp = BORDER ? Cp : Cp + K * (K + 1) / 2;
  double* nbx = Cp + (BORDER ? 1 : 2) * (K * (K + 1) / 2);  // K x kDMax (bordered: 2K x CS, two copies)
  // bordered: the slot aliases the coordinates (read only in the pair phase, before the slot's first
  // write; the next group's coordinate writes follow the slot reads in program order)
  double* slot_c = BORDER ? nbx : nbx + K * kDMax;          // column j of the current matrix
  double* slot_a1 = slot_c + K;                             // augmented entries (c, y_nbr)
  double* slot_a2 = slot_a1 + K;

  double acc[kVecchiaSums] = {0., 0., 0., 0., 0., 0.};
  unsigned long long tp[6] = {0, 0, 0, 0, 0, 0}, t0 = 0;
  const bool prof = PROF && blockIdx.x == 0 && threadIdx.x < 64;
  auto mark = [&](int q) {
    if (prof) {
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      const unsigned long long t1 = __builtin_amdgcn_s_memtime();
      tp[q] += t1 - t0;
      t0 = t1;
    }
  };

  const int total_groups = a.r1 - a.r0;
  for (int gbase_row = blockIdx.x * rows_per_block; gbase_row < total_groups; gbase_row += gridDim.x * rows_per_block) {
    if (prof) { t0 = __builtin_amdgcn_s_memtime(); ++tp[5]; }
    // bordered form: the lane index is made opaque per row group, so the lane-dependent LDS
    // addresses and pivot masks are recomputed each time instead of being hoisted out of the
    // loop (32 address VGPRs and 60 mask SGPRs held across the whole kernel)
    int r = r_lane;
    if constexpr (BORDER) asm volatile("" : "+v"(r));
    const int i = a.r0 + gbase_row + group_id;
    const bool active = i < a.r1;
    const int k = active ? min(i, a.m) : 0;
    const bool rv = r < k;
    const int irow = active ? i : a.r0;

    // ---- gather: neighbour index, coordinates, response (Vecchia order)
    const int nb = rv ? a.nbr[(size_t)(i - a.row_base) * a.m + r] : 0;
    double xi[kDMax], xr[kDMax];
#pragma unroll
    for (int q = 0; q < kDMax; ++q) {
      xi[q] = (q < d) ? a.X[(size_t)irow * d + q] : 0.;
      xr[q] = (q < d && rv) ? a.X[(size_t)nb * d + q] : 0.;
    }
    const double yi = want_like ? a.Y[irow] : 0.;
    const double ynb = (want_like && rv) ? a.Y[nb] : 0.;
    compiler_fence();   // previous iteration's LDS reads are issued before these writes
    // padding rows (r >= k) sit at distinct far-away points (1e30 (r + 1) on the first axis): their
    // covariances with every other row are exactly 0 (exp_nonpos clamps; the distance keeps the
    // Matern-2.5 derivative's x^3 finite for inverse ranges up to 1e72 and reaches the clamp for
    // ranges up to 1e27), so the pair phase needs no masking selects
#pragma unroll
    for (int q = 0; q < kDMax; ++q) {
      xr[q] = rv ? xr[q] : (q == 0 ? 1e30 * (r + 1) : 0.);
      if (q < CS) {
        nbx[r * CS + q] = xr[q];
        if constexpr (BORDER) nbx[(r + K) * CS + q] = xr[q];   // second copy: partner r + delta < 2K
      }
    }

    // observation-neighbour covariance c_r and its range derivative
    double cvec = 0., dcvec = 0.;
    {
      double s = 0.;
#pragma unroll
      for (int q = 0; q < ND; ++q) { const double t = xi[q] - xr[q]; s += t * t; }
      double cv, dcv;
      cov_dcov_sq<COV>(s, var, phi, cv, dcv);
      cvec = rv ? cv : 0.;
      dcvec = rv ? dcv : 0.;
    }
    Cp[packed(r, r)] = rv ? cdiag : 1.;
    if constexpr (!BORDER) dCp[packed(r, r)] = 0.;
    wave_lds_sync();
    mark(0);

    double wst[K / 2];   // bordered: dC of the lane's circulant pairs (delta = 1..K/2)
    // ---- 1. pairs (rr > cc): lanes l and l + K/2 share the rows {h, K-1-h}, h = l mod K/2: row h's
    // pairs are q = 0..h-1, row K-1-h's are q = h..K-2 (column q - h); lane l takes q = 0..K/2-1,
    // lane l + K/2 takes q = K/2..K-2. Per pair one compare selects between two precomputed bases
    // (row, column-coordinate and packed-entry addresses), the rest is an immediate offset.
    if constexpr (BORDER) {
      // lane r computes the pairs {r, (r + delta) mod K}, delta = 1..K/2 (circulant split: every
      // pair once, the K/2 pairs of delta = K/2 twice with identical values). Own coordinates stay
      // in registers, the partner's are read from the second coordinate copy at an immediate
      // offset; the destination packed(r + delta, r) = T(r) + r + r delta + T(delta) or, past the
      // wrap, packed(r, r + delta - K) = T(r) + r + delta - K (T(x) = x (x + 1) / 2).
      const int base = r * (r + 1) / 2 + r;
#pragma unroll
      for (int dl = 1; dl <= K / 2; ++dl) {
        const double* xp = nbx + (r + dl) * CS;
        double s = 0.;
#pragma unroll
        for (int qq = 0; qq < ND; ++qq) {
          const double t = xr[qq] - xp[qq];
          s += t * t;
        }
        double cv, dcv;
        cov_dcov_sq<COV>(s, var, phi, cv, dcv);
        const int pos = (r + dl < K) ? base + r * dl + dl * (dl + 1) / 2 : base + dl - K;
        Cp[pos] = cv;
        wst[dl - 1] = dcv;
      }
    } else {
      const int h = r & (K / 2 - 1);
      const int qlo = (r >= K / 2) ? K / 2 : 0;
      const double* xA = nbx + h * kDMax;                       // row h
      const double* xB = nbx + (K - 1 - h) * kDMax;             // row K-1-h
      const double* cA = nbx + qlo * kDMax;                     // column q     (q < h)
      const double* cB = nbx + (qlo - h) * kDMax;               // column q - h (q >= h)
      double* pA = Cp + packed(h, 0) + qlo;                     // packed(h, q)
      double* pB = Cp + packed(K - 1 - h, 0) - h + qlo;         // packed(K-1-h, q-h)
      constexpr int dCoff = K * (K + 1) / 2;                    // dCp - Cp
#pragma unroll kPairUnroll
      for (int qi = 0; qi < K / 2; ++qi) {
        const bool lo = qlo + qi < h;
        const double* xrr = lo ? xA : xB;
        const double* xcc = (lo ? cA : cB) + qi * kDMax;
        double* pe = (lo ? pA : pB) + qi;
        double s = 0.;
#pragma unroll
        for (int qq = 0; qq < kDMax; ++qq) {
          const double t = xrr[qq] - xcc[qq];
          s += t * t;
        }
        double cv, dcv;
        cov_dcov_sq<COV>(s, var, phi, cv, dcv);
        if (qi < K / 2 - 1 || qlo == 0) {   // lane l + K/2 has one pair less
          pe[0] = cv;
          pe[dCoff] = dcv;
        }
      }
    }
    wave_lds_sync();
    if constexpr (BORDER) {   // border rows MK (c) and MK + 1 (y_nbr) of the packed image
      if (r < MK) {
        Cp[packed(MK, r)] = cvec;
        Cp[packed(MK + 1, r)] = ynb;
      }
      wave_lds_sync();
    }
    mark(1);

    // ---- 2. symmetric Gauss-Jordan on [C | c | y_nbr], row r in registers
    double row[NC];
#pragma unroll
    for (int c = 0; c < NC; ++c) row[c] = (c <= r) ? Cp[packed(r, c)] : Cp[packed(c, r)];
    if constexpr (BORDER) {
      // dC over the packed C in the circulant layout (lane base + immediate; the row reads above
      // precede these writes in the wave's LDS order)
      compiler_fence();
#pragma unroll
      for (int dl = 1; dl <= K / 2; ++dl) dCp[(dl - 1) * K + r] = wst[dl - 1];
    }
    double aug1 = cvec, aug2 = ynb;
    double av_r = 0., vv_r = 0.;   // a = C^-1 c, v = C^-1 y_nbr (lanes r >= MK hold no row)
    if constexpr (BORDER) {
      // native 16-byte vector type: HIP's double2 struct is loaded field-wise (ds_read2_b64, 4x the
      // LDS cycles of ds_read_b128 per byte)
      typedef double v2d __attribute__((ext_vector_type(2)));
      auto recip = [](double piv) {   // hardware reciprocal + two Newton steps (~1 ulp)
        double x = __builtin_amdgcn_rcp(piv);
        x = fma(x, fma(-piv, x, 1.), x);
        return fma(x, fma(-piv, x, 1.), x);
      };
      const v2d* slot2 = reinterpret_cast<const v2d*>(__builtin_assume_aligned(slot_c, 16));
#pragma unroll
      for (int j = 0; j < MK; ++j) {
        double sv[NC];
        compiler_fence();
        slot_c[r] = row[j];
        wave_lds_sync();
#pragma unroll
        for (int p = j >> 1; p < NC / 2; ++p) {
          const v2d v = slot2[p];
          sv[2 * p] = v.x;
          sv[2 * p + 1] = v.y;
        }
        const double rinv = recip(sv[j]);
        const double q = row[j] * rinv;
        const double f = (r == j) ? 0. : q;
#pragma unroll
        for (int c = j + 1; c < NC; ++c) row[c] = fma(-f, sv[c], row[c]);
#pragma unroll
        for (int c = j + 1; c < NC; ++c) asm volatile("" : "+v"(row[c]));
      }
      aug1 = row[NC - 2];
      aug2 = row[NC - 1];
    } else if constexpr (DPPBC) {
      // lane c holds row c, so M[c][j] = lane c's row[j]: broadcast lane c's register
      auto bc = [&](auto CPc, double v, double& lo, double& hi) {
        constexpr int cp = decltype(CPc)::value;
        if constexpr (K == 32) {
          group_bcast_pair<cp>(v, lo, hi);
        } else {
          lo = row_bcast<cp>(v);
          hi = 0.;
        }
      };
      static_for<0, MK>([&](auto J) {
        constexpr int j = decltype(J)::value;
        constexpr int jp = j & 15;
        double plo, phi_, a1lo, a1hi, a2lo, a2hi;
        bc(std::integral_constant<int, jp>{}, row[j], plo, phi_);
        bc(std::integral_constant<int, jp>{}, aug1, a1lo, a1hi);
        bc(std::integral_constant<int, jp>{}, aug2, a2lo, a2hi);
        const double piv = j < 16 ? plo : phi_;
        const double a1j = j < 16 ? a1lo : a1hi;
        const double a2j = j < 16 ? a2lo : a2hi;
        double rinv = __builtin_amdgcn_rcp(piv);
        rinv = fma(rinv, fma(-piv, rinv, 1.), rinv);
        rinv = fma(rinv, fma(-piv, rinv, 1.), rinv);
        const double q = row[j] * rinv;
        const double f = (r == j) ? 0. : q;
        aug1 = fma(-f, a1j, aug1);
        aug2 = fma(-f, a2j, aug2);
        // columns c > j in pairs (cp, cp + 16) sharing one broadcast sequence
        static_for<0, 16>([&](auto CP) {
          constexpr int cp = decltype(CP)::value;
          constexpr bool need_lo = cp > j && cp < MK;
          constexpr bool need_hi = K == 32 && cp + 16 > j && cp + 16 < MK;
          if constexpr (need_lo || need_hi) {
            double vlo, vhi;
            if constexpr (cp == jp) {   // the pivot's broadcast already holds this pair
              vlo = plo;
              vhi = phi_;
            } else {
              bc(CP, row[j], vlo, vhi);
            }
            if constexpr (need_lo) row[cp] = fma(-f, vlo, row[cp]);
            if constexpr (need_hi) row[cp + 16] = fma(-f, vhi, row[cp + 16]);
          }
        });
#pragma unroll
        for (int c = j + 1; c < MK; ++c) asm volatile("" : "+v"(row[c]));
        asm volatile("" : "+v"(aug1), "+v"(aug2));
      });
    } else {
#pragma unroll
    for (int j = 0; j < MK; ++j) {
      compiler_fence();
      slot_c[r] = row[j];
      slot_a1[r] = aug1;
      slot_a2[r] = aug2;
      wave_lds_sync();
      const double piv = slot_c[j];
      // 1/piv by hardware reciprocal + two Newton steps (~1 ulp), cheaper than IEEE division
      double rinv = __builtin_amdgcn_rcp(piv);
      rinv = fma(rinv, fma(-piv, rinv, 1.), rinv);
      rinv = fma(rinv, fma(-piv, rinv, 1.), rinv);
      const double q = row[j] * rinv;
      const double f = (r == j) ? 0. : q;
      aug1 = fma(-f, slot_a1[j], aug1);
      aug2 = fma(-f, slot_a2[j], aug2);
#pragma unroll
      for (int c = j + 1; c < MK; ++c) row[c] = fma(-f, slot_c[c], row[c]);
      // Pin this step's updates here: without it the scheduler defers each column's FMAs to
      // the step that consumes it and keeps every broadcast value live (register blow-up).
#pragma unroll
      for (int c = j + 1; c < MK; ++c) asm volatile("" : "+v"(row[c]));
      asm volatile("" : "+v"(aug1), "+v"(aug2));
    }
    }
    {
    double mydiag = row[0];
#pragma unroll
    for (int c = 1; c < MK; ++c) mydiag = (c == r) ? row[c] : mydiag;
    if constexpr (BORDER) {   // one reciprocal (rcp + two Newton steps, ~1 ulp) for both quotients
      double dinv = __builtin_amdgcn_rcp(mydiag);
      dinv = fma(dinv, fma(-mydiag, dinv, 1.), dinv);
      dinv = fma(dinv, fma(-mydiag, dinv, 1.), dinv);
      av_r = rv ? aug1 * dinv : 0.;
      vv_r = rv ? aug2 * dinv : 0.;
    } else {
      av_r = rv ? aug1 / mydiag : 0.;
      vv_r = rv ? aug2 / mydiag : 0.;
    }
    }

    if (active && a.B_out != nullptr && r < a.m) a.B_out[(size_t)(i - a.row_base) * a.m + r] = rv ? -av_r : 0.;
    mark(2);

    // ---- 3. the dC forms a^T dC a and v^T dC a. Bordered: per lane over its circulant pairs
    // {r, p = r + delta}: with S1 = sum_{delta < K/2} w a_p, S1h = w_{K/2} a_{p}, S2 = sum_{delta < K/2} w v_p,
    // lane r adds a_r (2 S1 + S1h) to a^T dC a and v_r (S1 + S1h) + a_r S2 to v^T dC a (every ordered
    // pair once; the delta = K/2 pairs are held by both of their lanes). [a, v] pairs sit in a
    // doubled slot array, so p's entry is a 16-byte read at an immediate offset.
    double tA, tV;   // this lane's shares of a^T dC a and v^T dC a
    if constexpr (BORDER) {
      typedef double v2d __attribute__((ext_vector_type(2)));
      v2d* av2 = reinterpret_cast<v2d*>(__builtin_assume_aligned(nbx, 16));
      compiler_fence();
      const v2d mine = {av_r, vv_r};
      av2[r] = mine;
      av2[r + K] = mine;
      wave_lds_sync();
      double s1[2] = {0., 0.}, s2[2] = {0., 0.};
#pragma unroll
      for (int dl = 1; dl < K / 2; ++dl) {
        const double w = dCp[(dl - 1) * K + r];
        const v2d pv = av2[r + dl];
        s1[dl & 1] = fma(w, pv.x, s1[dl & 1]);
        s2[dl & 1] = fma(w, pv.y, s2[dl & 1]);
      }
      const double s1h = dCp[(K / 2 - 1) * K + r] * av2[r + K / 2].x;
      const double S1 = s1[0] + s1[1], S2 = s2[0] + s2[1];
      tA = av_r * (2. * S1 + s1h);
      tV = vv_r * (S1 + s1h) + av_r * S2;
    } else {
      // t = dC a (dC from the packed image; its diagonal is 0)
      compiler_fence();
      slot_c[r] = av_r;
      wave_lds_sync();
      // entries with c >= k are exact zeros (padding rows of dC and of a), so the sum runs over
      // all K columns, unrolled with four partial sums
      double tq[4] = {0., 0., 0., 0.};
#pragma unroll
      for (int c = 0; c < MK; ++c) {
        const double dcrc = (c < r) ? dCp[packed(r, c)] : dCp[packed(c, r)];
        tq[c & 3] = fma(dcrc, slot_c[c], tq[c & 3]);
      }
      double t = (tq[0] + tq[1]) + (tq[2] + tq[3]);
      t = rv ? t : 0.;
      tA = t * av_r;
      tV = t * vv_r;
    }
    mark(3);

    // ---- group reductions
    double ac, ay, aa, avv, dD_rng, uk_rng;
    if constexpr (K == 32) {
      // row 0 of the group sums {ac, ay, aa, avv}, row 1 {dca, dcv, ta, tv}; row 1 forms the two
      // range terms and hands them to row 0
      const double v8[8] = {av_r * cvec, av_r * ynb, av_r * av_r, av_r * vv_r,
                            dcvec * av_r, dcvec * vv_r, tA, tV};
      double s4[4];
      group_sum8_rows(v8, s4);
      ac = s4[0];
      ay = s4[1];
      aa = s4[2];
      avv = s4[3];
      dD_rng = odd_row_value(-(2. * s4[0] - s4[2]));   // row 1: -(2 dca - ta)
      uk_rng = odd_row_value(-(s4[1] - s4[3]));        // row 1: -(dcv - tv)
    } else {
      ac = group_sum<K>(av_r * cvec);
      ay = group_sum<K>(av_r * ynb);
      aa = group_sum<K>(av_r * av_r);
      avv = group_sum<K>(av_r * vv_r);
      const double dca = group_sum<K>(dcvec * av_r);
      const double dcv = group_sum<K>(dcvec * vv_r);
      const double ta = group_sum<K>(tA);
      const double tv = group_sum<K>(tV);
      dD_rng = -(2. * dca - ta);                         // dD/dlog phi
      uk_rng = -(dcv - tv);                              // (dB_range y)_i
    }

    const double D = var + a.d_nugget - ac;          // Vecchia_utils.cpp:1351, 1507, 1562
    const double Dinv = 1. / D;
    if (active && r == 0 && a.Dinv_out != nullptr) a.Dinv_out[i - a.row_base] = Dinv;
    if (want_like && active && r == 0) {
      const double By = yi - ay;                         // (B y)_i
      const double u = By * Dinv;                        // (D^-1 B y)_i
      const double dD_var = var - delta * aa - ac;       // dD/dlog var
      const double uk_var = -delta * avv;                // (dB_var y)_i
      acc[0] += log(D);
      acc[1] += By * u;
      acc[2] += uk_var * u - 0.5 * u * u * dD_var;
      acc[3] += uk_rng * u - 0.5 * u * u * dD_rng;
      acc[4] += Dinv * dD_var;
      acc[5] += Dinv * dD_rng;
    }
    mark(4);
  }
  if (prof && threadIdx.x == 0)
    for (int q = 0; q < 6; ++q) g_rows_prof[q] = tp[q];
  if (!want_like) return;

  // ---- block reduction of the per-group sums (fixed order -> deterministic)
  __syncthreads();
  double* red = smem;  // reuse: rows_per_block x kVecchiaSums
  if (r_lane == 0) {
#pragma unroll
    for (int s = 0; s < kVecchiaSums; ++s) red[group_id * kVecchiaSums + s] = acc[s];
  }
  __syncthreads();
  if (threadIdx.x < kVecchiaSums) {
    double v = 0.;
    for (int gi = 0; gi < rows_per_block; ++gi) v += red[gi * kVecchiaSums + threadIdx.x];
    a.block_sums[(size_t)blockIdx.x * kVecchiaSums + threadIdx.x] = v;
  }
}

// ---------------------------------------------------------------- v4: two matrix rows per lane
// For K = 16 / 32 (m <= 32) a row problem is owned by H = K/2 lanes; lane h owns matrix rows
// h and h + H. v3 is bound by LDS traffic (one ds_read broadcast per FMA in the Gauss-Jordan
// steps plus three slot writes per step, on an LDS shared by the CU's four SIMDs). Here every
// broadcast feeds two FMAs, the pivot row's augmented entries come from the pivot lane by a
// lane shuffle instead of LDS slots, and the packed triangle holds C until the rows are in
// registers and dC/dlog(phi) afterwards (the pair phase keeps dC in registers meanwhile), so
// a problem needs one triangle instead of two. The per-row arithmetic is v3's.
constexpr int kV4Threads = 64;   // one wave per block: 64 / H problems

template <int K>
constexpr int v4_lds_doubles() {
  return K * (K + 1) / 2 + kDMax * K + K;   // packed C (then dC) | neighbour coords | pivot slot
}

template <int K, int COV>
__global__ void __launch_bounds__(kV4Threads, 1) vecchia_rows2_kernel(VecchiaRowsArgs a) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  constexpr int H = K / 2;   // lanes per problem
  constexpr int P = 64 / H;  // problems per wave (= per block)
  const int lane = threadIdx.x & 63;
  const int g = lane / H;
  const int h = lane - g * H;
  const int gbase = g * H;
  const int r0 = h, r1 = h + H;
  const int d = a.d;
  const double var = a.var, phi = a.phi;
  const double cdiag = var * a.diag_mult + a.diag_add;
  const double delta = cdiag - var;
  const bool want_like = a.Y != nullptr;

  double* Cp = smem + g * v4_lds_doubles<K>();
  double* nbx = Cp + K * (K + 1) / 2;
  double* slot = nbx + K * kDMax;

  double acc[kVecchiaSums] = {0., 0., 0., 0., 0., 0.};
  const int total = a.r1 - a.r0;
  for (int base = blockIdx.x * P; base < total; base += gridDim.x * P) {
    const int i = a.r0 + base + g;
    const bool active = i < a.r1;
    const int k = active ? min(i, a.m) : 0;
    const bool v0 = r0 < k, v1 = r1 < k;
    const int irow = active ? i : a.r0;

    // ---- gather: neighbour indices, coordinates, responses (Vecchia order)
    const int nb0 = v0 ? a.nbr[(size_t)(i - a.row_base) * a.m + r0] : 0;
    const int nb1 = v1 ? a.nbr[(size_t)(i - a.row_base) * a.m + r1] : 0;
    double xi[kDMax], x0[kDMax], x1[kDMax];
#pragma unroll
    for (int q = 0; q < kDMax; ++q) {
      xi[q] = (q < d) ? a.X[(size_t)irow * d + q] : 0.;
      x0[q] = (q < d && v0) ? a.X[(size_t)nb0 * d + q] : 0.;
      x1[q] = (q < d && v1) ? a.X[(size_t)nb1 * d + q] : 0.;
    }
    const double yi = want_like ? a.Y[irow] : 0.;
    const double y0 = (want_like && v0) ? a.Y[nb0] : 0.;
    const double y1 = (want_like && v1) ? a.Y[nb1] : 0.;
    compiler_fence();   // previous iteration's LDS reads are issued before these writes
#pragma unroll
    for (int q = 0; q < kDMax; ++q) {
      nbx[r0 * kDMax + q] = x0[q];
      nbx[r1 * kDMax + q] = x1[q];
    }
    // observation-neighbour covariances c and their range derivatives
    double c0, dc0, c1, dc1;
    {
      double s0 = 0., s1 = 0.;
#pragma unroll
      for (int q = 0; q < kDMax; ++q) {
        const double t0 = xi[q] - x0[q], t1 = xi[q] - x1[q];
        s0 += t0 * t0;
        s1 += t1 * t1;
      }
      cov_dcov<COV>(sqrt(s0), var, phi, c0, dc0);
      cov_dcov<COV>(sqrt(s1), var, phi, c1, dc1);
      c0 = v0 ? c0 : 0.;
      dc0 = v0 ? dc0 : 0.;
      c1 = v1 ? c1 : 0.;
      dc1 = v1 ? dc1 : 0.;
    }
    Cp[packed(r0, r0)] = v0 ? cdiag : 1.;
    Cp[packed(r1, r1)] = v1 ? cdiag : 1.;
    wave_lds_sync();

    // ---- 1. pairs: lane h takes row h (columns < h) and row K-1-h (columns < K-1-h)
    double dstash[K - 1];
#pragma unroll
    for (int q = 0; q < K - 1; ++q) {
      const bool lo = q < h;
      const int rr = lo ? h : K - 1 - h;
      const int cc = lo ? q : q - h;
      double s = 0.;
#pragma unroll
      for (int qq = 0; qq < kDMax; ++qq) {
        const double t = nbx[rr * kDMax + qq] - nbx[cc * kDMax + qq];
        s += t * t;
      }
      double cv, dcv;
      cov_dcov<COV>(sqrt(s), var, phi, cv, dcv);
      Cp[packed(rr, cc)] = rr < k ? cv : 0.;
      dstash[q] = rr < k ? dcv : 0.;
    }
    wave_lds_sync();

    // ---- 2. rows r0, r1 of C into registers; then the triangle becomes dC
    double row0[K], row1[K];
#pragma unroll
    for (int c = 0; c < K; ++c) {
      row0[c] = (c <= r0) ? Cp[packed(r0, c)] : Cp[packed(c, r0)];
      row1[c] = (c <= r1) ? Cp[packed(r1, c)] : Cp[packed(c, r1)];
    }
    wave_lds_sync();   // every lane's reads of C have returned before dC overwrites it
#pragma unroll
    for (int q = 0; q < K - 1; ++q) {
      const bool lo = q < h;
      const int rr = lo ? h : K - 1 - h;
      const int cc = lo ? q : q - h;
      Cp[packed(rr, cc)] = dstash[q];
    }
    Cp[packed(r0, r0)] = 0.;
    Cp[packed(r1, r1)] = 0.;

    // ---- 3. symmetric Gauss-Jordan on [C | c | y_nbr], rows r0 and r1 in registers
    double p0a = c0, p0b = y0, p1a = c1, p1b = y1;
#pragma unroll
    for (int j = 0; j < K; ++j) {
      compiler_fence();
      slot[r0] = row0[j];
      slot[r1] = row1[j];
      // augmented entries of pivot row j, from its owner (row j < H: lane j's r0, else r1)
      const int src = gbase + (j < H ? j : j - H);
      const double sa1 = __shfl(j < H ? p0a : p1a, src, 64);
      const double sa2 = __shfl(j < H ? p0b : p1b, src, 64);
      wave_lds_sync();
      const double piv = slot[j];
      double rinv = __builtin_amdgcn_rcp(piv);
      rinv = fma(rinv, fma(-piv, rinv, 1.), rinv);
      rinv = fma(rinv, fma(-piv, rinv, 1.), rinv);
      // the pivot row itself is left unchanged
      const double f0 = (j < H && r0 == j) ? 0. : row0[j] * rinv;
      const double f1 = (j >= H && r1 == j) ? 0. : row1[j] * rinv;
      p0a = fma(-f0, sa1, p0a);
      p0b = fma(-f0, sa2, p0b);
      p1a = fma(-f1, sa1, p1a);
      p1b = fma(-f1, sa2, p1b);
#pragma unroll
      for (int c = j + 1; c < K; ++c) {
        const double s = slot[c];
        row0[c] = fma(-f0, s, row0[c]);
        row1[c] = fma(-f1, s, row1[c]);
      }
      // pin this step's updates here (see v3: otherwise every broadcast value stays live)
#pragma unroll
      for (int c = j + 1; c < K; ++c) asm volatile("" : "+v"(row0[c]), "+v"(row1[c]));
      asm volatile("" : "+v"(p0a), "+v"(p0b), "+v"(p1a), "+v"(p1b));
    }
    double dg0 = row0[0], dg1 = row1[H];
#pragma unroll
    for (int c = 1; c < H; ++c) dg0 = (c == r0) ? row0[c] : dg0;
#pragma unroll
    for (int c = H + 1; c < K; ++c) dg1 = (c == r1) ? row1[c] : dg1;
    const double a0 = p0a / dg0, w0 = p0b / dg0;   // a = C^-1 c, v = C^-1 y_nbr
    const double a1 = p1a / dg1, w1 = p1b / dg1;

    if (active && a.B_out != nullptr) {
      if (r0 < a.m) a.B_out[(size_t)(i - a.row_base) * a.m + r0] = v0 ? -a0 : 0.;
      if (r1 < a.m) a.B_out[(size_t)(i - a.row_base) * a.m + r1] = v1 ? -a1 : 0.;
    }

    // ---- 4. t = dC a (dC from the packed triangle; its diagonal is 0)
    compiler_fence();
    slot[r0] = a0;
    slot[r1] = a1;
    wave_lds_sync();
    double t0 = 0., t1 = 0.;
    for (int c = 0; c < k; ++c) {
      const double s = slot[c];
      t0 = fma((c < r0) ? Cp[packed(r0, c)] : Cp[packed(c, r0)], s, t0);
      t1 = fma((c < r1) ? Cp[packed(r1, c)] : Cp[packed(c, r1)], s, t1);
    }
    t0 = v0 ? t0 : 0.;
    t1 = v1 ? t1 : 0.;

    // ---- group reductions
    const double ac = group_sum<H>(a0 * c0 + a1 * c1);
    const double ay = group_sum<H>(a0 * y0 + a1 * y1);
    const double aa = group_sum<H>(a0 * a0 + a1 * a1);
    const double avv = group_sum<H>(a0 * w0 + a1 * w1);
    const double dca = group_sum<H>(dc0 * a0 + dc1 * a1);
    const double dcv = group_sum<H>(dc0 * w0 + dc1 * w1);
    const double ta = group_sum<H>(t0 * a0 + t1 * a1);
    const double tv = group_sum<H>(t0 * w0 + t1 * w1);

    const double D = var + a.d_nugget - ac;          // Vecchia_utils.cpp:1351, 1507, 1562
    const double Dinv = 1. / D;
    if (active && h == 0 && a.Dinv_out != nullptr) a.Dinv_out[i - a.row_base] = Dinv;
    if (want_like && active && h == 0) {
      const double By = yi - ay;
      const double u = By * Dinv;
      const double dD_var = var - delta * aa - ac;
      const double uk_var = -delta * avv;
      const double dD_rng = -(2. * dca - ta);
      const double uk_rng = -(dcv - tv);
      acc[0] += log(D);
      acc[1] += By * u;
      acc[2] += uk_var * u - 0.5 * u * u * dD_var;
      acc[3] += uk_rng * u - 0.5 * u * u * dD_rng;
      acc[4] += Dinv * dD_var;
      acc[5] += Dinv * dD_rng;
    }
  }
  if (!want_like) return;
  // ---- block (= wave) reduction of the per-problem sums, fixed order
  __syncthreads();
  double* red = smem;   // P x kVecchiaSums
  if (h == 0) {
#pragma unroll
    for (int s = 0; s < kVecchiaSums; ++s) red[g * kVecchiaSums + s] = acc[s];
  }
  __syncthreads();
  if (threadIdx.x < kVecchiaSums) {
    double v = 0.;
    for (int gi = 0; gi < P; ++gi) v += red[gi * kVecchiaSums + threadIdx.x];
    a.block_sums[(size_t)blockIdx.x * kVecchiaSums + threadIdx.x] = v;
  }
}

// A/B: GPB_SUM_FAST 1 = every partial load of a thread in flight at once and the published sums
// written through with system-scope stores (then the flag after their acknowledgement), 0 = four
// loads per step and a system-scope release fence (an L2 write-back) before the flag
#ifndef GPB_SUM_FAST
#define GPB_SUM_FAST 1
#endif
__global__ void __launch_bounds__(1024) sum_blocks_kernel(const double* __restrict__ in, int nblocks, int width,
                                                       double* __restrict__ out, unsigned long long* flag,
                                                       unsigned long long seq) {
  // width <= 8: thread t sums column (t & 7) over blocks (t >> 3) + 128 u
  __shared__ double red[1024];
  const int col = threadIdx.x & 7, lane_b = threadIdx.x >> 3;
#if GPB_SUM_FAST
  double acc = 0.;
  if (col < width) {
    constexpr int kU = 16;   // 2048 blocks (the row kernels' grid bound) in one round of loads
    int b0 = 0;
    for (; b0 + 128 * kU <= nblocks; b0 += 128 * kU) {
      double v[kU];
#pragma unroll
      for (int u = 0; u < kU; ++u) v[u] = in[(size_t)(b0 + lane_b + 128 * u) * width + col];
#pragma unroll
      for (int w = kU / 2; w >= 1; w >>= 1) {
#pragma unroll
        for (int u = 0; u < w; ++u) v[u] += v[u + w];
      }
      acc += v[0];
    }
    if (b0 < nblocks) {
      double v[kU];
#pragma unroll
      for (int u = 0; u < kU; ++u) {
        const int b = b0 + lane_b + 128 * u;
        v[u] = b < nblocks ? in[(size_t)b * width + col] : 0.;
      }
#pragma unroll
      for (int w = kU / 2; w >= 1; w >>= 1) {
#pragma unroll
        for (int u = 0; u < w; ++u) v[u] += v[u + w];
      }
      acc += v[0];
    }
  }
  red[threadIdx.x] = acc;
#else
  double acc0 = 0., acc1 = 0., acc2 = 0., acc3 = 0.;
  if (col < width) {
    int b = lane_b;
    for (; b + 384 < nblocks; b += 512) {
      acc0 += in[(size_t)b * width + col];
      acc1 += in[(size_t)(b + 128) * width + col];
      acc2 += in[(size_t)(b + 256) * width + col];
      acc3 += in[(size_t)(b + 384) * width + col];
    }
    for (; b < nblocks; b += 128) acc0 += in[(size_t)b * width + col];
  }
  red[threadIdx.x] = (acc0 + acc1) + (acc2 + acc3);
#endif
  __syncthreads();
  for (int off = 512; off >= 8; off >>= 1) {
    if ((int)threadIdx.x < off) red[threadIdx.x] += red[threadIdx.x + off];
    __syncthreads();
  }
#if GPB_SUM_FAST
  if ((int)threadIdx.x < width) {
    if (flag != nullptr) __hip_atomic_store(out + threadIdx.x, red[threadIdx.x], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    else out[threadIdx.x] = red[threadIdx.x];
  }
  if (flag != nullptr) {
    // Ordering of the sums before the flag: on gfx9 (this library targets gfx950 only) vmcnt also
    // counts stores, so waiting on it means the system-scope stores are acknowledged before the
    // barrier and the relaxed flag store. gfx10+ counts stores in vscnt instead: there this would
    // race, hence the guard.
#if defined(__HIP_DEVICE_COMPILE__) && !defined(__GFX9__)
#error "GPB_SUM_FAST relies on gfx9 vmcnt counting stores; use a release store for the flag elsewhere"
#endif
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the written-through sums are acknowledged
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_store(flag, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
#else
  if ((int)threadIdx.x < width) {
    out[threadIdx.x] = red[threadIdx.x];
    if (flag != nullptr) __threadfence_system();   // the sums reach the host before the flag
  }
  if (flag != nullptr) {
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_store(flag, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
#endif
}

// One thread per prediction point; entries in neighbour order.
__global__ void __launch_bounds__(256) predict_mean_var_kernel(int n_pred, int m, const int* __restrict__ nbr,
                                                               const double* __restrict__ B,
                                                               const double* __restrict__ Dinv,
                                                               const double* __restrict__ y, double sigma2,
                                                               double nugget_sub, double* __restrict__ out) {
  const int p = blockIdx.x * 256 + threadIdx.x;
  if (p >= n_pred) return;
  double mu = 0.;
  for (int r = 0; r < m; ++r) mu = fma(-B[(size_t)p * m + r], y[nbr[(size_t)p * m + r]], mu);
  out[p] = mu;
  out[n_pred + p] = (1. / Dinv[p] - nugget_sub) * sigma2;
}

int lanes_for_m(int m) {
  if (m <= 16) return 16;
  if (m <= 32) return 32;
  if (m <= 64) return 64;
  return 0;
}

// v3 is the default: measured on MI355X at n = 100k, m = 30 v4 took 0.578 ms per launch against
// v3's 0.474 ms (gpurun_out r01b). v4 (two rows per lane) stays selectable for K <= 32 with
// GPBOOST_AMD_ROWS_V4 for A/B measurements.
bool use_v4(int K) {
  static const bool v4 = std::getenv("GPBOOST_AMD_ROWS_V4") != nullptr;
  return K <= 32 && v4;
}

// Gauss-Jordan broadcasts: LDS slots (default) or DPP / row-swap permutes (GPBOOST_AMD_ROWS_DPP=1,
// A/B; read at every launch so a test can compare both forms in one process). Measured on MI355X
// (n = 100k, m = 30, profiles/r03/rows_dpp_ab_r03.log): DPP 0.604 ms vs LDS 0.378 ms per launch —
// 223 instead of 249 VGPRs, but every step's broadcast chain (row_newbcast -> permlane16_swap ->
// reciprocal -> FMAs) is a dependent VALU sequence with DPP hazard waits, while the LDS form issues
// the step's column reads as one burst whose latencies overlap.
bool rows_dpp() { return std::getenv("GPBOOST_AMD_ROWS_DPP") != nullptr; }
// Augmented entries: bordered rows (default where two lanes are spare) or the round-2 form with
// separate augmented slots (GPBOOST_AMD_ROWS_SLOTS=1, A/B; read at every launch).
bool rows_slots() { return std::getenv("GPBOOST_AMD_ROWS_SLOTS") != nullptr; }
// 16-lane form (vecchia_rows16.hip) for m <= 30, the default: measured on MI355X at n = 100k, m = 30
// (profiles/r03/rows_env_ab_r03i.log) 0.225 ms per launch against 0.284 ms for the bordered 32-lane
// LDS-broadcast form, which GPBOOST_AMD_ROWS16=0 selects (A/B; read at every launch)
bool rows16() {
  const char* e = std::getenv("GPBOOST_AMD_ROWS16");
  return e == nullptr || e[0] != '0';
}

template <int K>
int rows_per_block() { return use_v4(K) ? 64 / (K / 2) : (block_threads<K>() / 64) * (64 / K); }

template <int K>
int blocks_for(int rows) {
  const int rpb = rows_per_block<K>();
  const int need = (rows + rpb - 1) / rpb;
  return need < kMaxBlocks ? need : kMaxBlocks;
}

// Upper bound of any launch's grid (block-partial buffers are sized by it).
constexpr int kMaxBlocksAny = 2048;
static_assert(kMaxBlocks <= kMaxBlocksAny, "grid cap");

// Bordered forms: the grid is the resident capacity (blocks per CU from the occupancy calculator
// for this instance's registers and LDS, times the CU count), so every block strides over an
// equal share of row groups in a single round.
template <class KernelT>
int resident_grid(KernelT kernel, int threads, size_t lds, int rows, int rpb) {
  static int cap = 0;   // per kernel instance (one static per template instantiation)
  if (cap == 0) {
    int dev = 0, cus = 0, per_cu = 0;
    HIP_CHECK(hipGetDevice(&dev));
    HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, threads, lds));
    cap = std::max(1, std::min(per_cu * cus, kMaxBlocksAny));
  }
  const int need = (rows + rpb - 1) / rpb;
  return need < cap ? need : cap;
}

template <int K, int COV, int MK, int DIM>
int launch_border(const VecchiaRowsArgs& a, hipStream_t s) {
  constexpr int rpb = (block_threads<K>() / 64) * (64 / K);
  const size_t red = (size_t)rpb * kVecchiaSums * sizeof(double);
  size_t lds = (size_t)rpb * group_lds_doubles<K, true>() * sizeof(double);
  if (lds < red) lds = red;
  auto kern = vecchia_rows_kernel<K, COV, false, MK, false, true, DIM>;
  const int blocks = resident_grid(kern, block_threads<K>(), lds, a.r1 - a.r0, rpb);
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(block_threads<K>()), lds, s, a);
  HIP_CHECK(hipGetLastError());
  return blocks;
}

template <int K, int COV>
int launch_k(const VecchiaRowsArgs& a, hipStream_t s) {
  const int rpb = rows_per_block<K>();
  const int blocks = blocks_for<K>(a.r1 - a.r0);
  const size_t red = (size_t)rpb * kVecchiaSums * sizeof(double);
  if constexpr (K <= 32) {
    if (use_v4(K)) {
      size_t lds = (size_t)rpb * v4_lds_doubles<K>() * sizeof(double);
      if (lds < red) lds = red;
      hipLaunchKernelGGL((vecchia_rows2_kernel<K, COV>), dim3(blocks), dim3(kV4Threads), lds, s, a);
      HIP_CHECK(hipGetLastError());
      return blocks;
    }
  }
  size_t lds = (size_t)rpb * group_lds_doubles<K>() * sizeof(double);
  if (lds < red) lds = red;
  static const bool prof = std::getenv("GPBOOST_AMD_ROWS_PROF") != nullptr;
  const bool dpp = rows_dpp();
  if constexpr (K == 32) {
    if (!prof && a.m <= 30) {   // the headline configuration (m = 30): 30 elimination steps
      if (rows16() && !dpp && !rows_slots()) return launch_vecchia_rows16(COV, a, s);
      if (dpp) {
        hipLaunchKernelGGL((vecchia_rows_kernel<K, COV, false, 30, true>), dim3(blocks), dim3(block_threads<K>()), lds, s, a);
      } else if (rows_slots()) {
        hipLaunchKernelGGL((vecchia_rows_kernel<K, COV, false, 30>), dim3(blocks), dim3(block_threads<K>()), lds, s, a);
      } else if (a.d == 2) {   // planar coordinates (the BASELINE configurations)
        return launch_border<K, COV, 30, 2>(a, s);
      } else {
        return launch_border<K, COV, 30, 0>(a, s);
      }
      HIP_CHECK(hipGetLastError());
      return blocks;
    }
  }
  if constexpr (K == 16) {
    if (!prof && !dpp && a.m <= K - 2 && !rows_slots()) return launch_border<K, COV, K - 2, 0>(a, s);   // m <= 14
  }
  if constexpr (K == 16 || K == 32) {
    if (!prof && dpp) {
      hipLaunchKernelGGL((vecchia_rows_kernel<K, COV, false, K, true>), dim3(blocks), dim3(block_threads<K>()), lds, s, a);
      HIP_CHECK(hipGetLastError());
      return blocks;
    }
  }
  if (prof) {
    hipLaunchKernelGGL((vecchia_rows_kernel<K, COV, true>), dim3(blocks), dim3(block_threads<K>()), lds, s, a);
    unsigned long long h[8];
    HIP_CHECK(hipStreamSynchronize(s));
    HIP_CHECK(hipMemcpyFromSymbol(h, HIP_SYMBOL(g_rows_prof), sizeof(h)));
    std::fprintf(stderr, "[rows prof] K=%d blocks=%d iterations=%llu cycles: gather %llu pairs %llu gj %llu dca %llu reduce %llu\n",
                 K, blocks, h[5], h[0], h[1], h[2], h[3], h[4]);
  } else {
    hipLaunchKernelGGL((vecchia_rows_kernel<K, COV>), dim3(blocks), dim3(block_threads<K>()), lds, s, a);
  }
  HIP_CHECK(hipGetLastError());
  return blocks;
}

template <int K>
int launch_cov(int cov, const VecchiaRowsArgs& a, hipStream_t s) {
  switch (cov) {
    case kMatern05: return launch_k<K, kMatern05>(a, s);
    case kMatern15: return launch_k<K, kMatern15>(a, s);
    case kMatern25: return launch_k<K, kMatern25>(a, s);
    case kGaussian: return launch_k<K, kGaussian>(a, s);
    default: Fatal("unsupported covariance type %d", cov);
  }
  return 0;
}

}  // namespace

int vecchia_rows_blocks(int rows, int m) {
  if (lanes_for_m(m) == 0) Fatal("num_neighbors = %d > 64 is not supported by the GPU Vecchia kernel", m);
  return std::min(std::max(rows, 1), kMaxBlocksAny);   // >= any launch's grid (one row group per block at least)
}

int launch_vecchia_rows(int cov_type, const VecchiaRowsArgs& a, hipStream_t s) {
  if (a.d < 1 || a.d > kDMax) Fatal("GPU Vecchia kernel supports 1 <= dim_gp_coords <= %d, got %d", kDMax, a.d);
  if (a.r1 <= a.r0) return 0;
  switch (lanes_for_m(a.m)) {
    case 16: return launch_cov<16>(cov_type, a, s);
    case 32: return launch_cov<32>(cov_type, a, s);
    case 64: return launch_cov<64>(cov_type, a, s);
    default: Fatal("num_neighbors = %d > 64 is not supported by the GPU Vecchia kernel", a.m);
  }
  return 0;
}

void launch_predict_mean_var(int n_pred, int m, const int* nbr, const double* B, const double* Dinv, const double* y,
                             double sigma2, double nugget_sub, double* out, hipStream_t s) {
  if (n_pred <= 0) return;
  hipLaunchKernelGGL(predict_mean_var_kernel, dim3((n_pred + 255) / 256), dim3(256), 0, s, n_pred, m, nbr, B, Dinv, y,
                     sigma2, nugget_sub, out);
  HIP_CHECK(hipGetLastError());
}

void launch_sum_blocks(const double* block_sums, int nblocks, int width, double* out, hipStream_t s,
                       unsigned long long* flag, unsigned long long seq) {
  if (width > 8) Fatal("sum_blocks: width %d > 8", width);
  hipLaunchKernelGGL(sum_blocks_kernel, dim3(1), dim3(1024), 0, s, block_sums, nblocks, width, out, flag, seq);
  HIP_CHECK(hipGetLastError());
}

}  // namespace gpb_amd
