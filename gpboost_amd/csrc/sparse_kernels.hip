// Sparse Vecchia operators and block-CG vector kernels for the iterative path (gfx950).
//
// Reference replaced (CG_utils.cpp:21-217, likelihoods.h:2765-3076, 4951-5206,
// 12069-12546): the row-major Eigen SpMVs B*h, B^T*(D^-1 B h), the two triangular solves
// of the VADU preconditioner, the block-CG column updates and the column / row
// reductions of the stochastic traces.
//
// Thread mapping for blocks of t vectors stored row-major n x t: a group of T lanes
// (T = next power of two >= t, at most 64) owns one row; lane c owns column
// c + 64*blockIdx.y. A neighbour gather is therefore one contiguous t*8-byte read, and
// the per-row sparse pattern (nbr / values) is a same-address broadcast across the group.
// All reductions are two-pass with fixed orders, so results are bitwise reproducible.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>

#include "common.h"
#include "latent_kernels.h"
#include "lik_device.h"
#include "wave_ops.h"

namespace gpb_amd {
namespace {

constexpr int kBT = 256;          // threads per block
constexpr int kMaxGridX = 4096;

struct Lanes {
  int shift;  // log2(T)
  int T;
  int rpb;    // rows per block
  int gy;     // grid.y (column chunks of 64)
};

Lanes lanes_for(int t) {
  Lanes L;
  int T = 1, sh = 0;
  const int tc = t < 64 ? t : 64;
  while (T < tc) { T <<= 1; ++sh; }
  L.shift = sh;
  L.T = T;
  L.rpb = kBT >> sh;
  L.gy = (t + 63) / 64;
  return L;
}

int grid_x(int rows, int rpb, int cap = kMaxGridX) {
  int g = (rows + rpb - 1) / rpb;
  if (g > cap) g = cap;
  return g < 1 ? 1 : g;
}

// ------------------------------------------------------------------ SpMV
// Workgroups are dispatched round-robin over the 8 XCDs (block b on XCD b % 8). Rows are
// stored in a locality order (LatentVecchia::Relabel), so consecutive rows share most of
// their neighbours: give every XCD one contiguous range of row blocks so those shared
// neighbour rows are served from that XCD's L2.

// Row r of a t >= 2 operator runs on the lane group of (block, slot): with PERS the grid is
// capped and block b walks the row groups [L*span, (L+1)*span) of its logical index
// L = xcd_block(b) (one contiguous, spatially coherent range per XCD); otherwise one row
// group per block. CH = 0: the row's entries one after another (unroll 4); CH > 0: CH
// structure loads, then CH gathers in flight. Summation order is the same in every form:
// unit term, then entries ascending.
template <int CH>
__device__ __forceinline__ double row_dot(const int* __restrict__ idx, const double* __restrict__ val, int k,
                                          const double* __restrict__ pre, const double* __restrict__ X, int t, int c,
                                          int self, double s) {
  if constexpr (CH == 0) {
#pragma unroll 4
    for (int r = 0; r < k; ++r) {
      const int j = idx[r];
      const double w = pre ? val[r] * pre[j] : val[r];
      s = fma(w, X[(size_t)j * t + c], s);
    }
  } else {
    for (int r0 = 0; r0 < k; r0 += CH) {
      int id[CH];
      double w[CH], g[CH];
#pragma unroll
      for (int q = 0; q < CH; ++q) {
        const bool ok = r0 + q < k;
        id[q] = ok ? idx[r0 + q] : self;
        const double v = ok ? val[r0 + q] : 0.;
        w[q] = pre ? v * pre[id[q]] : v;
      }
#pragma unroll
      for (int q = 0; q < CH; ++q) g[q] = X[(size_t)id[q] * t + c];
#pragma unroll
      for (int q = 0; q < CH; ++q) s = fma(w[q], g[q], s);
    }
  }
  return s;
}

struct RowWalk {
  int g0, g1;   // row groups of this block
};
template <bool PERS>
__device__ __forceinline__ RowWalk row_walk(int ngroups) {
  if (!PERS) return {(int)blockIdx.x, (int)blockIdx.x + 1};
  const int G = gridDim.x;
  const int span = (ngroups + G - 1) / G;
  const int L = xcd_block(blockIdx.x, G);
  const int g0 = L * span;
  return {g0, min(g0 + span, ngroups)};
}

// Y = diag(scale) (unit*X + V X)
template <int CH, bool PERS>
__global__ void __launch_bounds__(kBT) b_apply_kernel(int n, int m, const int* __restrict__ nbr,
                                                      const double* __restrict__ vals, int unit,
                                                      const double* __restrict__ X, int t, int shift,
                                                      const double* __restrict__ scale, double* __restrict__ Y) {
  const int T = 1 << shift;
  const int c = (threadIdx.x & (T - 1)) + blockIdx.y * 64;
  const int rpb = kBT >> shift;
  if (c >= t) return;
  const RowWalk w = row_walk<PERS>((n + rpb - 1) / rpb);
  for (int g = w.g0; g < w.g1; ++g) {
    const int i = g * rpb + (threadIdx.x >> shift);
    if (i >= n) break;
    const int k = i < m ? i : m;
    double s = unit ? X[(size_t)i * t + c] : 0.;
    s = row_dot<CH>(nbr + (size_t)i * m, vals + (size_t)i * m, k, nullptr, X, t, c, i, s);
    if (scale) s *= scale[i];
    Y[(size_t)i * t + c] = s;
  }
}

// Y = unit*pre.*X + V^T (pre.*X) + W.*H over the transposed lists; values from tval (list
// order, contiguous) when given, else gathered through tslot (CH = 0 form only).
template <int CH, bool PERS>
__global__ void __launch_bounds__(kBT) bt_apply_kernel(int n, const int* __restrict__ tptr,
                                                       const int* __restrict__ trow, const int* __restrict__ tslot,
                                                       const double* __restrict__ vals,
                                                       const double* __restrict__ tval, int unit,
                                                       const double* __restrict__ X, int t, int shift,
                                                       const double* __restrict__ pre, const double* __restrict__ W,
                                                       const double* __restrict__ H, double* __restrict__ Y) {
  const int T = 1 << shift;
  const int c = (threadIdx.x & (T - 1)) + blockIdx.y * 64;
  const int rpb = kBT >> shift;
  if (c >= t) return;
  const RowWalk w = row_walk<PERS>((n + rpb - 1) / rpb);
  for (int g = w.g0; g < w.g1; ++g) {
    const int j = g * rpb + (threadIdx.x >> shift);
    if (j >= n) break;
    double s = 0.;
    if (unit) s = pre ? pre[j] * X[(size_t)j * t + c] : X[(size_t)j * t + c];
    const int e0 = tptr[j], e1 = tptr[j + 1];
    if (tval) {
      s = row_dot<CH>(trow + e0, tval + e0, e1 - e0, pre, X, t, c, j, s);
    } else {
      for (int e = e0; e < e1; ++e) {
        const int i = trow[e];
        const double v = vals[tslot[e]];
        s = fma(pre ? v * pre[i] : v, X[(size_t)i * t + c], s);
      }
    }
    if (W) s = fma(W[j], H[(size_t)j * t + c], s);
    Y[(size_t)j * t + c] = s;
  }
}

// ---- wave-per-row forms (t >= 2): the TA issue rate, not bandwidth, bounds the per-entry
// forms above (every entry costs a structure load AND a gather, 64 lanes each). Here lane r
// loads entry r of the row's structure (ONE coalesced load for up to 64 entries), and the
// gathers take each entry's index and value from that lane with v_readlane (scalar
// registers), so a row costs one vector-memory instruction per entry. Same summation order
// as the other forms (unit term, entries ascending).
constexpr int kWaveChunk = 16;   // gathers in flight per lane (A/B: GPBOOST_AMD_SPMV ch = -2 -> 32)

// Y = diag(scale) (unit*X + V X); 4 waves per block, one row per wave, lane = column.
template <int CH>
__global__ void __launch_bounds__(kBT) b_apply_wave_kernel(int n, int m, const int* __restrict__ nbr,
                                                           const double* __restrict__ vals, int unit,
                                                           const double* __restrict__ X, int t,
                                                           const double* __restrict__ scale, double* __restrict__ Y) {
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int i = xcd_block(blockIdx.x, gridDim.x) * (kBT / 64) + wave;
  if (i >= n) return;
  const int c = lane + blockIdx.y * 64;
  const int cc = c < t ? c : t - 1;   // lanes beyond t gather a valid column, result unused
  const int k = i < m ? i : m;
  const int my_id = lane < k ? nbr[(size_t)i * m + lane] : i;
  const double my_w = lane < k ? vals[(size_t)i * m + lane] : 0.;
  double s = unit ? X[(size_t)i * t + cc] : 0.;
  s = wave_dot<CH>(my_id, my_w, k, X, t, cc, i, s);
  if (scale) s *= scale[i];
  if (c < t) Y[(size_t)i * t + c] = s;
}

// Y = unit*pre.*X + V^T (pre.*X) + W.*H over the transposed lists (values in list order).
template <int CH>
__global__ void __launch_bounds__(kBT) bt_apply_wave_kernel(int n, const int* __restrict__ tptr,
                                                            const int* __restrict__ trow,
                                                            const double* __restrict__ tval, int unit,
                                                            const double* __restrict__ X, int t,
                                                            const double* __restrict__ pre,
                                                            const double* __restrict__ W,
                                                            const double* __restrict__ H, double* __restrict__ Y) {
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int j = xcd_block(blockIdx.x, gridDim.x) * (kBT / 64) + wave;
  if (j >= n) return;
  const int c = lane + blockIdx.y * 64;
  const int cc = c < t ? c : t - 1;
  double s = 0.;
  if (unit) s = pre ? pre[j] * X[(size_t)j * t + cc] : X[(size_t)j * t + cc];
  const int e0 = tptr[j], e1 = tptr[j + 1];
  for (int b0 = e0; b0 < e1; b0 += 64) {
    const int e = b0 + lane;
    const bool ok = e < e1;
    const int my_id = ok ? trow[e] : j;
    double my_w = ok ? tval[e] : 0.;
    if (pre && ok) my_w *= pre[my_id];
    const int cnt = e1 - b0 < 64 ? e1 - b0 : 64;
    s = wave_dot<CH>(my_id, my_w, cnt, X, t, cc, j, s);
  }
  if (W) s = fma(W[j], H[(size_t)j * t + cc], s);
  if (c < t) Y[(size_t)j * t + c] = s;
}

// t = 1: G lanes per row, entry r on lane r mod G (structure loads coalesced, one gather
// instruction per row instead of a serial chain per lane); fixed shuffle tree -> deterministic.
template <int G>
__global__ void __launch_bounds__(kBT) b_apply1_kernel(int n, int m, const int* __restrict__ nbr,
                                                       const double* __restrict__ vals, int unit,
                                                       const double* __restrict__ X,
                                                       const double* __restrict__ scale, double* __restrict__ Y) {
  const int lane = threadIdx.x & (G - 1);
  constexpr int rpb = kBT / G;
  {
    const int i = xcd_block(blockIdx.x, gridDim.x) * rpb + threadIdx.x / G;
    if (i >= n) return;   // whole lane groups exit together
    const int k = i < m ? i : m;
    const size_t o = (size_t)i * m;
    double acc = 0.;
    for (int r = lane; r < k; r += G) acc = fma(vals[o + r], X[nbr[o + r]], acc);
#pragma unroll
    for (int off = G / 2; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 64);
    if (lane == 0) {
      double s = unit ? X[i] + acc : acc;
      if (scale) s *= scale[i];
      Y[i] = s;
    }
  }
}

template <int G>
__global__ void __launch_bounds__(kBT) bt_apply1_kernel(int n, const int* __restrict__ tptr,
                                                        const int* __restrict__ trow,
                                                        const double* __restrict__ tval, int unit,
                                                        const double* __restrict__ X,
                                                        const double* __restrict__ pre,
                                                        const double* __restrict__ W,
                                                        const double* __restrict__ H, double* __restrict__ Y) {
  const int lane = threadIdx.x & (G - 1);
  constexpr int rpb = kBT / G;
  {
    const int j = xcd_block(blockIdx.x, gridDim.x) * rpb + threadIdx.x / G;
    if (j >= n) return;   // whole lane groups exit together
    const int e1 = tptr[j + 1];
    double acc = 0.;
    for (int e = tptr[j] + lane; e < e1; e += G) {
      const int i = trow[e];
      acc = fma(pre ? tval[e] * pre[i] : tval[e], X[i], acc);
    }
#pragma unroll
    for (int off = G / 2; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 64);
    if (lane == 0) {
      double s = unit ? (pre ? pre[j] * X[j] : X[j]) : 0.;
      s += acc;
      if (W) s = fma(W[j], H[j], s);
      Y[j] = s;
    }
  }
}

// t = 1, several rows per lane group in flight: a group of G lanes owns R rows (rows
// base + q * (kBT / G)) and issues every structure load of all R rows, then every gather, then
// reduces. The one-row forms above are latency-bound (structure load -> gather -> store per
// row, ~50 blocks per CU in turn); here each wave keeps R times as many loads in flight.
// Lane l holds entries l and l + G of a row (m <= 2G); the B^T form loops over the rest.
constexpr int k1G = 16, k1R = 4;

template <int G, int R>
__global__ void __launch_bounds__(kBT) b_apply1m_kernel(int n, int m, const int* __restrict__ nbr,
                                                        const double* __restrict__ vals, int unit,
                                                        const double* __restrict__ X,
                                                        const double* __restrict__ scale, double* __restrict__ Y) {
  constexpr int NG = kBT / G;
  const int lane = threadIdx.x & (G - 1);
  const int base = xcd_block(blockIdx.x, gridDim.x) * (NG * R) + (int)threadIdx.x / G;
  int id[R][2];
  double w[R][2], g[R][2], xs[R];
#pragma unroll
  for (int q = 0; q < R; ++q) {
    const int i = base + q * NG;
    const int k = i < n ? min(i, m) : 0;
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int r = lane + e * G;
      const bool ok = r < k;
      const size_t o = (size_t)i * m + r;
      id[q][e] = ok ? nbr[o] : 0;
      w[q][e] = ok ? vals[o] : 0.;
    }
    xs[q] = (unit && lane == 0 && i < n) ? X[i] : 0.;
  }
#pragma unroll
  for (int q = 0; q < R; ++q)
#pragma unroll
    for (int e = 0; e < 2; ++e) g[q][e] = X[id[q][e]];
#pragma unroll
  for (int q = 0; q < R; ++q) {
    double acc = fma(w[q][1], g[q][1], w[q][0] * g[q][0]);
    acc = lane_group_sum<G>(acc);
    const int i = base + q * NG;
    if (lane == 0 && i < n) {
      double s = xs[q] + acc;
      if (scale) s *= scale[i];
      Y[i] = s;
    }
  }
}

// Rows longer than kLongRow: one wave each, lanes stride the list, 4 chunks of loads in
// flight (a 16-lane group walking a 300-entry list was the launch's critical path).
__device__ __forceinline__ void bt_long_row(int j, const int* __restrict__ tptr, const int* __restrict__ trow,
                                            const double* __restrict__ tval, int unit, const double* __restrict__ X,
                                            const double* __restrict__ pre, const double* __restrict__ W,
                                            const double* __restrict__ H, double* __restrict__ Y) {
  const int lane = threadIdx.x & 63;
  const int e0 = tptr[j], e1 = tptr[j + 1];
  double acc = 0.;
  for (int b = e0 + lane; b < e1; b += 4 * 64) {
    int id[4];
    double w[4], g[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int e = b + k * 64;
      const bool ok = e < e1;
      id[k] = ok ? trow[e] : 0;
      w[k] = ok ? tval[e] : 0.;
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      g[k] = X[id[k]];
      if (pre) w[k] *= pre[id[k]];
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) acc = fma(w[k], g[k], acc);
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 64);
  if (lane == 0) {
    double s = unit ? (pre ? pre[j] * X[j] : X[j]) : 0.;
    s += acc;
    if (W) s = fma(W[j], H[j], s);
    Y[j] = s;
  }
}

template <int G, int R, int E>
__global__ void __launch_bounds__(kBT) bt_apply1m_kernel(int n, const int* __restrict__ tptr,
                                                         const int* __restrict__ trow,
                                                         const double* __restrict__ tval, int unit,
                                                         const double* __restrict__ X,
                                                         const double* __restrict__ pre,
                                                         const double* __restrict__ W,
                                                         const double* __restrict__ H, double* __restrict__ Y,
                                                         int nmain, const int* __restrict__ longr, int nlong) {
  if ((int)blockIdx.x >= nmain) {   // trailing blocks: the long rows, one wave each
    const int w = ((int)blockIdx.x - nmain) * (kBT / 64) + (int)(threadIdx.x >> 6);
    if (w < nlong) bt_long_row(longr[w], tptr, trow, tval, unit, X, pre, W, H, Y);
    return;
  }
  constexpr int NG = kBT / G;
  const int lane = threadIdx.x & (G - 1);
  const int base = xcd_block(blockIdx.x, nmain) * (NG * R) + (int)threadIdx.x / G;
  int e0[R], e1[R], id[R][E];
  double w[R][E], g[R][E], xs[R], wv[R], hv[R];
#pragma unroll
  for (int q = 0; q < R; ++q) {
    const int j = base + q * NG;
    e0[q] = j < n ? tptr[j] : 0;
    e1[q] = j < n ? tptr[j + 1] : 0;
    if (e1[q] - e0[q] > kLongRow) e1[q] = e0[q];   // a long-row wave writes this row
    const bool own = lane == 0 && j < n;
    xs[q] = (unit && own) ? (pre ? pre[j] * X[j] : X[j]) : 0.;
    wv[q] = (W && own) ? W[j] : 0.;
    hv[q] = (W && own) ? H[j] : 0.;
  }
#pragma unroll
  for (int q = 0; q < R; ++q)
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const int ee = e0[q] + lane + e * G;
      const bool ok = ee < e1[q];
      id[q][e] = ok ? trow[ee] : 0;
      w[q][e] = ok ? tval[ee] : 0.;
    }
#pragma unroll
  for (int q = 0; q < R; ++q)
#pragma unroll
    for (int e = 0; e < E; ++e) {
      g[q][e] = X[id[q][e]];
      if (pre) w[q][e] *= pre[id[q][e]];
    }
#pragma unroll
  for (int q = 0; q < R; ++q) {
    double acc = w[q][0] * g[q][0];
#pragma unroll
    for (int e = 1; e < E; ++e) acc = fma(w[q][e], g[q][e], acc);
    for (int ee = e0[q] + lane + E * G; ee < e1[q]; ee += G) {   // rows with > E G entries
      const int i = trow[ee];
      acc = fma(pre ? tval[ee] * pre[i] : tval[ee], X[i], acc);
    }
    acc = lane_group_sum<G>(acc);
    const int j = base + q * NG;
    if (lane == 0 && j < n && tptr[j + 1] - tptr[j] <= kLongRow) {
      double s = xs[q] + acc;
      if (W) s = fma(wv[q], hv[q], s);
      Y[j] = s;
    }
  }
}

// t = 1 default form of B^T (SparseB::seg_*): one wave per run of consecutive storage rows
// (<= kSegEntries entries, or one longer row). The run's entries are consumed 64 at a time, lane =
// entry, kSegU chunks of coalesced (row, value, run-row) loads and gathers in flight; per chunk a
// segmented inclusive scan over the wave (rows are contiguous in the list, so "same run-row as the
// lane off below" is the segment test) leaves each row's chunk sum in its last lane, which adds it
// to the row's LDS accumulator (one lane per row per chunk: no conflicts, chunk order fixed ->
// bitwise repeatable). Every wave reads the same number of bytes whatever its rows' lengths,
// where the lane-group form (bt_apply1m) idles lanes on short lists and serialises long ones.
constexpr int kSegWaves = 4;
#ifndef GPB_SEG_U
#define GPB_SEG_U 4
#endif
constexpr int kSegU = GPB_SEG_U;   // 64-entry chunks per iteration (A/B builds override)
__device__ __forceinline__ double shfl_up_f64(double v, int off) {
  const int lo = __shfl_up(__double2loint(v), off, 64);
  const int hi = __shfl_up(__double2hiint(v), off, 64);
  return __hiloint2double(hi, lo);
}
// Segmented inclusive scan step: p += p[src lane] where the source lane has the same key.
// DPP form (no LDS crossbar): row_shr 1/2/4/8 inside 16-lane rows, then row_bcast 15 (rows 1, 3)
// and 31 (rows 2, 3) across rows; lanes without a source see key -1 / value 0.
template <int CTRL, int ROWMASK>
__device__ __forceinline__ void seg_step_dpp(double& p, int k) {
  const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(p), CTRL, ROWMASK, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(p), CTRL, ROWMASK, 0xF, false);
  const int kq = __builtin_amdgcn_update_dpp(-1, k, CTRL, ROWMASK, 0xF, false);
  if (kq == k) p += __hiloint2double(hi, lo);
}
template <bool DPP>
__device__ __forceinline__ double seg_scan(double p, int k, int lane) {
  if constexpr (DPP) {
    seg_step_dpp<0x111, 0xF>(p, k);   // row_shr:1
    seg_step_dpp<0x112, 0xF>(p, k);   // row_shr:2
    seg_step_dpp<0x114, 0xF>(p, k);   // row_shr:4
    seg_step_dpp<0x118, 0xF>(p, k);   // row_shr:8
    seg_step_dpp<0x142, 0xA>(p, k);   // row_bcast:15 -> rows 1, 3
    seg_step_dpp<0x143, 0xC>(p, k);   // row_bcast:31 -> rows 2, 3
  } else {
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const double q = shfl_up_f64(p, off);
      const int kq = __shfl_up(k, off, 64);
      if (lane >= off && kq == k) p += q;
    }
  }
  return p;
}

template <bool DPP>
__global__ void __launch_bounds__(64 * kSegWaves) bt_apply1s_kernel(
    int nseg, const int* __restrict__ seg_rb, const uint32_t* __restrict__ seg_pk, const int* __restrict__ tptr,
    const double* __restrict__ tval, int unit, const double* __restrict__ X, const double* __restrict__ pre,
    const double* __restrict__ W, const double* __restrict__ H, double* __restrict__ Y) {
  __shared__ double acc_s[kSegWaves][kSegRows + 1];
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  const int w = xcd_block(blockIdx.x, gridDim.x) * kSegWaves + wv;
  if (w >= nseg) return;   // whole waves only; no block-level synchronisation below
  const int rb = seg_rb[w], re = seg_rb[w + 1];
  const int nr = re - rb;
  double* acc = acc_s[wv];
  for (int q = lane; q < nr; q += 64) acc[q] = 0.;
  const int e0 = tptr[rb], e1 = tptr[re];
  for (int c = e0; c < e1; c += 64 * kSegU) {
    uint32_t pk[kSegU];
    double v[kSegU];
#pragma unroll
    for (int u = 0; u < kSegU; ++u) {
      const int e = c + u * 64 + lane;
      const bool ok = e < e1;
      pk[u] = ok ? seg_pk[e] : ((uint32_t)kSegRows << 24);   // padding: key 127, never a row end
      v[u] = ok ? tval[e] : 0.;
    }
#pragma unroll
    for (int u = 0; u < kSegU; ++u) {
      const int id = (int)(pk[u] & 0xFFFFFFu);
      double g = X[id];
      if (pre) g *= pre[id];
      v[u] *= g;
    }
#pragma unroll
    for (int u = 0; u < kSegU; ++u) {
      const int k = (int)((pk[u] >> 24) & 0x7Fu);
      const double p = seg_scan<DPP>(v[u], k, lane);
      // a row's sum leaves the chunk at its last entry, or at lane 63 when it continues
      if (k != kSegRows && ((pk[u] >> 31) != 0u || lane == 63)) acc[k] += p;
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // this wave's accumulator writes before its reads
  for (int q = lane; q < nr; q += 64) {
    const int j = rb + q;
    double s = unit ? (pre ? pre[j] * X[j] : X[j]) : 0.;
    s += acc[q];
    if (W) s = fma(W[j], H[j], s);
    Y[j] = s;
  }
}

// Two entries per lane (entries c + 2 lane, c + 2 lane + 1 of a 128-entry chunk): one segmented
// scan per 128 entries instead of per 64. A lane's element is the running sum of its LAST entry's row
// (both entries when they share a row); when its first entry closes an earlier row, that row's
// chunk sum is the first entry plus the previous lane's scanned value (wave_shr:1). Runs hold whole
// rows, so the last valid entry of a run carries the row-end flag and padding never needs a flush.
template <bool DPP>
__global__ void __launch_bounds__(64 * kSegWaves) bt_apply1s2_kernel(
    int nseg, const int* __restrict__ seg_rb, const uint32_t* __restrict__ seg_pk, const int* __restrict__ tptr,
    const double* __restrict__ tval, int unit, const double* __restrict__ X, const double* __restrict__ pre,
    const double* __restrict__ W, const double* __restrict__ H, double* __restrict__ Y) {
  __shared__ double acc_s[kSegWaves][kSegRows + 1];
  constexpr uint32_t kPad = (uint32_t)kSegRows << 24;
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  const int w = xcd_block(blockIdx.x, gridDim.x) * kSegWaves + wv;
  if (w >= nseg) return;   // whole waves only; no block-level synchronisation below
  const int rb = seg_rb[w], re = seg_rb[w + 1];
  const int nr = re - rb;
  double* acc = acc_s[wv];
  for (int q = lane; q < nr; q += 64) acc[q] = 0.;
  const int e0 = tptr[rb], e1 = tptr[re];
  for (int c = e0; c < e1; c += 128 * kSegU) {
    uint32_t pa[kSegU], pb[kSegU];
    double va[kSegU], vb[kSegU];
#pragma unroll
    for (int u = 0; u < kSegU; ++u) {
      const int e = c + u * 128 + 2 * lane;
      pa[u] = e < e1 ? seg_pk[e] : kPad;
      pb[u] = e + 1 < e1 ? seg_pk[e + 1] : kPad;
      va[u] = e < e1 ? tval[e] : 0.;
      vb[u] = e + 1 < e1 ? tval[e + 1] : 0.;
    }
#pragma unroll
    for (int u = 0; u < kSegU; ++u) {
      const int ia = (int)(pa[u] & 0xFFFFFFu), ib = (int)(pb[u] & 0xFFFFFFu);
      double ga = X[ia], gb = X[ib];
      if (pre) { ga *= pre[ia]; gb *= pre[ib]; }
      va[u] *= ga;
      vb[u] *= gb;
    }
#pragma unroll
    for (int u = 0; u < kSegU; ++u) {
      const int ka = (int)((pa[u] >> 24) & 0x7Fu), kb = (int)((pb[u] >> 24) & 0x7Fu);
      const bool same = ka == kb;
      const double p = seg_scan<DPP>(same ? va[u] + vb[u] : vb[u], kb, lane);
      // previous lane's scanned value and key (lane 0: none)
      const int plo = __builtin_amdgcn_update_dpp(0, __double2loint(p), 0x138, 0xF, 0xF, false);
      const int phi = __builtin_amdgcn_update_dpp(0, __double2hiint(p), 0x138, 0xF, 0xF, false);
      const int pk = __builtin_amdgcn_update_dpp(-1, kb, 0x138, 0xF, 0xF, false);
      if (!same && ka != kSegRows) acc[ka] += va[u] + (pk == ka ? __hiloint2double(phi, plo) : 0.);
      if (kb != kSegRows && ((pb[u] >> 31) != 0u || lane == 63)) acc[kb] += p;
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // this wave's accumulator writes before its reads
  for (int q = lane; q < nr; q += 64) {
    const int j = rb + q;
    double s = unit ? (pre ? pre[j] * X[j] : X[j]) : 0.;
    s += acc[q];
    if (W) s = fma(W[j], H[j], s);
    Y[j] = s;
  }
}

// E entries per lane (entries c + E lane + q of a 64 E-entry chunk), U chunks in flight, run bounds
// and entry range from one 16-byte load: a lane walks its E entries (sorted by row), closes the rows
// that end inside it (the first one takes the previous lane's scanned value as carry), and the
// running sum of its last row enters ONE segmented scan per 64 E entries.
template <int E, int U>
__global__ void __launch_bounds__(64 * kSegWaves) bt_apply1sE_kernel(
    int nseg, const int4* __restrict__ seg_info, const uint32_t* __restrict__ seg_pk, const double* __restrict__ tval,
    int unit, const double* __restrict__ X, const double* __restrict__ pre, const double* __restrict__ W,
    const double* __restrict__ H, double* __restrict__ Y) {
  __shared__ double acc_s[kSegWaves][kSegRows + 1];
  constexpr uint32_t kPad = (uint32_t)kSegRows << 24;
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  const int w = xcd_block(blockIdx.x, gridDim.x) * kSegWaves + wv;
  if (w >= nseg) return;   // whole waves only; no block-level synchronisation below
  const int4 inf = seg_info[w];   // rows [x, y), entries [z, w)
  const int rb = inf.x, nr = inf.y - inf.x, e1 = inf.w;
  double* acc = acc_s[wv];
  for (int q = lane; q < nr; q += 64) acc[q] = 0.;
  for (int c = inf.z; c < e1; c += 64 * E * U) {
    uint32_t pk[U][E];
    double v[U][E];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int q = 0; q < E; ++q) {
        const int e = c + u * 64 * E + E * lane + q;
        pk[u][q] = e < e1 ? seg_pk[e] : kPad;
        v[u][q] = e < e1 ? tval[e] : 0.;
      }
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int q = 0; q < E; ++q) {
        const int id = (int)(pk[u][q] & 0xFFFFFFu);
        double g = X[id];
        if (pre) g *= pre[id];
        v[u][q] *= g;
      }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int kf = (int)((pk[u][0] >> 24) & 0x7Fu);
      int kc = kf;
      double sc = v[u][0], sf = 0.;
      bool open = true;   // the lane's first row has not closed inside the lane
#pragma unroll
      for (int q = 1; q < E; ++q) {
        const int kq = (int)((pk[u][q] >> 24) & 0x7Fu);
        if (kq == kc) {
          sc += v[u][q];
        } else {
          if (open) { sf = sc; open = false; }
          else if (kc != kSegRows) acc[kc] += sc;   // a row wholly inside this lane
          kc = kq;
          sc = v[u][q];
        }
      }
      const double p = seg_scan<true>(sc, kc, lane);
      const int plo = __builtin_amdgcn_update_dpp(0, __double2loint(p), 0x138, 0xF, 0xF, false);   // wave_shr:1
      const int phi = __builtin_amdgcn_update_dpp(0, __double2hiint(p), 0x138, 0xF, 0xF, false);
      const int pkey = __builtin_amdgcn_update_dpp(-1, kc, 0x138, 0xF, 0xF, false);
      if (!open && kf != kSegRows) acc[kf] += sf + (pkey == kf ? __hiloint2double(phi, plo) : 0.);
      if (kc != kSegRows && ((pk[u][E - 1] >> 31) != 0u || lane == 63)) acc[kc] += p;
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // this wave's accumulator writes before its reads
  for (int q = lane; q < nr; q += 64) {
    const int j = rb + q;
    double s = unit ? (pre ? pre[j] * X[j] : X[j]) : 0.;
    s += acc[q];
    if (W) s = fma(W[j], H[j], s);
    Y[j] = s;
  }
}

// Paired layout (SparseB::seg_pk2 / seg_val2: runs start at even positions): the E = 2 form with a
// lane's two entries as one 8-byte structure load and one 16-byte value load.
template <int U>
__global__ void __launch_bounds__(64 * kSegWaves) bt_apply1p_kernel(
    int nseg, const int4* __restrict__ seg_info, const uint2* __restrict__ pk2, const double2* __restrict__ val2,
    int unit, const double* __restrict__ X, const double* __restrict__ pre, const double* __restrict__ W,
    const double* __restrict__ H, double* __restrict__ Y) {
  __shared__ double acc_s[kSegWaves][kSegRows + 1];
  constexpr uint32_t kPad = (uint32_t)kSegRows << 24;
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  const int w = xcd_block(blockIdx.x, gridDim.x) * kSegWaves + wv;
  if (w >= nseg) return;   // whole waves only; no block-level synchronisation below
  const int4 inf = seg_info[w];   // rows [x, y), entries [z, w) (z even)
  const int rb = inf.x, nr = inf.y - inf.x, e1 = inf.w;
  double* acc = acc_s[wv];
  for (int q = lane; q < nr; q += 64) acc[q] = 0.;
  for (int c = inf.z; c < e1; c += 128 * U) {
    uint2 pk[U];
    double2 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int e = c + u * 128 + 2 * lane;   // even; e + 1 is a real or pad slot of this run when e < e1
      if (e < e1) { pk[u] = pk2[e >> 1]; v[u] = val2[e >> 1]; }
      else { pk[u] = make_uint2(kPad, kPad); v[u] = make_double2(0., 0.); }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int ia = (int)(pk[u].x & 0xFFFFFFu), ib = (int)(pk[u].y & 0xFFFFFFu);
      double ga = X[ia], gb = X[ib];
      if (pre) { ga *= pre[ia]; gb *= pre[ib]; }
      v[u].x *= ga;
      v[u].y *= gb;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int ka = (int)((pk[u].x >> 24) & 0x7Fu), kb = (int)((pk[u].y >> 24) & 0x7Fu);
      const bool same = ka == kb;
      const double p = seg_scan<true>(same ? v[u].x + v[u].y : v[u].y, kb, lane);
      const int plo = __builtin_amdgcn_update_dpp(0, __double2loint(p), 0x138, 0xF, 0xF, false);   // wave_shr:1
      const int phi = __builtin_amdgcn_update_dpp(0, __double2hiint(p), 0x138, 0xF, 0xF, false);
      const int pkey = __builtin_amdgcn_update_dpp(-1, kb, 0x138, 0xF, 0xF, false);
      if (!same && ka != kSegRows) acc[ka] += v[u].x + (pkey == ka ? __hiloint2double(phi, plo) : 0.);
      if (kb != kSegRows && ((pk[u].y >> 31) != 0u || lane == 63)) acc[kb] += p;
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // this wave's accumulator writes before its reads
  for (int q = lane; q < nr; q += 64) {
    const int j = rb + q;
    double s = unit ? (pre ? pre[j] * X[j] : X[j]) : 0.;
    s += acc[q];
    if (W) s = fma(W[j], H[j], s);
    Y[j] = s;
  }
}

// t = 1 default form of B (SparseB::ell_*): one row per lane, entries in a fixed ascending order,
// kU1 loads in flight per lane. (The same form for B^T — sliced ELL, rows sorted by length in
// windows — measured 37-48 us against the lane groups' 20 us: rows-as-lanes only pays where every
// row has the same length.)
#ifndef GPB_U1
#define GPB_U1 10
#endif
constexpr int kU1 = GPB_U1;   // loads in flight per lane (A/B builds override)
__global__ void __launch_bounds__(kBT) b_apply1e_kernel(int n, int m, const int* __restrict__ idx,
                                                        const double* __restrict__ val, int unit,
                                                        const double* __restrict__ X,
                                                        const double* __restrict__ scale, double* __restrict__ Y) {
  const int i = xcd_block(blockIdx.x, gridDim.x) * kBT + (int)threadIdx.x;
  if (i >= n) return;
  const int k = i < m ? i : m;
  double acc = 0.;
  for (int r0 = 0; r0 < k; r0 += kU1) {
    int id[kU1];
    double w[kU1], g[kU1];
#pragma unroll
    for (int u = 0; u < kU1; ++u) {
      const int r = r0 + u;
      const bool ok = r < k;
      id[u] = ok ? idx[(size_t)r * n + i] : i;
      w[u] = ok ? val[(size_t)r * n + i] : 0.;
    }
#pragma unroll
    for (int u = 0; u < kU1; ++u) g[u] = X[id[u]];
#pragma unroll
    for (int u = 0; u < kU1; ++u) acc = fma(w[u], g[u], acc);
  }
  double s = unit ? X[i] + acc : acc;
  if (scale) s *= scale[i];
  Y[i] = s;
}

// LDS-tiled operator (TileOp; opt-in A/B form, GPBOOST_AMD_SPMV_TILED=1): 8 waves; the tile's union rows are staged into LDS (lane = column,
// row stride tc = this column block's width), then wave w takes the tile's rows w, w + 8, ...:
// a 64-entry chunk of the row's list is ONE coalesced load of (lidx, value) per lane, each entry
// read by v_readlane, its operand row from LDS. Fixed entry order (bitwise repeatable). Blocks
// beyond ntile: the fallback rows, one wave each, global gathers. Measured at n = 100k, t = 51
// (unions of <= 256 / 176 / 128 rows): b 0.132 / 0.110 / 0.119 ms, b^T 0.188 / 0.160 / 0.172 ms
// against the global-gather wave kernels' 0.104 / 0.134 ms: staging a tile's ~250 union rows
// costs ~5 us and the per-entry v_readlane + LDS read chain ~100 cycles at 8 waves per CU, which
// the L2 hits of the wave kernels (87-90 %) beat.
constexpr int kTileThreads = 512;
template <bool TRANS>
__global__ void __launch_bounds__(kTileThreads) apply_tile_kernel(int n, int m, const int* __restrict__ nbr,
                                                                  const int* __restrict__ tptr,
                                                                  const int* __restrict__ trow, TileOp op,
                                                                  const double* __restrict__ vals,
                                                                  const double* __restrict__ X, int t,
                                                                  const double* __restrict__ scale,
                                                                  const double* __restrict__ W,
                                                                  const double* __restrict__ H,
                                                                  double* __restrict__ Y) {
  extern __shared__ double xs[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  constexpr int NW = kTileThreads / 64;
  const int cb = blockIdx.y * 64;
  const int c = lane + cb;
  const int tc = t - cb < 64 ? t - cb : 64;
  const int cc = c < t ? c : t - 1;
  const int tile = blockIdx.x;
  if (tile >= op.ntile) {   // fallback rows: one wave each, dependencies gathered from global memory
    const int w = (tile - op.ntile) * NW + wave;
    if (w >= op.nfb) return;
    const int j = op.fb[w];
    double sacc = X[(size_t)j * t + cc];
    const int e0 = TRANS ? tptr[j] : j * m, e1 = TRANS ? tptr[j + 1] : j * m + (j < m ? j : m);
    for (int b0 = e0; b0 < e1; b0 += 64) {
      const int e = b0 + lane;
      const bool ok = e < e1;
      const int my_id = ok ? (TRANS ? trow[e] : nbr[e]) : j;
      const double my_w = ok ? vals[e] : 0.;
      const int cnt = e1 - b0 < 64 ? e1 - b0 : 64;
      sacc = wave_dot<16>(my_id, my_w, cnt, X, t, cc, j, sacc);
    }
    if (TRANS) { if (W) sacc = fma(W[j], H[(size_t)j * t + cc], sacc); }
    else if (scale) sacc *= scale[j];
    if (c < t) Y[(size_t)j * t + c] = sacc;
    return;
  }
  const int u0 = op.uoff[tile], nu = op.uoff[tile + 1] - u0;
  // ---- stage the union rows (lane = column), kStageU rows in flight per wave
  constexpr int kStageU = 16;
  for (int k0 = wave; k0 < nu; k0 += kStageU * NW) {
    int r[kStageU];
    double v[kStageU];
#pragma unroll
    for (int q = 0; q < kStageU; ++q) {
      const int k = k0 + q * NW;
      r[q] = op.urow[u0 + (k < nu ? k : 0)];
    }
#pragma unroll
    for (int q = 0; q < kStageU; ++q) v[q] = X[(size_t)r[q] * t + cc];
#pragma unroll
    for (int q = 0; q < kStageU; ++q) {
      const int k = k0 + q * NW;
      if (k < nu && lane < tc) xs[k * tc + lane] = v[q];
    }
  }
  __syncthreads();
  const int lc = lane < tc ? lane : tc - 1;
  // this wave's rows i_k = r0 + wave + k NW (k < kTileRows / NW): lane k holds row k's entry range
  // (empty for a fallback row), so the loop below needs no global load before its first chunk
  const int rb = op.r0[tile], re = op.r0[tile + 1];
  int my_e0 = 0, my_e1 = 0;   // my_e1 = -1: a fallback row (written by the fallback waves)
  {
    const int i = rb + wave + lane * NW;
    if (lane < kTileRows / NW && i < re) {
      if (op.isfb[i]) {
        my_e1 = -1;
      } else {
        my_e0 = TRANS ? tptr[i] : i * m;
        my_e1 = TRANS ? tptr[i + 1] : i * m + (i < m ? i : m);
      }
    }
  }
  auto load_chunk = [&](int e0, int e1, int& l, double& w) {
    const int e = e0 + lane;
    const bool ok = e < e1;
    l = ok ? (int)op.lidx[e] : 0;
    w = ok ? vals[e] : 0.;
  };
  // every structure chunk and own operand of the wave's rows issued up front, consumed in issue
  // order (in-order vmcnt waits: row k waits only for its own loads)
  constexpr int RW = kTileRows / NW;
  int L[RW];
  double Wt[RW], Xo[RW], Ho[RW];
#pragma unroll
  for (int k = 0; k < RW; ++k) {
    const int i = rb + wave + k * NW;
    const int ii = i < re ? i : rb;
    load_chunk(__builtin_amdgcn_readlane(my_e0, k), __builtin_amdgcn_readlane(my_e1, k), L[k], Wt[k]);
    Xo[k] = X[(size_t)ii * t + cc];
    Ho[k] = (TRANS && W) ? H[(size_t)ii * t + cc] : 0.;
  }
#pragma unroll
  for (int k = 0; k < RW; ++k) {
    const int i = rb + wave + k * NW;
    if (i >= re) break;
    const int e0 = __builtin_amdgcn_readlane(my_e0, k), e1 = __builtin_amdgcn_readlane(my_e1, k);
    if (e1 < 0) continue;   // wave-uniform
    double acc = Xo[k];
    for (int b0 = e0; b0 < e1; b0 += 64) {
      int cl = L[k];
      double cw = Wt[k];
      if (b0 != e0) load_chunk(b0, e1, cl, cw);   // lists longer than 64 (B^T): further chunks
      const int cnt = e1 - b0 < 64 ? e1 - b0 : 64;
      // lanes >= cnt hold (0, 0.): reading them is harmless, so the batches need no bounds checks
      for (int q0 = 0; q0 < cnt; q0 += 16) {
        double g[16], w[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) {
          const int l = __builtin_amdgcn_readlane(cl, q0 + u);
          w[u] = readlane_f64(cw, q0 + u);
          g[u] = xs[l * tc + lc];
        }
#pragma unroll
        for (int u = 0; u < 16; ++u) acc = fma(w[u], g[u], acc);
      }
    }
    if (TRANS) { if (W) acc = fma(W[i], Ho[k], acc); }
    else if (scale) acc *= scale[i];
    if (c < t) Y[(size_t)i * t + c] = acc;
  }
}

__global__ void __launch_bounds__(kBT) gather_kernel(int count, const int* __restrict__ idx,
                                                     const double* __restrict__ src, double* __restrict__ dst) {
  for (int e = blockIdx.x * kBT + threadIdx.x; e < count; e += gridDim.x * kBT) {
    const int k = idx[e];
    dst[e] = k >= 0 ? src[k] : (k == -2 ? -1. : 0.);   // -1: zero padding; -2: the constant -1
  }
}

// ------------------------------------------------------------------ column reductions
// Block-level fixed-order tree over the row slots of one block; writes partials[blk][q*t+c].
template <int NP>
__device__ __forceinline__ void block_col_reduce(double (&acc)[NP], int shift, int c, int t, double* partials) {
  __shared__ double red[NP][kBT];
  const int rpb = kBT >> shift;
  const int slot = threadIdx.x >> shift;
#pragma unroll
  for (int q = 0; q < NP; ++q) red[q][threadIdx.x] = acc[q];
  __syncthreads();
  for (int off = rpb >> 1; off > 0; off >>= 1) {
    if (slot < off) {
#pragma unroll
      for (int q = 0; q < NP; ++q) red[q][threadIdx.x] += red[q][threadIdx.x + (off << shift)];
    }
    __syncthreads();
  }
  if (slot == 0 && c < t) {
#pragma unroll
    for (int q = 0; q < NP; ++q) partials[(size_t)blockIdx.x * NP * t + (size_t)q * t + c] = red[q][threadIdx.x];
  }
}

template <int NP>
__global__ void __launch_bounds__(kBT) coldots_kernel(int n, int t, int shift, const double* A0, const double* B0,
                                                      const double* A1, const double* B1, const double* A2,
                                                      const double* B2, double* partials) {
  const int T = 1 << shift;
  const int c = (threadIdx.x & (T - 1)) + blockIdx.y * 64;
  const int rpb = kBT >> shift;
  double acc[NP];
#pragma unroll
  for (int q = 0; q < NP; ++q) acc[q] = 0.;
  if (c < t) {
    for (int i = blockIdx.x * rpb + (threadIdx.x >> shift); i < n; i += gridDim.x * rpb) {
      const size_t o = (size_t)i * t + c;
      acc[0] = fma(A0[o], B0[o], acc[0]);
      if constexpr (NP > 1) acc[1] = fma(A1[o], B1[o], acc[1]);
      if constexpr (NP > 2) acc[2] = fma(A2[o], B2[o], acc[2]);
    }
  }
  block_col_reduce<NP>(acc, shift, c, t, partials);
}

// out[w] = sum over blocks of partials[b*width + w]; one block per output, fixed order.
__global__ void __launch_bounds__(kBT) reduce_blocks_kernel(const double* __restrict__ partials, int nblocks,
                                                            int width, double* __restrict__ out) {
  __shared__ double red[kBT];
  const int w = blockIdx.x;
  double s = 0.;
  for (int b = threadIdx.x; b < nblocks; b += kBT) s += partials[(size_t)b * width + w];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int off = kBT / 2; off > 0; off >>= 1) {
    if ((int)threadIdx.x < off) red[threadIdx.x] += red[threadIdx.x + off];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[w] = red[0];
}

__global__ void __launch_bounds__(kBT) cg_update_kernel(int n, int t, int shift, const double* __restrict__ a,
                                                        const double* __restrict__ H, const double* __restrict__ V,
                                                        double* __restrict__ U, double* __restrict__ R,
                                                        double* partials) {
  const int T = 1 << shift;
  const int c = (threadIdx.x & (T - 1)) + blockIdx.y * 64;
  const int rpb = kBT >> shift;
  double acc[1] = {0.};
  if (c < t) {
    const double ac = a[c];
    for (int i = blockIdx.x * rpb + (threadIdx.x >> shift); i < n; i += gridDim.x * rpb) {
      const size_t o = (size_t)i * t + c;
      U[o] = fma(ac, H[o], U[o]);
      const double r = fma(-ac, V[o], R[o]);
      R[o] = r;
      acc[0] = fma(r, r, acc[0]);
    }
  }
  block_col_reduce<1>(acc, shift, c, t, partials);
}

__global__ void __launch_bounds__(kBT) h_update_kernel(size_t total, int t, const double* __restrict__ b,
                                                       const double* __restrict__ Z, double* __restrict__ H) {
  for (size_t o = (size_t)blockIdx.x * kBT + threadIdx.x; o < total; o += (size_t)gridDim.x * kBT) {
    const int c = (int)(o % t);
    H[o] = fma(b[c], H[o], Z[o]);
  }
}

__global__ void copy_kernel(size_t total, const double* __restrict__ X, double* __restrict__ Y) {
  for (size_t o = (size_t)blockIdx.x * kBT + threadIdx.x; o < total; o += (size_t)gridDim.x * kBT) Y[o] = X[o];
}

__global__ void axpby_kernel(size_t total, double alpha, const double* X, double beta, const double* Y, double* Z) {
  for (size_t o = (size_t)blockIdx.x * kBT + threadIdx.x; o < total; o += (size_t)gridDim.x * kBT)
    Z[o] = alpha * X[o] + beta * Y[o];
}

// Columns whose CG has stopped (act[c] == 0) get a = b = 0: their U and R stay frozen.
__global__ void cg_alpha_kernel(int t, const double* rz, const double* hv, const int* act, double* a, double* hist) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= t) return;
  const double v = (act == nullptr || act[c]) ? rz[c] / hv[c] : 0.;
  a[c] = v;
  if (hist) hist[c] = v;
}

__global__ void cg_beta_kernel(int t, const double* rz_new, double* rz, const int* act, double* b, double* hist) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= t) return;
  if (act != nullptr && !act[c]) {
    b[c] = 0.;
    return;
  }
  const double v = rz_new[c] / rz[c];
  rz[c] = rz_new[c];
  b[c] = v;
  if (hist) hist[c] = v;
}

// Columns >= n_valid are padding of a probe-sharded block: never active.
__global__ void pcg_init_kernel(int t, int n_valid, int n_single, int pmax_single, int pmax_block, double zero_sq,
                                const double* rr0, int* act, int* ctl) {
  if (threadIdx.x != 0) return;
  int any = 0;
  for (int c = 0; c < t; ++c) {
    const int a = (c >= n_valid || (c < n_single && rr0 && rr0[c] < zero_sq)) ? 0 : 1;
    act[c] = a;
    if (c < n_single) any |= a;
  }
  ctl[kCtlActS] = (any && pmax_single > 0) ? 1 : 0;
  ctl[kCtlActB] = (n_single < t && pmax_block > 0) ? 1 : 0;
  ctl[kCtlItsS] = 0;
  ctl[kCtlItsB] = 0;
  ctl[kCtlNan] = 0;
}

// Sum of the block columns' norms of this rank (probe-sharded blocks: all-reduced before the check).
__global__ void pcg_block_sum_kernel(int n_valid, int n_single, const double* rr, double* out) {
  if (threadIdx.x != 0) return;
  double norm = 0.;
  for (int c = n_single; c < n_valid; ++c) norm += sqrt(rr[c]);
  out[0] = norm;
}

// One thread, columns in a fixed order (the block mean is bitwise repeatable). gsum != null: the
// block's norm sum over all ranks (pcg_block_sum_kernel + all-reduce) and its column count nblock.
__global__ void pcg_check_kernel(int j, int t, int n_single, int pmax_single, int pmax_block, double delta,
                                 const double* rr, const double* gsum, int nblock, int* act, int* ctl, int* host_ctl,
                                 int seq) {
  if (threadIdx.x != 0) return;
  if (ctl[kCtlActS]) {
    ctl[kCtlItsS] = j + 1;
    bool all_done = true;
    for (int c = 0; c < n_single; ++c) {
      if (!act[c]) continue;
      const double norm = sqrt(rr[c]);
      if (isnan(norm) || isinf(norm)) ctl[kCtlNan] = 1;
      if (norm < delta || j + 1 >= pmax_single) act[c] = 0;
      else all_done = false;
    }
    if (all_done) ctl[kCtlActS] = 0;
  }
  if (ctl[kCtlActB]) {
    ctl[kCtlItsB] = j + 1;
    double norm = 0.;
    if (gsum) {
      norm = gsum[0] / nblock;
    } else {
      for (int c = n_single; c < t; ++c) norm += sqrt(rr[c]);
      norm /= (t - n_single);
    }
    if (isnan(norm) || isinf(norm)) ctl[kCtlNan] = 1;
    if (norm < delta || j + 1 >= pmax_block) {
      for (int c = n_single; c < t; ++c) act[c] = 0;
      ctl[kCtlActB] = 0;
    }
  }
  if (host_ctl) {
    // the verdict as ONE 64-bit word (pcg_pack) in host-coherent memory: a single untorn store,
    // so no system-scope fence (which would write back the whole L2 and stall the stream)
    const unsigned long long v = pcg_pack(seq, ctl[kCtlActS], ctl[kCtlActB], ctl[kCtlNan], ctl[kCtlItsS], ctl[kCtlItsB]);
    __hip_atomic_store(reinterpret_cast<unsigned long long*>(host_ctl), v, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

__global__ void pack_columns_kernel(size_t rows, int ncols, const double* __restrict__ src, int ld_src, int c_src,
                                   double* __restrict__ dst, int ld_dst, int c_dst) {
  const size_t total = rows * ncols;
  for (size_t o = (size_t)blockIdx.x * kBT + threadIdx.x; o < total; o += (size_t)gridDim.x * kBT) {
    const size_t i = o / ncols, c = o - i * ncols;
    dst[i * ld_dst + c_dst + c] = src[i * ld_src + c_src + c];
  }
}

// ------------------------------------------------------------------ likelihoods: lik_device.h

__global__ void __launch_bounds__(kBT) grad_f_kernel(int n, const double* __restrict__ d1,
                                                     const double* __restrict__ dmll, const double* __restrict__ W,
                                                     const double* __restrict__ vS, double* __restrict__ out) {
  for (int i = blockIdx.x * kBT + threadIdx.x; i < n; i += gridDim.x * kBT) {
    double g = -d1[i];
    if (dmll) g += dmll[i] - W[i] * vS[i];
    out[i] = g;
  }
}

// Sums over the observations of row i (ObsMap) of the likelihood's derivative and information at
// mode_i + offset_e; one observation per row: the row's own y / offset.
__device__ __forceinline__ void obs_d1_info(const ObsMap& ob, int lik, double aux, int i, double mi,
                                            const double* y, const double* offset, bool want_info, double& d1,
                                            double& w) {
  if (ob.ptr == nullptr) {
    const double l = offset ? mi + offset[i] : mi;
    d1 = lik_d1(lik, aux, y[i], l);
    if (want_info) w = lik_info(lik, aux, y[i], l);
    return;
  }
  double s1 = 0., sw = 0.;
  for (int e = ob.ptr[i]; e < ob.ptr[i + 1]; ++e) {
    const double l = ob.offset ? mi + ob.offset[e] : mi;
    s1 += lik_d1(lik, aux, ob.y[e], l);
    if (want_info) sw += lik_info(lik, aux, ob.y[e], l);
  }
  d1 = s1;
  if (want_info) w = sw;
}

__global__ void __launch_bounds__(kBT) newton_prep_kernel(NewtonPrepArgs a) {
  for (int i = blockIdx.x * kBT + threadIdx.x; i < a.n; i += gridDim.x * kBT) {
    double d1 = 0., winfo = 0.;
    obs_d1_info(a.obs, a.lik, a.aux, i, a.loc[i], a.y, a.offset, a.W_update != 0, d1, winfo);
    a.d1[i] = d1;
    // W is only refreshed when requested (information_changes_*); otherwise the stored W is used
    const double w = a.W_update ? winfo : a.W[i];
    if (a.W_update) a.W[i] = w;
    if (a.rhs) a.rhs[i] = fma(w, a.mode[i], d1);
    if (a.dw) {
      const double dw = a.Dinv[i] + w;
      a.dw[i] = dw;
      if (a.sdw) a.sdw[i] = sqrt(dw);
    }
  }
}

__global__ void __launch_bounds__(kBT) latent_scalars_kernel(ScalarArgs a, double* partials) {
  double acc[kLatentScalars];
#pragma unroll
  for (int q = 0; q < kLatentScalars; ++q) acc[q] = 0.;
  for (int i = blockIdx.x * kBT + threadIdx.x; i < a.n; i += gridDim.x * kBT) {
    const int k = i < a.m ? i : a.m;
    const int* nb = a.nbr + (size_t)i * a.m;
    const double* v = a.Bv + (size_t)i * a.m;
    const double mi = a.mode[i];
    double bm = mi, dbm = 0., bv = 0., dbv = 0.;
    if (a.vS) bv = a.vS[i];
    for (int r = 0; r < k; ++r) {
      const int j = nb[r];
      const double mj = a.mode[j];
      bm = fma(v[r], mj, bm);
      if (a.dBv) dbm = fma(a.dBv[(size_t)i * a.m + r], mj, dbm);
      if (a.vS) {
        const double sj = a.vS[j];
        bv = fma(v[r], sj, bv);
        if (a.dBv) dbv = fma(a.dBv[(size_t)i * a.m + r], sj, dbv);
      }
    }
    const double Di = a.Dinv[i];
    acc[kSqQuad] += bm * Di * bm;
    double cnt = 1.;
    if (a.obs.ptr == nullptr) {
      const double li = a.offset ? mi + a.offset[i] : mi;
      acc[kSqLogLik] += lik_loglik(a.lik, a.aux, a.y[i], li);
      const double r = a.y[i] - li;
      acc[kSqRss] += r * r;
    } else {   // the row's observations (repeated coordinates)
      const int e0 = a.obs.ptr[i], e1 = a.obs.ptr[i + 1];
      cnt = (double)(e1 - e0);
      for (int e = e0; e < e1; ++e) {
        const double li = a.obs.offset ? mi + a.obs.offset[e] : mi;
        acc[kSqLogLik] += lik_loglik(a.lik, a.aux, a.obs.y[e], li);
        const double r = a.obs.y[e] - li;
        acc[kSqRss] += r * r;
      }
    }
    acc[kSqLogDinv] += log(Di);
    if (a.dw) {
      const double dwi = a.dw[i];
      acc[kSqLogDw] += log(dwi);
      acc[kSqTrVar] += Di / dwi;
      acc[kSqTrDw] += cnt / dwi;   // x dW_i/dlog aux = -cnt_i / aux on the host
      if (a.dD) acc[kSqTrRng] += Di * a.dD[i] * Di / dwi;
    }
    if (a.dBv) {
      const double dDi = a.dD[i];
      acc[kSqDQuadRng] += dbm * Di * bm;
      acc[kSqDDQuad] += bm * Di * dDi * Di * bm;
      acc[kSqDinvDD] += Di * dDi;
      if (a.vS) {
        acc[kSqImpVar] += bv * Di * bm;
        acc[kSqImpRng] += dbv * Di * bm + bv * Di * dbm - bv * Di * dDi * Di * bm;
      }
    }
  }
  __shared__ double red[kLatentScalars][kBT];
#pragma unroll
  for (int q = 0; q < kLatentScalars; ++q) red[q][threadIdx.x] = acc[q];
  __syncthreads();
  for (int off = kBT / 2; off > 0; off >>= 1) {
    if ((int)threadIdx.x < off) {
#pragma unroll
      for (int q = 0; q < kLatentScalars; ++q) red[q][threadIdx.x] += red[q][threadIdx.x + off];
    }
    __syncthreads();
  }
  if ((int)threadIdx.x < kLatentScalars)
    partials[(size_t)blockIdx.x * kLatentScalars + threadIdx.x] = red[threadIdx.x][0];
}

// Per-column trace sums for the gradient (likelihoods.h:12440-12465, 12520-12546).
__global__ void __launch_bounds__(kBT) grad_cols_kernel(GradColsArgs a, int shift, double* partials) {
  const int T = 1 << shift;
  const int c = (threadIdx.x & (T - 1)) + blockIdx.y * 64;
  const int rpb = kBT >> shift;
  const int t = a.t;
  double acc[kGradCols];
#pragma unroll
  for (int q = 0; q < kGradCols; ++q) acc[q] = 0.;
  if (c < t) {
    for (int i = blockIdx.x * rpb + (threadIdx.x >> shift); i < a.n; i += gridDim.x * rpb) {
      const int k = i < a.m ? i : a.m;
      const int* nb = a.nbr + (size_t)i * a.m;
      const double* bv = a.Bv + (size_t)i * a.m;
      const double* dbv = a.dBv + (size_t)i * a.m;
      const size_t o = (size_t)i * t + c;
      const double ui = a.U[o], pi = a.P[o];
      double bu = ui, dbu = 0., bp = pi, dbp = 0.;
#pragma unroll 2
      for (int r = 0; r < k; ++r) {
        const size_t oj = (size_t)nb[r] * t + c;
        const double uj = a.U[oj], pj = a.P[oj];
        bu = fma(bv[r], uj, bu);
        bp = fma(bv[r], pj, bp);
        dbu = fma(dbv[r], uj, dbu);
        dbp = fma(dbv[r], pj, dbp);
      }
      const double Di = a.Dinv[i], dDi = a.dD[i], wi = a.W[i];
      const double daux = a.obs_ptr ? a.daux * (double)(a.obs_ptr[i + 1] - a.obs_ptr[i]) : a.daux;
      acc[0] -= Di * bu * bp;
      acc[1] -= Di * bp * bp;
      acc[2] += Di * (dbu * bp + bu * dbp - Di * dDi * bu * bp);
      acc[3] += Di * (2. * dbp * bp - Di * dDi * bp * bp) + 2. * wi * bp * dbp;
      acc[4] += ui * daux * pi;
      acc[5] += bp * daux * bp;
    }
  }
  block_col_reduce<kGradCols>(acc, shift, c, t, partials);
}

// Row-wise stochastic d log|Sigma W + I| / d mode (vadu branch, likelihoods.h:12320-12341).
__global__ void __launch_bounds__(kBT) mode_deriv_kernel(ModeDerivArgs a, int shift) {
  // No FMA contraction in this kernel: pass 2 must recompute the products of pass 1
  // bit-identically (for t = 1 the centred values are then exactly 0 -> c = 1).
#pragma clang fp contract(off)
  const int T = 1 << shift;
  const int lane = threadIdx.x & (T - 1);
  const int rpb = kBT >> shift;
  const int t = a.t;
  for (int i = blockIdx.x * rpb + (threadIdx.x >> shift); i < a.n; i += gridDim.x * rpb) {
    const int k = i < a.m ? i : a.m;
    const int* nb = a.nbr + (size_t)i * a.m;
    const double* bv = a.Bv + (size_t)i * a.m;
    double dWi;
    if (a.obs.ptr == nullptr) {
      dWi = lik_dinfo(a.lik, a.aux, a.y ? a.y[i] : 0., a.offset ? a.loc[i] + a.offset[i] : a.loc[i]);
    } else {   // Z^T dW: the row's observations
      dWi = 0.;
      for (int e = a.obs.ptr[i]; e < a.obs.ptr[i + 1]; ++e)
        dWi += lik_dinfo(a.lik, a.aux, a.obs.y[e], a.obs.offset ? a.loc[i] + a.obs.offset[e] : a.loc[i]);
    }
    // pass 1: row means of z1 = U dW P and zP = (BP)^2 dW over the t probes
    // (c_var == 0 -> c = 1, CG_utils.cpp:1036-1039).
    double s1 = 0., sP = 0.;
    if (a.stage < 2) {
      for (int c = lane; c < a.t_valid; c += T) {
        const size_t o = (size_t)i * t + c;
        double bp = a.P[o];
        for (int r = 0; r < k; ++r) bp = fma(bv[r], a.P[(size_t)nb[r] * t + c], bp);
        s1 += a.U[o] * dWi * a.P[o];
        sP += bp * dWi * bp;
      }
      for (int off = T >> 1; off > 0; off >>= 1) {
        s1 += __shfl_xor(s1, off, 64);
        sP += __shfl_xor(sP, off, 64);
      }
      if (a.stage == 1) {   // sharded: this rank's column sums, all-reduced by the caller
        if (lane == 0) { a.mom[2 * (size_t)i] = s1; a.mom[2 * (size_t)i + 1] = sP; }
        continue;
      }
    } else {
      s1 = a.mom[2 * (size_t)i];
      sP = a.mom[2 * (size_t)i + 1];
    }
    const double tr1 = s1 / a.t_all, trP = sP / a.t_all;
    // pass 2: centred covariance / variance -> optimal c (CalcOptimalCVectorized)
    double cv = 0., vv = 0.;
    if (a.stage < 3) {
      for (int c = lane; c < a.t_valid; c += T) {
        const size_t o = (size_t)i * t + c;
        double bp = a.P[o];
        for (int r = 0; r < k; ++r) bp = fma(bv[r], a.P[(size_t)nb[r] * t + c], bp);
        const double z1 = a.U[o] * dWi * a.P[o] - tr1;
        const double zP = bp * dWi * bp - trP;
        cv += z1 * zP;
        vv += zP * zP;
      }
      for (int off = T >> 1; off > 0; off >>= 1) {
        cv += __shfl_xor(cv, off, 64);
        vv += __shfl_xor(vv, off, 64);
      }
      if (a.stage == 2) {   // sharded: centred sums of this rank
        if (lane == 0) { a.mom2[2 * (size_t)i] = cv; a.mom2[2 * (size_t)i + 1] = vv; }
        continue;
      }
    } else {
      cv = a.mom2[2 * (size_t)i];
      vv = a.mom2[2 * (size_t)i + 1];
    }
    cv /= a.t_all;
    vv /= a.t_all;
    const double copt = (vv == 0.) ? 1. : cv / vv;
    if (lane == 0) a.dmll[i] = 0.5 * (tr1 + copt * (dWi / a.dw[i]) - copt * trP);
  }
}

}  // namespace

// ------------------------------------------------------------------ launchers
// Form of the t >= 2 operator kernels (A/B switch GPBOOST_AMD_SPMV="ch,pers,cap"; ch = -1,
// the default, selects the wave-per-row kernels).
struct SpmvForm {
  int ch, pers, cap;
};
SpmvForm spmv_form() {
  static const SpmvForm f = [] {
    SpmvForm r{-1, 0, 2048};
    if (const char* e = std::getenv("GPBOOST_AMD_SPMV")) std::sscanf(e, "%d,%d,%d", &r.ch, &r.pers, &r.cap);
    if (r.cap < 8) r.cap = 8;
    return r;
  }();
  return f;
}

// The SpMV grids cover every row with one pass (no grid-stride loop): the XCD block mapping
// needs the whole grid, and at n <= 2^31 / rpb the x dimension never overflows.
void launch_b_apply(const SparseB& B, const double* vals, bool unit, const double* X, int t, const double* scale,
                    double* Y, hipStream_t s) {
  if (B.n <= 0) return;
  static const bool old1 = std::getenv("GPBOOST_AMD_SPMV1_OLD") != nullptr;   // A/B: one row per group
  static const bool groups1 = std::getenv("GPBOOST_AMD_SPMV1_GROUPS") != nullptr;   // A/B: lane-group forms
  if (t == 1 && !old1 && !groups1 && B.ell_idx != nullptr && vals == B.vals_of) {
    hipLaunchKernelGGL(b_apply1e_kernel, dim3(grid_x(B.n, kBT, 1 << 30)), dim3(kBT), 0, s, B.n, B.m, B.ell_idx,
                       B.ell_val, unit ? 1 : 0, X, scale, Y);
    HIP_CHECK(hipGetLastError());
    return;
  }
  if (t == 1 && B.m <= 2 * k1G && !old1) {
    hipLaunchKernelGGL((b_apply1m_kernel<k1G, k1R>), dim3(grid_x(B.n, kBT / k1G * k1R, 1 << 30)), dim3(kBT), 0, s,
                       B.n, B.m, B.nbr, vals, unit ? 1 : 0, X, scale, Y);
    HIP_CHECK(hipGetLastError());
    return;
  }
  if (t == 1) {
    constexpr int G = 32;
    hipLaunchKernelGGL(b_apply1_kernel<G>, dim3(grid_x(B.n, kBT / G, 1 << 30)), dim3(kBT), 0, s, B.n, B.m, B.nbr,
                       vals, unit ? 1 : 0, X, scale, Y);
    HIP_CHECK(hipGetLastError());
    return;
  }
  const Lanes L = lanes_for(t);
  const SpmvForm f = spmv_form();
  if (f.ch < 0 && B.m <= 64) {   // default: wave-per-row form
    const dim3 g(grid_x(B.n, kBT / 64, 1 << 30), L.gy);
    if (f.ch == -2)
      hipLaunchKernelGGL(b_apply_wave_kernel<32>, g, dim3(kBT), 0, s, B.n, B.m, B.nbr, vals, unit ? 1 : 0, X, t, scale, Y);
    else
      hipLaunchKernelGGL(b_apply_wave_kernel<kWaveChunk>, g, dim3(kBT), 0, s, B.n, B.m, B.nbr, vals, unit ? 1 : 0, X, t,
                         scale, Y);
    HIP_CHECK(hipGetLastError());
    return;
  }
  const dim3 grid(grid_x(B.n, L.rpb, f.pers ? f.cap : (1 << 30)), L.gy);
#define GPB_B_APPLY(CH, P)                                                                                     \
  hipLaunchKernelGGL((b_apply_kernel<CH, P>), grid, dim3(kBT), 0, s, B.n, B.m, B.nbr, vals, unit ? 1 : 0, X, t, \
                     L.shift, scale, Y)
  if (f.ch == 0) { if (f.pers) GPB_B_APPLY(0, true); else GPB_B_APPLY(0, false); }
  else { if (f.pers) GPB_B_APPLY(16, true); else GPB_B_APPLY(16, false); }
#undef GPB_B_APPLY
  HIP_CHECK(hipGetLastError());
}

void launch_bt_apply(const SparseB& B, const double* vals, bool unit, const double* X, int t, const double* pre,
                     const double* W, const double* H, double* Y, hipStream_t s) {
  if (B.n <= 0) return;
  const double* tval = (B.tval != nullptr && vals == B.tval_of) ? B.tval : nullptr;
  static const bool old1 = std::getenv("GPBOOST_AMD_SPMV1_OLD") != nullptr;
  static const bool groups1 = std::getenv("GPBOOST_AMD_BT1_GROUPS") != nullptr;   // A/B: lane-group form
  if (t == 1 && tval != nullptr && !old1 && !groups1 && B.seg_rb != nullptr) {
    static const bool shfl = std::getenv("GPBOOST_AMD_BT1_SCAN_SHFL") != nullptr;   // A/B: ds_bpermute scan
    static const bool one = std::getenv("GPBOOST_AMD_BT1_E1") != nullptr;   // A/B: one entry per lane
    static const int epl = [] {   // A/B: GPBOOST_AMD_BT1_E = 2 / 4 (unpaired layout, E entries per lane)
      const char* e = std::getenv("GPBOOST_AMD_BT1_E");
      return e ? std::atoi(e) : 0;
    }();
    const dim3 g((B.nseg + kSegWaves - 1) / kSegWaves), b(64 * kSegWaves);
    if (!one && !shfl && epl == 0 && B.seg_info != nullptr) {   // default: paired layout
#ifndef GPB_PAIR_U
#define GPB_PAIR_U 4
#endif
      hipLaunchKernelGGL((bt_apply1p_kernel<GPB_PAIR_U>), g, b, 0, s, B.nseg, B.seg_info,
                         reinterpret_cast<const uint2*>(B.seg_pk2), reinterpret_cast<const double2*>(B.seg_val2),
                         unit ? 1 : 0, X, pre, W, H, Y);
    } else if (!one && !shfl && B.seg_info != nullptr && (epl == 2 || epl == 4)) {
      if (epl == 4)
        hipLaunchKernelGGL((bt_apply1sE_kernel<4, 2>), g, b, 0, s, B.nseg, B.seg_info, B.seg_pk2, B.seg_val2,
                           unit ? 1 : 0, X, pre, W, H, Y);
      else
        hipLaunchKernelGGL((bt_apply1sE_kernel<2, 4>), g, b, 0, s, B.nseg, B.seg_info, B.seg_pk2, B.seg_val2,
                           unit ? 1 : 0, X, pre, W, H, Y);
    } else if (!one && !shfl)
      hipLaunchKernelGGL(bt_apply1s2_kernel<true>, g, b, 0, s, B.nseg, B.seg_rb, B.seg_pk, B.tptr, tval,
                         unit ? 1 : 0, X, pre, W, H, Y);
    else if (shfl)
      hipLaunchKernelGGL(bt_apply1s_kernel<false>, g, b, 0, s, B.nseg, B.seg_rb, B.seg_pk, B.tptr, tval,
                         unit ? 1 : 0, X, pre, W, H, Y);
    else
      hipLaunchKernelGGL(bt_apply1s_kernel<true>, g, b, 0, s, B.nseg, B.seg_rb, B.seg_pk, B.tptr, tval,
                         unit ? 1 : 0, X, pre, W, H, Y);
    HIP_CHECK(hipGetLastError());
    return;
  }
  if (t == 1 && tval != nullptr && !old1) {
    const int nlb = (B.nlong + kBT / 64 - 1) / (kBT / 64);
    // lane-group shape (A/B builds: GPB_BT1_SHAPE): 1 = 16 lanes x 4 entries, 2 rows per group (the
    // whole <= kLongRow list in one shot; 18.1 us at n = 100k), 0 = 16 x 2, 4 rows (20.3 us),
    // 2 = 32 x 2, 2 rows (22.1 us), 3 = 16 x 4, 4 rows (23.9 us)
#ifndef GPB_BT1_SHAPE
#define GPB_BT1_SHAPE 1
#endif
#if GPB_BT1_SHAPE == 1
    constexpr int G1 = 16, R1 = 2, E1 = 4;
#elif GPB_BT1_SHAPE == 2
    constexpr int G1 = 32, R1 = 2, E1 = 2;
#elif GPB_BT1_SHAPE == 3
    constexpr int G1 = 16, R1 = 4, E1 = 4;
#else
    constexpr int G1 = k1G, R1 = k1R, E1 = 2;
#endif
    const int nmain = grid_x(B.n, kBT / G1 * R1, 1 << 30);
    hipLaunchKernelGGL((bt_apply1m_kernel<G1, R1, E1>), dim3(nmain + nlb), dim3(kBT), 0, s, B.n, B.tptr, B.trow, tval,
                       unit ? 1 : 0, X, pre, W, H, Y, nmain, B.longr, B.nlong);
    HIP_CHECK(hipGetLastError());
    return;
  }
  if (t == 1 && tval != nullptr) {
    constexpr int G = 32;
    hipLaunchKernelGGL(bt_apply1_kernel<G>, dim3(grid_x(B.n, kBT / G, 1 << 30)), dim3(kBT), 0, s, B.n, B.tptr,
                       B.trow, tval, unit ? 1 : 0, X, pre, W, H, Y);
    HIP_CHECK(hipGetLastError());
    return;
  }
  const Lanes L = lanes_for(t);
  const SpmvForm f = spmv_form();
  if (f.ch < 0 && tval != nullptr) {   // default: wave-per-row form
    const dim3 g(grid_x(B.n, kBT / 64, 1 << 30), L.gy);
    if (f.ch == -2)
      hipLaunchKernelGGL(bt_apply_wave_kernel<32>, g, dim3(kBT), 0, s, B.n, B.tptr, B.trow, tval, unit ? 1 : 0, X, t,
                         pre, W, H, Y);
    else
      hipLaunchKernelGGL(bt_apply_wave_kernel<kWaveChunk>, g, dim3(kBT), 0, s, B.n, B.tptr, B.trow, tval, unit ? 1 : 0,
                         X, t, pre, W, H, Y);
    HIP_CHECK(hipGetLastError());
    return;
  }
  const dim3 grid(grid_x(B.n, L.rpb, f.pers ? f.cap : (1 << 30)), L.gy);
#define GPB_BT_APPLY(CH, P)                                                                                     \
  hipLaunchKernelGGL((bt_apply_kernel<CH, P>), grid, dim3(kBT), 0, s, B.n, B.tptr, B.trow, B.tslot, vals, tval, \
                     unit ? 1 : 0, X, t, L.shift, pre, W, H, Y)
  if (f.ch == 0) { if (f.pers) GPB_BT_APPLY(0, true); else GPB_BT_APPLY(0, false); }
  else { if (f.pers) GPB_BT_APPLY(16, true); else GPB_BT_APPLY(16, false); }
#undef GPB_BT_APPLY
  HIP_CHECK(hipGetLastError());
}

namespace {
template <bool TRANS>
void launch_tiled(const SparseB& B, const TileOp& op, const double* vals, const double* X, int t,
                  const double* scale, const double* W, const double* H, double* Y, hipStream_t s) {
  if (B.n <= 0 || t <= 0) return;
  const int tc = t < 64 ? t : 64;
  const size_t lds = (size_t)std::max(op.umax, 1) * tc * sizeof(double);
  static bool attr = false;
  if (!attr) {   // the largest union the plan builder admits (kTileUnion rows x 64 columns)
    HIP_CHECK(hipFuncSetAttribute((const void*)apply_tile_kernel<TRANS>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)(sizeof(double) * kTileUnion * 64)));
    attr = true;
  }
  const int nb = op.ntile + (op.nfb + kTileThreads / 64 - 1) / (kTileThreads / 64);
  hipLaunchKernelGGL((apply_tile_kernel<TRANS>), dim3(nb, (t + 63) / 64), dim3(kTileThreads), lds, s, B.n, B.m, B.nbr,
                     B.tptr, B.trow, op, vals, X, t, scale, W, H, Y);
  HIP_CHECK(hipGetLastError());
}
}  // namespace

void launch_b_apply_tiled(const SparseB& B, const TileOp& op, const double* vals, const double* X, int t,
                          const double* scale, double* Y, hipStream_t s) {
  launch_tiled<false>(B, op, vals, X, t, scale, nullptr, nullptr, Y, s);
}

void launch_bt_apply_tiled(const SparseB& B, const TileOp& op, const double* tval, const double* X, int t,
                           const double* W, const double* H, double* Y, hipStream_t s) {
  launch_tiled<true>(B, op, tval, X, t, nullptr, W, H, Y, s);
}

void launch_gather(int count, const int* idx, const double* src, double* dst, hipStream_t s) {
  if (count <= 0) return;
  hipLaunchKernelGGL(gather_kernel, dim3(grid_x(count, kBT)), dim3(kBT), 0, s, count, idx, src, dst);
  HIP_CHECK(hipGetLastError());
}

void launch_coldots(int n, int t, int np, const double* const* A, const double* const* Bm, double* partials,
                    double* out, hipStream_t s) {
  const Lanes L = lanes_for(t);
  const int gx = grid_x(n, L.rpb, kMaxRedBlocks);
  const dim3 grid(gx, L.gy);
  switch (np) {
    case 1:
      hipLaunchKernelGGL(coldots_kernel<1>, grid, dim3(kBT), 0, s, n, t, L.shift, A[0], Bm[0], nullptr, nullptr,
                         nullptr, nullptr, partials);
      break;
    case 2:
      hipLaunchKernelGGL(coldots_kernel<2>, grid, dim3(kBT), 0, s, n, t, L.shift, A[0], Bm[0], A[1], Bm[1], nullptr,
                         nullptr, partials);
      break;
    case 3:
      hipLaunchKernelGGL(coldots_kernel<3>, grid, dim3(kBT), 0, s, n, t, L.shift, A[0], Bm[0], A[1], Bm[1], A[2],
                         Bm[2], partials);
      break;
    default: Fatal("coldots: np = %d", np);
  }
  HIP_CHECK(hipGetLastError());
  hipLaunchKernelGGL(reduce_blocks_kernel, dim3(np * t), dim3(kBT), 0, s, partials, gx, np * t, out);
  HIP_CHECK(hipGetLastError());
}

void launch_cg_update(int n, int t, const double* a, const double* H, const double* V, double* U, double* R,
                      double* partials, double* rr, hipStream_t s) {
  const Lanes L = lanes_for(t);
  const int gx = grid_x(n, L.rpb, kMaxRedBlocks);
  hipLaunchKernelGGL(cg_update_kernel, dim3(gx, L.gy), dim3(kBT), 0, s, n, t, L.shift, a, H, V, U, R, partials);
  HIP_CHECK(hipGetLastError());
  hipLaunchKernelGGL(reduce_blocks_kernel, dim3(t), dim3(kBT), 0, s, partials, gx, t, rr);
  HIP_CHECK(hipGetLastError());
}

void launch_h_update(int n, int t, const double* b, const double* Z, double* H, hipStream_t s) {
  const size_t total = (size_t)n * t;
  int g = (int)((total + kBT - 1) / kBT);
  if (g > kMaxGridX) g = kMaxGridX;
  hipLaunchKernelGGL(h_update_kernel, dim3(g), dim3(kBT), 0, s, total, t, b, Z, H);
  HIP_CHECK(hipGetLastError());
}

void launch_pcg_init(int t, int n_valid, int n_single, int pmax_single, int pmax_block, double zero_sq,
                     const double* rr0, int* act, int* ctl, hipStream_t s) {
  hipLaunchKernelGGL(pcg_init_kernel, dim3(1), dim3(64), 0, s, t, n_valid, n_single, pmax_single, pmax_block, zero_sq,
                     rr0, act, ctl);
  HIP_CHECK(hipGetLastError());
}

void launch_pcg_block_sum(int n_valid, int n_single, const double* rr, double* out, hipStream_t s) {
  hipLaunchKernelGGL(pcg_block_sum_kernel, dim3(1), dim3(64), 0, s, n_valid, n_single, rr, out);
  HIP_CHECK(hipGetLastError());
}

void launch_pcg_check(int j, int t, int n_single, int pmax_single, int pmax_block, double delta, const double* rr,
                      const double* gsum, int nblock, int* act, int* ctl, int* host_ctl, int seq, hipStream_t s) {
  hipLaunchKernelGGL(pcg_check_kernel, dim3(1), dim3(64), 0, s, j, t, n_single, pmax_single, pmax_block, delta, rr,
                     gsum, nblock, act, ctl, host_ctl, seq);
  HIP_CHECK(hipGetLastError());
}

void launch_pack_columns(int n, int ncols, const double* src, int ld_src, int c_src, double* dst, int ld_dst,
                         int c_dst, hipStream_t s) {
  const size_t total = (size_t)n * ncols;
  int g = (int)((total + kBT - 1) / kBT);
  if (g > kMaxGridX) g = kMaxGridX;
  if (g < 1) g = 1;
  hipLaunchKernelGGL(pack_columns_kernel, dim3(g), dim3(kBT), 0, s, (size_t)n, ncols, src, ld_src, c_src, dst, ld_dst,
                     c_dst);
  HIP_CHECK(hipGetLastError());
}

void launch_copy(size_t count, const double* X, double* Y, hipStream_t s) {
  int g = (int)((count + kBT - 1) / kBT);
  if (g > kMaxGridX) g = kMaxGridX;
  if (g < 1) g = 1;
  hipLaunchKernelGGL(copy_kernel, dim3(g), dim3(kBT), 0, s, count, X, Y);
  HIP_CHECK(hipGetLastError());
}

// CapChangeModeUpdateNewton (likelihoods.h:11800-11810): |mnew - mode| capped at MAX_CHANGE_MODE_NEWTON_ = log(100)
__global__ void cap_mode_kernel(size_t total, const double* __restrict__ mode, double* __restrict__ mnew) {
  constexpr double kMaxChange = 4.605170185988091;
  for (size_t o = (size_t)blockIdx.x * kBT + threadIdx.x; o < total; o += (size_t)gridDim.x * kBT) {
    const double c = fabs(mnew[o] - mode[o]);
    if (c > kMaxChange) mnew[o] = mode[o] + (mnew[o] - mode[o]) / c * kMaxChange;
  }
}

void launch_cap_mode_change(size_t count, const double* mode, double* mnew, hipStream_t s) {
  int g = (int)((count + kBT - 1) / kBT);
  if (g > kMaxGridX) g = kMaxGridX;
  if (g < 1) g = 1;
  hipLaunchKernelGGL(cap_mode_kernel, dim3(g), dim3(kBT), 0, s, count, mode, mnew);
  HIP_CHECK(hipGetLastError());
}

void launch_axpby(size_t count, double alpha, const double* X, double beta, const double* Y, double* Z,
                  hipStream_t s) {
  int g = (int)((count + kBT - 1) / kBT);
  if (g > kMaxGridX) g = kMaxGridX;
  if (g < 1) g = 1;
  hipLaunchKernelGGL(axpby_kernel, dim3(g), dim3(kBT), 0, s, count, alpha, X, beta, Y, Z);
  HIP_CHECK(hipGetLastError());
}

void launch_cg_alpha(int t, const double* rz, const double* hv, const int* act, double* a, double* hist,
                     hipStream_t s) {
  hipLaunchKernelGGL(cg_alpha_kernel, dim3((t + 63) / 64), dim3(64), 0, s, t, rz, hv, act, a, hist);
  HIP_CHECK(hipGetLastError());
}

void launch_cg_beta(int t, const double* rz_new, double* rz, const int* act, double* b, double* hist,
                    hipStream_t s) {
  hipLaunchKernelGGL(cg_beta_kernel, dim3((t + 63) / 64), dim3(64), 0, s, t, rz_new, rz, act, b, hist);
  HIP_CHECK(hipGetLastError());
}

void launch_newton_prep(const NewtonPrepArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(newton_prep_kernel, dim3(grid_x(a.n, kBT, 1024)), dim3(kBT), 0, s, a);
  HIP_CHECK(hipGetLastError());
}

void launch_latent_scalars(const ScalarArgs& a, double* partials, double* out, hipStream_t s) {
  const int gx = grid_x(a.n, kBT, kMaxRedBlocks);
  hipLaunchKernelGGL(latent_scalars_kernel, dim3(gx), dim3(kBT), 0, s, a, partials);
  HIP_CHECK(hipGetLastError());
  hipLaunchKernelGGL(reduce_blocks_kernel, dim3(kLatentScalars), dim3(kBT), 0, s, partials, gx, kLatentScalars, out);
  HIP_CHECK(hipGetLastError());
}

void launch_grad_cols(const GradColsArgs& a, double* partials, double* out, hipStream_t s) {
  const Lanes L = lanes_for(a.t);
  const int gx = grid_x(a.n, L.rpb, kMaxRedBlocks);
  hipLaunchKernelGGL(grad_cols_kernel, dim3(gx, L.gy), dim3(kBT), 0, s, a, L.shift, partials);
  HIP_CHECK(hipGetLastError());
  hipLaunchKernelGGL(reduce_blocks_kernel, dim3(kGradCols * a.t), dim3(kBT), 0, s, partials, gx, kGradCols * a.t,
                     out);
  HIP_CHECK(hipGetLastError());
}

// gamma shape gradient records (likelihoods.h:5139-5202 with SigmaI_plus_W_inv_diag = d_log_det / dinfo,
// :5126-5127, d_log_det = 2 d_mll_d_mode): [l + y e^-l, W (2 dmll / dinfo), d1 vS]
__global__ void gamma_aux_rec_kernel(int n, double aux, const double* __restrict__ y, const double* __restrict__ off,
                                     const double* __restrict__ loc, const double* __restrict__ W,
                                     const double* __restrict__ dmll, const double* __restrict__ d1,
                                     const double* __restrict__ vS, double* __restrict__ rec) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double l = off ? loc[i] + off[i] : loc[i];
  const double e = y[i] * exp(-l);
  rec[3 * (size_t)i] = l + e;
  rec[3 * (size_t)i + 1] = W[i] * ((2. * dmll[i]) / (-aux * e));
  rec[3 * (size_t)i + 2] = d1[i] * vS[i];
}

void launch_gamma_aux_rec(int n, double aux, const double* y, const double* off, const double* loc, const double* W,
                          const double* dmll, const double* d1, const double* vS, double* rec, hipStream_t s) {
  hipLaunchKernelGGL(gamma_aux_rec_kernel, dim3(grid_x(n, kBT)), dim3(kBT), 0, s, n, aux, y, off, loc, W, dmll, d1, vS,
                     rec);
  HIP_CHECK(hipGetLastError());
}

void launch_grad_f(int n, const double* d1, const double* dmll, const double* W, const double* vS, double* out,
                   hipStream_t s) {
  hipLaunchKernelGGL(grad_f_kernel, dim3(grid_x(n, kBT)), dim3(kBT), 0, s, n, d1, dmll, W, vS, out);
  HIP_CHECK(hipGetLastError());
}

void launch_mode_deriv(const ModeDerivArgs& a, hipStream_t s) {
  const Lanes L = lanes_for(a.t);
  hipLaunchKernelGGL(mode_deriv_kernel, dim3(grid_x(a.n, L.rpb)), dim3(kBT), 0, s, a, L.shift);
  HIP_CHECK(hipGetLastError());
}

}  // namespace gpb_amd
