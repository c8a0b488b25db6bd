// Numeric phases of the sparse Cholesky of Sigma^-1 + W (sparse_chol.h) on gfx950.
//
// Every launch executes one CholOp of a host-built schedule (sparse_chol_sym.cpp): the tasks of one
// level of the supernodal tree, so independent fronts of a level share one grid. Kernels:
//   chol_asm_tile   one workgroup per lower 64 x 64 front tile: the children's update blocks gathered through
//                   their position maps (extend-add as a gather, children in a fixed order, no atomics)
//   chol_asm_entries A's entries (+ W on the diagonal) added to the panel columns
//   chol_diag       one workgroup (4 waves) per 64 x 64 diagonal block: the Cholesky pivots and the
//                   block inverse W = L^-1 in one register-resident sweep (row r of L and column r of
//                   W on lane r, columns / rows split over the waves, the pivot column broadcast
//                   through LDS, one barrier per step)
//   chol_gemm       one 64 x 64 output tile per 256-thread workgroup, v_mfma_f64_16x16x4 on 4 waves
//                   (2 x 2 MFMA tiles each), K staged through double-buffered LDS: TRSM (times W^T),
//                   the panel updates, the update block U -= L21 L21^T (K = ns), the solves' block
//                   steps and the selected inverse's products
//   chol_gather_s / chol_mirror / chol_asmv / chol_gather_x / chol_scatter_x: the selected inverse's
//                   parent-to-child gathers, symmetric completion, and the solves' front vectors.
// Reductions (log-determinant, traces) are two-pass with a fixed order: results are bitwise repeatable.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <string>
#include <map>
#include <utility>
#include <vector>

#include "sparse_chol.h"

namespace gpb_amd {
namespace {

typedef double double4_t __attribute__((ext_vector_type(4)));

struct Bufs {
  double* p[5];   // kCbF, kCbS, kCbW, kCbY, kCbP
};

struct DevPlan {
  int n;
  const int* sfirst;
  const int64_t* rptr;
  const int* rows;
  const int64_t* foff;
  const int* rel;
  const int* cptr;
  const int* child;
  const int* sparent;
  const int* perm;
  const int64_t* cinv_off;
  const int* cinv;
};

__device__ __forceinline__ int lower_bound_dev(const int* a, int n, int v) {
  int lo = 0, hi = n;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (a[mid] < v) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

// ---- A's entries: clique sums of D^-1 B B^T and of its range derivative
__global__ void __launch_bounds__(256) chol_entry_values_kernel(int64_t ne, const int64_t* __restrict__ cptr,
                                                                const uint64_t* __restrict__ ctr, int m,
                                                                const double* __restrict__ Bv,
                                                                const double* __restrict__ Dinv,
                                                                const double* __restrict__ dBv,
                                                                const double* __restrict__ dD, double* __restrict__ aval,
                                                                double* __restrict__ daval) {
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < ne; e += (int64_t)gridDim.x * blockDim.x) {
    double v = 0., dv = 0.;
    for (int64_t c = cptr[e]; c < cptr[e + 1]; ++c) {
      const uint64_t w = ctr[c];
      const int r = (int)(w >> 16), a = (int)((w >> 8) & 255), b = (int)(w & 255);
      const double* br = Bv + (size_t)r * m;
      const double ba = a == 0 ? 1. : br[a - 1];
      const double bb = b == 0 ? 1. : br[b - 1];
      const double di = Dinv[r];
      v += di * ba * bb;
      if (daval != nullptr) {
        const double* dr = dBv + (size_t)r * m;
        const double da = a == 0 ? 0. : dr[a - 1];
        const double db = b == 0 ? 0. : dr[b - 1];
        dv += di * (da * bb + ba * db) - di * di * dD[r] * ba * bb;
      }
    }
    aval[e] = v;
    if (daval != nullptr) daval[e] = dv;
  }
}

// ---- front assembly (factorization), two launches per level:
// (1) one workgroup per lower 64 x 64 tile of a front: F[i][j] = sum over the children of U_child[inv(i)][inv(j)]
//     (the extend-add as a gather through the children's position maps, children in a fixed order; zero where
//     no child contributes), so every tile of every front of the level is written in parallel;
// (2) A's entries of the panel columns (and W on the diagonal) added, one target per entry.
__global__ void __launch_bounds__(256) chol_asm_tile_kernel(const CholColTask* __restrict__ tasks, int64_t t0,
                                                            DevPlan P, double* __restrict__ F, int* info_reset) {
  const CholColTask tk = tasks[t0 + blockIdx.x];
  if (info_reset != nullptr && blockIdx.x == 0 && threadIdx.x == 0) *info_reset = 0;   // first op of a factorization
  const int s = tk.s, rt = tk.c0, ct = tk.c1;
  const int ns = P.sfirst[s + 1] - P.sfirst[s];
  const int fs = ns + (int)(P.rptr[s + 1] - P.rptr[s]);
  __shared__ int ri[64], ci[64];
  const int tid = threadIdx.x;
  const int ii = tid & 63;
  double acc[16];
#pragma unroll
  for (int q = 0; q < 16; ++q) acc[q] = 0.;
  for (int qc = P.cptr[s]; qc < P.cptr[s + 1]; ++qc) {
    const int ch = P.child[qc];
    const int* inv = P.cinv + P.cinv_off[ch];
    __syncthreads();
    if (tid < 64) ri[tid] = rt + tid < fs ? inv[rt + tid] : -1;
    else if (tid < 128) ci[tid - 64] = ct + tid - 64 < fs ? inv[ct + tid - 64] : -1;
    __syncthreads();
    const int nsc = P.sfirst[ch + 1] - P.sfirst[ch];
    const int fc = nsc + (int)(P.rptr[ch + 1] - P.rptr[ch]);
    const double* U = F + P.foff[ch] + nsc + (size_t)nsc * fc;
    const int ia = ri[ii];
    // unconditional loads (all 16 in flight): a missing or upper entry reads the child's lower element at the
    // swapped / clamped indices (finite) and adds it times 0; fma(v, 1, acc) is the rounding of acc + v
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int ib = ci[(tid >> 6) + 4 * q];
      const double m = (ia >= 0 && ib >= 0 && ia >= ib) ? 1. : 0.;
      const int hi = max(max(ia, ib), 0), lo = max(min(ia, ib), 0);
      acc[q] = fma(U[hi + (size_t)lo * fc], m, acc[q]);
    }
  }
  const int i = rt + ii;
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int j = ct + (tid >> 6) + 4 * q;
    if (i < fs && j < fs && i >= j) F[P.foff[s] + i + (size_t)j * fs] = acc[q];
  }
}

__global__ void __launch_bounds__(256) chol_asm_entries_kernel(const CholColTask* __restrict__ tasks, int64_t t0,
                                                               DevPlan P, double* __restrict__ F,
                                                               const int64_t* __restrict__ ecol,
                                                               const int64_t* __restrict__ eoff,
                                                               const double* __restrict__ aval,
                                                               const double* __restrict__ W) {
  const CholColTask tk = tasks[t0 + blockIdx.x];
  const int sf = P.sfirst[tk.s];
  const int64_t e0 = ecol[sf + tk.c0], e1 = ecol[sf + tk.c1];
  for (int64_t e = e0 + threadIdx.x; e < e1; e += 256) F[eoff[e]] += aval[e];
  if (W != nullptr) {   // the diagonal leads each column's entries
    __syncthreads();
    for (int j = tk.c0 + threadIdx.x; j < tk.c1; j += 256) F[eoff[ecol[sf + j]]] += W[P.perm[sf + j]];
  }
}

// ---- split-K reduction: C = beta C + alpha sum of the P slices (64 x 64, ld 64)
__global__ void __launch_bounds__(256) chol_reduce_kernel(const CholReduceTask* __restrict__ tasks, int64_t t0,
                                                          Bufs bufs) {
  const CholReduceTask r = tasks[t0 + blockIdx.x];
  double* C = bufs.p[r.bufc] + r.c;
  const double* Pb = bufs.p[kCbP] + r.p;
  // the 16 elements' C reads issued together, then 16 partial loads in flight per slice (slice order kept per element)
  double cv[16], sv[16];
#pragma unroll
  for (int u = 0; u < 16; ++u) {
    const int e = threadIdx.x + 256 * u, i = e & 63, j = e >> 6;
    sv[u] = 0.;
    cv[u] = r.beta == 0. ? 0. : C[min(i, r.M - 1) + (size_t)min(j, r.N - 1) * r.ldc];
  }
  for (int q = 0; q < r.nslices; ++q) {
    const double* Pq = Pb + (size_t)q * r.pstride + threadIdx.x;
#pragma unroll
    for (int u = 0; u < 16; ++u) sv[u] += Pq[256 * u];
  }
#pragma unroll
  for (int u = 0; u < 16; ++u) {
    const int e = threadIdx.x + 256 * u, i = e & 63, j = e >> 6;
    if (i < r.M && j < r.N)
      C[i + (size_t)j * r.ldc] = (r.beta == 0. ? 0. : r.beta * cv[u]) + r.alpha * sv[u];
  }
}

// ---- one 64 x 64 diagonal block: L and W = L^-1 by four waves. Lane r of wave w holds row r of the block
// at the columns x = 4k + w (L) and column r of W at the rows x = 4k + w. Step j: the wave owning column
// j takes the pivot from lane j, scales its column (divisions, as the LLT) and its W row j, publishes
// l_x = L[x][j] and W[j][r] to LDS; after one barrier every wave applies them to its columns of the
// trailing matrix (A[r][x] -= l_r l_x) and its rows of W (W[x][r] -= l_x W[j][r]). The padding of a
// partial block (ib < 64) is the identity.
__global__ void __launch_bounds__(256) chol_diag_kernel(const CholDiagTask* __restrict__ tasks, int64_t t0,
                                                        double* __restrict__ F, double* __restrict__ Wd,
                                                        int* __restrict__ info) {
  const CholDiagTask tk = tasks[t0 + blockIdx.x];
  double* A = F + tk.c;
  const int ld = tk.ld, ib = tk.ib;
  const int r = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  __shared__ double lsh[2][64];
  __shared__ double wsh[2][64];
  double row[16], wc[16];
  const int rr = min(r, ib - 1);
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int x = 4 * k + w;
    const double v = A[rr + (size_t)min(x, ib - 1) * ld];
    row[k] = (r < ib && x < ib) ? (x <= r ? v : 0.) : (r == x ? 1. : 0.);
    wc[k] = (x == r) ? 1. : 0.;
  }
  bool bad = false;
#pragma unroll
  for (int j = 0; j < 64; ++j) {
    const int kj = j >> 2;
    if (w == (j & 3)) {
      const int lo = __builtin_amdgcn_readlane(__double2loint(row[kj]), j);
      const int hi = __builtin_amdgcn_readlane(__double2hiint(row[kj]), j);
      const double p = __hiloint2double(hi, lo);
      bad = bad || !(p > 0.);
      // y = 1 / sqrt(p) by the hardware estimate and two Newton steps, d = p y; the column and W row scaled by y
      // (multiplies instead of a square root and two IEEE divisions on the pivot chain)
      const double ps = p > 0. ? p : 1., h = 0.5 * ps;
      double y = __builtin_amdgcn_rsq(ps);
      y = y * fma(-h * y, y, 1.5);
      y = y * fma(-h * y, y, 1.5);
      const double d = ps * y;
      const double l = r > j ? row[kj] * y : (r == j ? d : 0.);
      row[kj] = l;
      wc[kj] = wc[kj] * y;   // W[j][r] final
      lsh[j & 1][r] = r > j ? l : 0.;
      wsh[j & 1][r] = wc[kj];
    }
    __syncthreads();
    const double lr = lsh[j & 1][r], wjr = wsh[j & 1][r];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      if (4 * k + 3 <= j) continue;   // every column / row of register k is <= j
      const double lx = lsh[j & 1][4 * k + w];   // 0 for x <= j
      row[k] = fma(-lr, lx, row[k]);
      wc[k] = fma(-lx, wjr, wc[k]);
    }
  }
  if (bad && r == 0) atomicAdd(info, 1);
  double* W = Wd + tk.w;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int x = 4 * k + w;
    if (r < ib && x < ib) {
      if (x <= r) A[r + (size_t)x * ld] = row[k];
      W[x + (size_t)r * 64] = wc[k];   // W[x][r] (zero above the diagonal)
    }
  }
}

// ---- batched GEMM tile: C = alpha op(A) op(B) + beta C, one task per workgroup
constexpr int GT = 64, GK = 16;   // GK = 32 measured slower (2 waves per SIMD instead of 4)
// the tile's epilogue: the beta C reads issued together (clamped addresses, unconditional), then the masked stores
// (one memory round trip per tile instead of one per element)
__device__ __forceinline__ void chol_gemm_epilogue(const CholGemmTask& g, double* C, const double4_t (&acc)[2][2], int wm,
                                                   int wn, int lane) {
  const bool lower = g.flags & kCgLower;
  double prev[2][2][4];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int rg = 0; rg < 4; ++rg) {
        const int i = min(wm + a * 16 + (lane >> 4) + 4 * rg, g.M - 1);
        const int j = min(wn + b * 16 + (lane & 15), g.N - 1);
        prev[a][b][rg] = g.beta == 0. ? 0. : C[(size_t)i + (size_t)j * g.ldc];
      }
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int rg = 0; rg < 4; ++rg) {
        const int i = wm + a * 16 + (lane >> 4) + 4 * rg;
        const int j = wn + b * 16 + (lane & 15);
        const double v = (g.beta == 0. ? 0. : g.beta * prev[a][b][rg]) + g.alpha * acc[a][b][rg];
        if (i < g.M && j < g.N && !(lower && i - j + g.doff < 0)) C[(size_t)i + (size_t)j * g.ldc] = v;
      }
}
__global__ void __launch_bounds__(256) chol_gemm_kernel(const CholGemmTask* __restrict__ tasks, int64_t t0, Bufs bufs) {
  const CholGemmTask g = tasks[t0 + blockIdx.x];
  if (g.M <= 0 || g.N <= 0) return;   // empty tile (the clamped loads below need M, N >= 1)
  const double* A = bufs.p[(g.flags >> 4) & 7] + g.a;
  const double* B = bufs.p[(g.flags >> 7) & 7] + g.b;
  double* C = bufs.p[(g.flags >> 10) & 7] + g.c;
  const bool ta = g.flags & kCgTA, tb = g.flags & kCgTB;
  __shared__ double As[2][GK][GT + 1];
  __shared__ double Bs[2][GK][GT + 1];
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = (wave >> 1) * 32, wn = (wave & 1) * 32;
  double4_t acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[a][b] = (double4_t){0., 0., 0., 0.};
  constexpr int EPT = GK * GT / 256;
  double ra[EPT], rb[EPT];
  // branch-free tile loads: out-of-range elements read a clamped (valid, finite) address and are multiplied by 0
  // when stored to LDS (a product, not a select, so the loads stay unconditional; the product after the MFMAs of the
  // current tile, so the loads of the next tile are in flight meanwhile)
  unsigned okA = 0, okB = 0;
  auto load = [&](int kk) {
    okA = okB = 0;
#pragma unroll
    for (int e = 0; e < EPT; ++e) {
      const int idx = tid + e * 256;
      int i, k;
      if (ta) { k = idx & (GK - 1); i = idx / GK; } else { i = idx & (GT - 1); k = idx / GT; }
      const int gk = kk + k;
      const int ic = min(i, g.M - 1), kc = min(gk, g.K - 1);
      ra[e] = ta ? A[(size_t)kc + (size_t)ic * g.lda] : A[(size_t)ic + (size_t)kc * g.lda];
      okA |= (i < g.M && gk < g.K) ? 1u << e : 0u;
      int j, kb;
      if (tb) { j = idx & (GT - 1); kb = idx / GT; } else { kb = idx & (GK - 1); j = idx / GK; }
      const int gkb = kk + kb;
      const int jc = min(j, g.N - 1), kbc = min(gkb, g.K - 1);
      rb[e] = tb ? B[(size_t)jc + (size_t)kbc * g.ldb] : B[(size_t)kbc + (size_t)jc * g.ldb];
      okB |= (j < g.N && gkb < g.K) ? 1u << e : 0u;
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int e = 0; e < EPT; ++e) {
      const int idx = tid + e * 256;
      int i, k;
      if (ta) { k = idx & (GK - 1); i = idx / GK; } else { i = idx & (GT - 1); k = idx / GT; }
      As[buf][k][i] = ra[e] * ((okA >> e) & 1u ? 1. : 0.);
      int j, kb;
      if (tb) { j = idx & (GT - 1); kb = idx / GT; } else { kb = idx & (GK - 1); j = idx / GK; }
      Bs[buf][kb][j] = rb[e] * ((okB >> e) & 1u ? 1. : 0.);
    }
  };
  if (g.K > 0) {
    load(0);
    store(0);
  }
  __syncthreads();
  int buf = 0;
  for (int kk = 0; kk < g.K; kk += GK) {
    const bool more = kk + GK < g.K;
    if (more) load(kk + GK);
#pragma unroll
    for (int k4 = 0; k4 < GK; k4 += 4) {
      const int kl = k4 + (lane >> 4);
      const double a0 = As[buf][kl][wm + (lane & 15)], a1 = As[buf][kl][wm + 16 + (lane & 15)];
      const double b0 = Bs[buf][kl][wn + (lane & 15)], b1 = Bs[buf][kl][wn + 16 + (lane & 15)];
      acc[0][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b0, acc[0][0], 0, 0, 0);
      acc[0][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b1, acc[0][1], 0, 0, 0);
      acc[1][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b0, acc[1][0], 0, 0, 0);
      acc[1][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b1, acc[1][1], 0, 0, 0);
    }
    if (more) store(buf ^ 1);
    __syncthreads();
    buf ^= 1;
  }
  chol_gemm_epilogue(g, C, acc, wm, wn, lane);
}

// ---- the same tile product for tasks with K <= 64 in launches of few tiles (the solves' per-block steps, the
// small fronts): all of op(A) (64 x K) and op(B) (K x 64) are loaded at once (16 + 16 loads in flight per thread),
// one barrier, then the K / 4 MFMA steps; a lone tile costs one memory round trip instead of one per K step of 16.
// Same k order through the MFMA as chol_gemm_kernel, so the same bits.
constexpr int kSmallGemmTiles = 2048;
__global__ void __launch_bounds__(256) chol_gemm_k64_kernel(const CholGemmTask* __restrict__ tasks, int64_t t0, Bufs bufs) {
  const CholGemmTask g = tasks[t0 + blockIdx.x];
  if (g.M <= 0 || g.N <= 0) return;   // empty tile (the clamped loads below need M, N >= 1)
  const double* A = bufs.p[(g.flags >> 4) & 7] + g.a;
  const double* B = bufs.p[(g.flags >> 7) & 7] + g.b;
  double* C = bufs.p[(g.flags >> 10) & 7] + g.c;
  const bool ta = g.flags & kCgTA, tb = g.flags & kCgTB;
  __shared__ double As[64][GT + 1];
  __shared__ double Bs[64][GT + 1];
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = (wave >> 1) * 32, wn = (wave & 1) * 32;
  constexpr int EPT = 64 * GT / 256;
  double ra[EPT], rb[EPT];
  unsigned okA = 0, okB = 0;
  // K = 0 (an empty product): every element is masked; the clamped loads then read element 0 of the operands,
  // which is avoided by pointing them at C's (valid) tile origin instead
  const int Kc = max(g.K, 1);
  const double* Ar = g.K > 0 ? A : C;
  const double* Br = g.K > 0 ? B : C;
  const int lda = g.K > 0 ? g.lda : 0, ldb = g.K > 0 ? g.ldb : 0;
#pragma unroll
  for (int e = 0; e < EPT; ++e) {
    const int idx = tid + e * 256;
    int i, k;
    if (ta) { k = idx & 63; i = idx >> 6; } else { i = idx & (GT - 1); k = idx / GT; }
    const int ic = g.K > 0 ? min(i, g.M - 1) : 0, kc = min(k, Kc - 1);
    ra[e] = ta ? Ar[(size_t)kc + (size_t)ic * lda] : Ar[(size_t)ic + (size_t)kc * lda];
    okA |= (i < g.M && k < g.K) ? 1u << e : 0u;
    int j, kb;
    if (tb) { j = idx & (GT - 1); kb = idx / GT; } else { kb = idx & 63; j = idx >> 6; }
    const int jc = g.K > 0 ? min(j, g.N - 1) : 0, kbc = min(kb, Kc - 1);
    rb[e] = tb ? Br[(size_t)jc + (size_t)kbc * ldb] : Br[(size_t)kbc + (size_t)jc * ldb];
    okB |= (j < g.N && kb < g.K) ? 1u << e : 0u;
  }
#pragma unroll
  for (int e = 0; e < EPT; ++e) {
    const int idx = tid + e * 256;
    int i, k;
    if (ta) { k = idx & 63; i = idx >> 6; } else { i = idx & (GT - 1); k = idx / GT; }
    As[k][i] = ra[e] * ((okA >> e) & 1u ? 1. : 0.);
    int j, kb;
    if (tb) { j = idx & (GT - 1); kb = idx / GT; } else { kb = idx & 63; j = idx >> 6; }
    Bs[kb][j] = rb[e] * ((okB >> e) & 1u ? 1. : 0.);
  }
  __syncthreads();
  double4_t acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[a][b] = (double4_t){0., 0., 0., 0.};
  const int kmax = (g.K + 3) & ~3;
  for (int k4 = 0; k4 < kmax; k4 += 4) {
    const int kl = k4 + (lane >> 4);
    const double a0 = As[kl][wm + (lane & 15)], a1 = As[kl][wm + 16 + (lane & 15)];
    const double b0 = Bs[kl][wn + (lane & 15)], b1 = Bs[kl][wn + 16 + (lane & 15)];
    acc[0][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b0, acc[0][0], 0, 0, 0);
    acc[0][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b1, acc[0][1], 0, 0, 0);
    acc[1][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b0, acc[1][0], 0, 0, 0);
    acc[1][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b1, acc[1][1], 0, 0, 0);
  }
  chol_gemm_epilogue(g, C, acc, wm, wn, lane);
}

// ---- selected inverse: S_RR of supernode s from its parent's front (both triangles), R columns [c0, c1)
__global__ void __launch_bounds__(256) chol_gather_s_kernel(const CholColTask* __restrict__ tasks, int64_t t0,
                                                            DevPlan P, double* __restrict__ S) {
  const CholColTask tk = tasks[t0 + blockIdx.x];
  const int s = tk.s, p = P.sparent[s];
  const int ns = P.sfirst[s + 1] - P.sfirst[s];
  const int nr = (int)(P.rptr[s + 1] - P.rptr[s]);
  const int fs = ns + nr;
  const int fp = (P.sfirst[p + 1] - P.sfirst[p]) + (int)(P.rptr[p + 1] - P.rptr[p]);
  const int* rel = P.rel + P.rptr[s];
  double* Ss = S + P.foff[s];
  const double* Sp = S + P.foff[p];
  // the position map in LDS (one pass), then per column one gather per element with four elements in flight per
  // thread (the round-5 loop re-read the map from global memory before every gather: two dependent round trips)
  constexpr int kRelLds = 6144;
  __shared__ int rel_s[kRelLds];
  const bool in_lds = nr <= kRelLds;
  if (in_lds)
    for (int a = threadIdx.x; a < nr; a += 256) rel_s[a] = rel[a];
  __syncthreads();
  const int* rm = in_lds ? rel_s : rel;
  for (int b = tk.c0; b < tk.c1; ++b) {
    const double* src = Sp + (size_t)rel[b] * fp;
    double* dst = Ss + ns + (size_t)(ns + b) * fs;
    for (int a0 = threadIdx.x; a0 < nr; a0 += 1024) {
      double v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int a = a0 + 256 * u;
        v[u] = a < nr ? src[rm[a]] : 0.;
      }
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (a0 + 256 * u < nr) dst[a0 + 256 * u] = v[u];
    }
  }
}

// S[j, r] = S[r, j] for front columns j in [c0, c1) and rows r > j of the 64-row tile at pad (LDS-transposed)
__global__ void __launch_bounds__(256) chol_mirror_kernel(const CholColTask* __restrict__ tasks, int64_t t0,
                                                          DevPlan P, double* __restrict__ S) {
  const CholColTask tk = tasks[t0 + blockIdx.x];
  const int s = tk.s, R0 = tk.pad;
  const int ns = P.sfirst[s + 1] - P.sfirst[s];
  const int fs = ns + (int)(P.rptr[s + 1] - P.rptr[s]);
  double* Ss = S + P.foff[s];
  __shared__ double T[64][65];
  const int nc = tk.c1 - tk.c0;
  const int tid = threadIdx.x;
  for (int e = tid; e < 64 * 64; e += 256) {
    const int rr = e & 63, cc = e >> 6;
    if (cc < nc && R0 + rr < fs) T[rr][cc] = Ss[(R0 + rr) + (size_t)(tk.c0 + cc) * fs];
  }
  __syncthreads();
  for (int e = tid; e < 64 * 64; e += 256) {
    const int cc = e & 63, rr = e >> 6;
    const int row = R0 + rr, col = tk.c0 + cc;
    if (cc < nc && row < fs && row > col) Ss[col + (size_t)row * fs] = T[rr][cc];
  }
}

// ---- solves: front vectors V_s (fs x t, ld fs)
struct SolveArgs {
  double* V;
  const int64_t* vofs;
  const double* b;   // input, matrix labels, n x t (ld n)
  double* X;         // global X, matrix labels, n x t (ld n)
  int t;
  double* XS;        // t = 1 fused forward steps: the block results (V's layout)
  const double* F;   // the factor's fronts
  const double* Wd;  // diagonal-block inverses
  const int64_t* woff;
};

constexpr int kSolveColGroup = 4;   // right-hand sides per block of the solve's assembly / gather / scatter passes

__global__ void __launch_bounds__(256) chol_asmv_kernel(const CholColTask* __restrict__ tasks, int64_t t0, DevPlan P,
                                                        SolveArgs a) {
  const CholColTask tk = tasks[t0 + blockIdx.x];
  const int s = tk.s;
  const int sf = P.sfirst[s], ns = P.sfirst[s + 1] - sf;
  const int fs = ns + (int)(P.rptr[s + 1] - P.rptr[s]);
  double* V = a.V + a.vofs[s];
  // columns [k0, k1) of this block (blockIdx.y: column group of kSolveColGroup right-hand sides)
  const int k0 = blockIdx.y * kSolveColGroup, k1 = min(a.t, k0 + kSolveColGroup);
  for (int k = k0; k < k1; ++k)
    for (int r = threadIdx.x; r < fs; r += 256)
      V[r + (size_t)k * fs] = r < ns ? a.b[P.perm[sf + r] + (size_t)k * P.n] : 0.;
  for (int q = P.cptr[s]; q < P.cptr[s + 1]; ++q) {
    __syncthreads();
    const int ch = P.child[q];
    const int nsc = P.sfirst[ch + 1] - P.sfirst[ch];
    const int nrc = (int)(P.rptr[ch + 1] - P.rptr[ch]);
    const int fc = nsc + nrc;
    const int* rel = P.rel + P.rptr[ch];
    const double* Vc = a.V + a.vofs[ch];
    for (int k = k0; k < k1; ++k)
      for (int i = threadIdx.x; i < nrc; i += 256) V[rel[i] + (size_t)k * fs] += Vc[nsc + i + (size_t)k * fc];
  }
}

__global__ void __launch_bounds__(256) chol_gather_x_kernel(const CholColTask* __restrict__ tasks, int64_t t0,
                                                            DevPlan P, SolveArgs a) {
  const CholColTask tk = tasks[t0 + blockIdx.x];
  const int s = tk.s;
  const int ns = P.sfirst[s + 1] - P.sfirst[s];
  const int nr = (int)(P.rptr[s + 1] - P.rptr[s]);
  const int fs = ns + nr;
  const int* R = P.rows + P.rptr[s];
  double* V = a.V + a.vofs[s];
  const int k0 = blockIdx.y * kSolveColGroup, k1 = min(a.t, k0 + kSolveColGroup);
  for (int k = k0; k < k1; ++k)
    for (int i = tk.c0 + threadIdx.x; i < tk.c1; i += 256) V[ns + i + (size_t)k * fs] = a.X[P.perm[R[i]] + (size_t)k * P.n];
}

__global__ void __launch_bounds__(256) chol_scatter_x_kernel(const CholColTask* __restrict__ tasks, int64_t t0,
                                                             DevPlan P, SolveArgs a) {
  const CholColTask tk = tasks[t0 + blockIdx.x];
  const int s = tk.s;
  const int sf = P.sfirst[s], ns = P.sfirst[s + 1] - sf;
  const int fs = ns + (int)(P.rptr[s + 1] - P.rptr[s]);
  const double* V = a.V + a.vofs[s];
  const int k0 = blockIdx.y * kSolveColGroup, k1 = min(a.t, k0 + kSolveColGroup);
  for (int k = k0; k < k1; ++k)
    for (int i = tk.c0 + threadIdx.x; i < tk.c1; i += 256) a.X[P.perm[sf + i] + (size_t)k * P.n] = V[i + (size_t)k * fs];
}

__global__ void __launch_bounds__(256) chol_load_v_kernel(const CholColTask* __restrict__ tasks, int64_t t0, DevPlan P,
                                                          SolveArgs a) {
  const CholColTask tk = tasks[t0 + blockIdx.x];
  const int s = tk.s;
  const int sf = P.sfirst[s], ns = P.sfirst[s + 1] - sf;
  const int fs = ns + (int)(P.rptr[s + 1] - P.rptr[s]);
  double* V = a.V + a.vofs[s];
  const int k0 = blockIdx.y * kSolveColGroup, k1 = min(a.t, k0 + kSolveColGroup);
  for (int k = k0; k < k1; ++k)
    for (int i = tk.c0 + threadIdx.x; i < tk.c1; i += 256) V[i + (size_t)k * fs] = a.b[P.perm[sf + i] + (size_t)k * P.n];
}

__device__ __forceinline__ double readlane_f64(double v, int l) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), l);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), l);
  return __hiloint2double(hi, lo);
}

// ---- t = 1, one block step of a large level's forward sweep in one launch: every wave (task {s, k, rt}) forms
// x_b = W_b v_b itself (lane i: sum over j of W[i][j] v_j, j ascending: fsolve1's order; W_b is zero above the
// diagonal and beyond ib), the first row tile's wave stores it to XS (V[j0:j0+ib] is still being read by the other
// waves), then rows rt + lane: v_r -= sum_j L[r][j0 + j] x_j (j ascending, as fsolve1)
__global__ void __launch_bounds__(64) chol_fwd_vec_kernel(const CholColTask* __restrict__ tasks, int64_t t0, DevPlan P,
                                                          SolveArgs a) {
  const CholColTask tk = tasks[t0 + blockIdx.x];
  const int s = tk.s, k = tk.c0, rt = tk.c1;
  const int sf = P.sfirst[s], ns = P.sfirst[s + 1] - sf;
  const int fs = ns + (int)(P.rptr[s + 1] - P.rptr[s]);
  const int j0 = 64 * k, ib = min(64, ns - j0), r0 = j0 + ib;
  double* V = a.V + a.vofs[s];
  const int lane = threadIdx.x;
  const double vl = lane < ib ? V[j0 + min(lane, ib - 1)] : 0.;
  const double* W = a.Wd + a.woff[s] + (int64_t)k * 4096;
  double x = 0.;
#pragma unroll
  for (int j = 0; j < 64; ++j) x = fma(W[lane + 64 * j], readlane_f64(vl, j), x);
  if (rt == r0 && lane < ib) a.XS[a.vofs[s] + j0 + lane] = x;
  const int r = rt + lane;
  if (rt >= fs) return;
  const int rc = min(r, fs - 1);
  const double* Lr = a.F + P.foff[s] + rc + (size_t)j0 * fs;
  double acc = V[rc];
#pragma unroll
  for (int j = 0; j < 64; ++j)   // x_j = 0 for j >= ib (those columns read column ib - 1: finite, times 0)
    acc = fma(-Lr[(size_t)min(j, ib - 1) * fs], readlane_f64(x, j), acc);
  if (r < fs) V[r] = acc;
}

// ---- t = 1 backward block step of a large level: partial sums of L[chunk, b]^T v[chunk] over 256-row chunks (lane =
// row, wave w = columns w + 4 q, four rows per lane in flight; wave-reduced), then per supernode the reduce in chunk
// order and x_b = W_b^T v_b (lane i: sum over j of W[j][i] v_j, j ascending: bsolve1's order)
__global__ void __launch_bounds__(256) chol_bwd_vec_part_kernel(const CholColTask* __restrict__ tasks, int64_t t0,
                                                                DevPlan P, SolveArgs a, double* __restrict__ part) {
  const CholColTask tk = tasks[t0 + blockIdx.x];
  const int s = tk.s, k = tk.c0, kc = tk.c1, slot = tk.pad;
  const int sf = P.sfirst[s], ns = P.sfirst[s + 1] - sf;
  const int fs = ns + (int)(P.rptr[s + 1] - P.rptr[s]);
  const int j0 = 64 * k, ib = min(64, ns - j0), r0 = j0 + ib;
  const int rs = r0 + 256 * kc, re = min(rs + 256, fs);
  const double* V = a.V + a.vofs[s];
  const double* L = a.F + P.foff[s] + (size_t)j0 * fs;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  double acc[16];
#pragma unroll
  for (int q = 0; q < 16; ++q) acc[q] = 0.;
  double vr[4];
  int rc[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int r = rs + 64 * u + lane;
    rc[u] = min(r, re - 1);
    vr[u] = r < re ? V[rc[u]] : 0.;
  }
#pragma unroll
  for (int u = 0; u < 4; ++u)
#pragma unroll
    for (int q = 0; q < 16; ++q) acc[q] = fma(L[rc[u] + (size_t)min(w + 4 * q, ib - 1) * fs], vr[u], acc[q]);
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    double v = acc[q];
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    if (lane == 0) part[(size_t)slot * 64 + w + 4 * q] = v;
  }
}

__global__ void __launch_bounds__(64) chol_bwd_vec_fin_kernel(const CholColTask* __restrict__ tasks, int64_t t0,
                                                              DevPlan P, SolveArgs a, const double* __restrict__ part) {
  const CholColTask tk = tasks[t0 + blockIdx.x];
  const int s = tk.s, k = tk.c0, nch = tk.c1, slot0 = tk.pad;
  const int ns = P.sfirst[s + 1] - P.sfirst[s];
  const int j0 = 64 * k, ib = min(64, ns - j0);
  double* V = a.V + a.vofs[s];
  const int lane = threadIdx.x;
  double v = lane < ib ? V[j0 + min(lane, ib - 1)] : 0.;
  double d = 0.;
  for (int c = 0; c < nch; ++c) d += part[(size_t)(slot0 + c) * 64 + lane];
  v = lane < ib ? v - d : 0.;
  const double* W = a.Wd + a.woff[s] + (int64_t)k * 4096;
  double x = 0.;
#pragma unroll
  for (int j = 0; j < 64; ++j) x = fma(W[j + 64 * lane], readlane_f64(v, j), x);
  if (lane < ib) V[j0 + lane] = x;
}

__global__ void __launch_bounds__(256) chol_copy_xs_kernel(const CholColTask* __restrict__ tasks, int64_t t0, SolveArgs a) {
  const CholColTask tk = tasks[t0 + blockIdx.x];
  const int64_t o = a.vofs[tk.s];
  for (int i = tk.c0 + threadIdx.x; i < tk.c1; i += 256) a.V[o + i] = a.XS[o + i];
}

// ---- single right-hand side: one workgroup per supernode of a level runs its whole panel (the forward
// sweep assembles its front vector from b and the children, then per 64-column block x_b = W_b v_b and
// v[below] -= L[below, b] x_b; the backward sweep gathers x at its rows R_s, then per block from the last
// v_b -= L[below, b]^T v[below] (one wave per 16 columns, wave-reduced) and x_b = W_b^T v_b), so a solve is
// two launches per tree level instead of one per block step.
struct Solve1Args {
  const int* lvl_sup;
  int l0;
  const double* F;
  const double* Wd;
  const int64_t* woff;
  double* V;
  const int64_t* vofs;
  const double* b;
  double* x;
};

__global__ void __launch_bounds__(256) chol_fsolve1_kernel(DevPlan P, Solve1Args a) {
  const int s = a.lvl_sup[a.l0 + blockIdx.x];
  const int sf = P.sfirst[s], ns = P.sfirst[s + 1] - sf;
  const int fs = ns + (int)(P.rptr[s + 1] - P.rptr[s]);
  double* V = a.V + a.vofs[s];
  const double* L = a.F + P.foff[s];
  const int tid = threadIdx.x;
  for (int r = tid; r < fs; r += 256) V[r] = r < ns ? a.b[P.perm[sf + r]] : 0.;
  for (int q = P.cptr[s]; q < P.cptr[s + 1]; ++q) {
    __syncthreads();
    const int ch = P.child[q];
    const int nsc = P.sfirst[ch + 1] - P.sfirst[ch];
    const int nrc = (int)(P.rptr[ch + 1] - P.rptr[ch]);
    const int* rel = P.rel + P.rptr[ch];
    const double* Vc = a.V + a.vofs[ch] + nsc;
    for (int i = tid; i < nrc; i += 256) V[rel[i]] += Vc[i];
  }
  __shared__ double vb[64], xb[64];
  const int nblk = (ns + 63) / 64;
  for (int k = 0; k < nblk; ++k) {
    const int j0 = 64 * k, ib = min(64, ns - j0);
    __syncthreads();
    if (tid < 64) vb[tid] = tid < ib ? V[j0 + tid] : 0.;
    __syncthreads();
    if (tid < ib) {
      const double* W = a.Wd + a.woff[s] + (int64_t)k * 4096;
      double x = 0.;
      for (int j = 0; j <= tid; ++j) x = fma(W[tid + j * 64], vb[j], x);
      xb[tid] = x;
      V[j0 + tid] = x;
    } else if (tid < 64) {
      xb[tid] = 0.;
    }
    __syncthreads();
    // all 64 column loads of a row in flight (columns >= ib read column ib - 1, times x_j = 0)
    for (int r = j0 + ib + tid; r < fs; r += 256) {
      double acc = V[r];
      const double* Lr = L + r + (size_t)j0 * fs;
#pragma unroll
      for (int j = 0; j < 64; ++j) acc = fma(-Lr[(size_t)min(j, ib - 1) * fs], xb[j], acc);
      V[r] = acc;
    }
  }
}

__global__ void __launch_bounds__(256) chol_bsolve1_kernel(DevPlan P, Solve1Args a) {
  const int s = a.lvl_sup[a.l0 + blockIdx.x];
  const int sf = P.sfirst[s], ns = P.sfirst[s + 1] - sf;
  const int nr = (int)(P.rptr[s + 1] - P.rptr[s]);
  const int fs = ns + nr;
  double* V = a.V + a.vofs[s];
  const double* L = a.F + P.foff[s];
  const int* R = P.rows + P.rptr[s];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  for (int i = tid; i < nr; i += 256) V[ns + i] = a.x[P.perm[R[i]]];
  __shared__ double vb[64], dsum[64];
  const int nblk = (ns + 63) / 64;
  for (int k = nblk - 1; k >= 0; --k) {
    const int j0 = 64 * k, ib = min(64, ns - j0), r0 = j0 + ib;
    __syncthreads();
    double acc[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) acc[q] = 0.;
    // four rows per lane per iteration (64 loads in flight; rows past fs read row fs - 1 times v = 0, columns
    // >= ib column ib - 1 times 0); each acc[q] still sums its rows in ascending order
    for (int rb = r0; rb < fs; rb += 256) {
      double vr[4];
      const double* Lr[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int r = rb + 64 * u + lane;
        vr[u] = r < fs ? V[min(r, fs - 1)] : 0.;
        Lr[u] = L + min(r, fs - 1) + (size_t)j0 * fs;
      }
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          const int j = w + 4 * q;
          const double l = Lr[u][(size_t)min(j, ib - 1) * fs] * (j < ib ? 1. : 0.);
          acc[q] = fma(l, vr[u], acc[q]);
        }
    }
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      double v = acc[q];
      for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
      if (lane == 0) dsum[w + 4 * q] = v;
    }
    __syncthreads();
    if (tid < 64) vb[tid] = tid < ib ? V[j0 + tid] - dsum[tid] : 0.;
    __syncthreads();
    if (tid < ib) {
      const double* W = a.Wd + a.woff[s] + (int64_t)k * 4096;
      double x = 0.;
      for (int j = tid; j < ib; ++j) x = fma(W[j + tid * 64], vb[j], x);
      V[j0 + tid] = x;
    }
  }
  __syncthreads();
  for (int i = tid; i < ns; i += 256) a.x[P.perm[sf + i]] = V[i];
}

// ---- reductions (two passes, fixed order)
constexpr int kRedBlocks = 1024;
// part[blk * 4 + q]: q = 0: sum 2 log L_gg; 1: sum_e aval S; 2: sum_diag aval S; 3: sum_e daval S;
// (diagonal part of daval in part2[blk])
__global__ void __launch_bounds__(256) chol_logdet_kernel(int n, const int64_t* __restrict__ dpos,
                                                          const double* __restrict__ F, double* __restrict__ part) {
  __shared__ double red[256];
  double s = 0.;
  for (int g = blockIdx.x * 256 + threadIdx.x; g < n; g += gridDim.x * 256) s += 2. * log(F[dpos[g]]);
  red[threadIdx.x] = s;
  __syncthreads();
  for (int off = 128; off > 0; off >>= 1) {
    if ((int)threadIdx.x < off) red[threadIdx.x] += red[threadIdx.x + off];
    __syncthreads();
  }
  if (threadIdx.x == 0) part[blockIdx.x] = red[0];
}

__global__ void __launch_bounds__(256) chol_trace_kernel(int n, const int64_t* __restrict__ ecol,
                                                         const int64_t* __restrict__ eoff,
                                                         const double* __restrict__ aval,
                                                         const double* __restrict__ daval,
                                                         const double* __restrict__ S, double* __restrict__ part) {
  // per column g: off-diagonal entries count twice (symmetric), the diagonal (first entry) once
  __shared__ double red[2][256];
  double s0 = 0., s1 = 0.;
  for (int g = blockIdx.x * 256 + threadIdx.x; g < n; g += gridDim.x * 256) {
    const int64_t e0 = ecol[g], e1 = ecol[g + 1];
    for (int64_t e = e0; e < e1; ++e) {
      const double w = e == e0 ? 1. : 2.;
      const double sv = S[eoff[e]];
      s0 += w * aval[e] * sv;
      if (daval != nullptr) s1 += w * daval[e] * sv;
    }
  }
  red[0][threadIdx.x] = s0;
  red[1][threadIdx.x] = s1;
  __syncthreads();
  for (int off = 128; off > 0; off >>= 1) {
    if ((int)threadIdx.x < off) {
      red[0][threadIdx.x] += red[0][threadIdx.x + off];
      red[1][threadIdx.x] += red[1][threadIdx.x + off];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    part[2 * blockIdx.x] = red[0][0];
    part[2 * blockIdx.x + 1] = red[1][0];
  }
}

__global__ void __launch_bounds__(256) chol_sum_parts_kernel(const double* __restrict__ part, int nblk, int stride,
                                                             int q, double* __restrict__ out) {
  __shared__ double red[256];
  double s = 0.;
  for (int b = threadIdx.x; b < nblk; b += 256) s += part[(size_t)b * stride + q];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int off = 128; off > 0; off >>= 1) {
    if ((int)threadIdx.x < off) red[threadIdx.x] += red[threadIdx.x + off];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[q] = red[0];
}

__global__ void __launch_bounds__(256) chol_diag_s_kernel(int n, const int64_t* __restrict__ dpos,
                                                          const int* __restrict__ perm, const double* __restrict__ S,
                                                          double* __restrict__ diag) {
  const int g = blockIdx.x * 256 + threadIdx.x;
  if (g < n) diag[perm[g]] = S[dpos[g]];
}

template <typename T>
void upload(DevBuf<T>& d, const std::vector<T>& h) {
  d.alloc(std::max<size_t>(h.size(), 1));
  if (!h.empty()) HIP_CHECK(hipMemcpy(d.get(), h.data(), sizeof(T) * h.size(), hipMemcpyHostToDevice));
}

int grid_for(int64_t n, int per) { return (int)std::max<int64_t>(1, std::min<int64_t>((n + per - 1) / per, 65536)); }

}  // namespace

// ---------------------------------------------------------------------------------------------------
struct SparseCholDev {
  DevBuf<CholGemmTask> gemm;
  DevBuf<CholDiagTask> diag;
  DevBuf<CholColTask> col;
  DevBuf<CholReduceTask> red;
  std::vector<CholOp> ops;
  std::vector<char> k64;   // per op: a GEMM launch of few tiles, all with K <= 64 (chol_gemm_k64_kernel)
  int64_t y_doubles = 0, p_doubles = 0;
  void Upload(const CholSchedule& S) {
    k64.assign(S.ops.size(), 0);
    const char* e = std::getenv("GPBOOST_AMD_CHOL_K64");   // "0": always the K-pipelined form (A/B)
    if (!(e && std::string(e) == "0"))
      for (size_t o = 0; o < S.ops.size(); ++o) {
        const CholOp& op = S.ops[o];
        if (op.type != kOpGemm || op.ntask > kSmallGemmTiles) continue;
        int kmax = 0;
        for (int64_t t = op.task0; t < op.task0 + op.ntask; ++t) kmax = std::max(kmax, S.gemm[t].K);
        k64[o] = kmax <= 64;
      }
    upload(gemm, S.gemm);
    upload(diag, S.diag);
    upload(col, S.col);
    upload(red, S.red);
    ops = S.ops;
    y_doubles = S.y_doubles;
    p_doubles = S.p_doubles;
  }
};

struct SparseChol::Impl {
  SparseCholDev factor, selinv;
  std::map<std::pair<int, int>, std::unique_ptr<SparseCholDev>> solve;   // (t, forward_only)
  std::map<std::pair<int, int>, std::vector<int64_t>> vofs_h;
  std::map<std::pair<int, int>, std::unique_ptr<DevBuf<int64_t>>> vofs_d;
  DevPlan dp{};
  DevBuf<double> V;   // solve scratch
  DevBuf<double> XS;  // t = 1 fused forward steps' block results
};

SparseChol::SparseChol(int n, int m, const int* nbr, int d, const double* X, hipStream_t s)
    : s_(s), n_(n), m_(m), impl_(new Impl) {
  int leaf = 64;
  if (const char* e = std::getenv("GPBOOST_AMD_CHOL_LEAF")) leaf = std::max(1, std::atoi(e));
  chol_analyze(n, m, nbr, d, X, leaf, plan_);
  CholEntries E;
  chol_entry_lists(plan_, m, nbr, E);
  nent_ = E.ecol[n];
  const CholPlan& P = plan_;
  upload(d_perm_, P.perm);
  upload(d_sfirst_, P.sfirst);
  upload(d_rptr_, P.rptr);
  upload(d_rows_, P.rows);
  upload(d_foff_, P.foff);
  upload(d_rel_, P.rel);
  upload(d_cptr_, P.cptr);
  upload(d_child_, P.child);
  upload(d_sparent_, P.sparent);
  upload(d_cinv_off_, P.cinv_off);
  upload(d_cinv_, P.cinv);
  upload(d_ecol_, E.ecol);
  upload(d_eoff_, E.eoff);
  upload(d_ecptr_, E.cptr);
  upload(d_ctr_, E.ctr);
  upload(d_dpos_, E.dpos);
  upload(d_lvl_sup_, P.lvl_sup);
  upload(d_woff_, P.woff);
  {
    std::vector<int64_t> v1(P.nsup + 1, 0);
    for (int s = 0; s < P.nsup; ++s) v1[s + 1] = v1[s] + P.fs(s);
    vofs1_total_ = v1[P.nsup];
    upload(d_vofs1_, v1);
  }
  impl_->factor.Upload(P.factor);
  impl_->selinv.Upload(P.selinv);
  DevPlan& dp = impl_->dp;
  dp.n = n;
  dp.sfirst = d_sfirst_.get();
  dp.rptr = d_rptr_.get();
  dp.rows = d_rows_.get();
  dp.foff = d_foff_.get();
  dp.rel = d_rel_.get();
  dp.cptr = d_cptr_.get();
  dp.child = d_child_.get();
  dp.sparent = d_sparent_.get();
  dp.perm = d_perm_.get();
  dp.cinv_off = d_cinv_off_.get();
  dp.cinv = d_cinv_.get();
  d_F_.alloc(std::max<int64_t>(P.front_doubles, 1));
  d_Wd_.alloc(std::max<int64_t>(P.woff[P.nsup], 1));
  d_aval_.alloc(std::max<int64_t>(nent_, 1));
  d_daval_.alloc(std::max<int64_t>(nent_, 1));
  d_info_.alloc(1);
  d_red_.alloc((size_t)2 * kRedBlocks + 8);
  HIP_CHECK(hipMemset(d_Wd_.get(), 0, sizeof(double) * d_Wd_.size()));
  HIP_CHECK(hipEventCreate(&ev0_));
  HIP_CHECK(hipEventCreate(&ev1_));
}

SparseChol::~SparseChol() {
  if (ev0_) (void)hipEventDestroy(ev0_);
  if (ev1_) (void)hipEventDestroy(ev1_);
}

void SparseChol::SetB(const double* Bv, const double* Dinv, const double* dBv, const double* dD) {
  has_dA_ = dBv != nullptr;
  hipLaunchKernelGGL(chol_entry_values_kernel, dim3(grid_for(nent_, 256)), dim3(256), 0, s_, nent_, d_ecptr_.get(),
                     d_ctr_.get(), m_, Bv, Dinv, dBv, dD, d_aval_.get(), has_dA_ ? d_daval_.get() : nullptr);
  HIP_CHECK(hipGetLastError());
}

void SparseChol::Run(const SparseCholDev& sch, double* ybuf, const void* solve_args) {
  if ((int64_t)d_P_.size() < sch.p_doubles) d_P_.alloc(sch.p_doubles);
  Bufs b{{d_F_.get(), d_S_.get(), d_Wd_.get(), ybuf, d_P_.get()}};
  const DevPlan& dp = impl_->dp;
  for (size_t oi = 0; oi < sch.ops.size(); ++oi) {
    const CholOp& op = sch.ops[oi];
    const dim3 grid(op.ntask);
    switch (op.type) {
      case kOpAsmTile:
        hipLaunchKernelGGL(chol_asm_tile_kernel, grid, dim3(256), 0, s_, sch.col.get(), op.task0, dp, d_F_.get(),
                           (&op == &sch.ops.front() && &sch == &impl_->factor) ? d_info_.get() : nullptr);
        break;
      case kOpAsmEntries:
        hipLaunchKernelGGL(chol_asm_entries_kernel, grid, dim3(256), 0, s_, sch.col.get(), op.task0, dp, d_F_.get(),
                           d_ecol_.get(), d_eoff_.get(), d_aval_.get(), cur_W_);
        break;
      case kOpDiag:
        hipLaunchKernelGGL(chol_diag_kernel, grid, dim3(256), 0, s_, sch.diag.get(), op.task0, d_F_.get(), d_Wd_.get(),
                           d_info_.get());
        break;
      case kOpGemm:
        if (sch.k64[oi])
          hipLaunchKernelGGL(chol_gemm_k64_kernel, grid, dim3(256), 0, s_, sch.gemm.get(), op.task0, b);
        else
          hipLaunchKernelGGL(chol_gemm_kernel, grid, dim3(256), 0, s_, sch.gemm.get(), op.task0, b);
        break;
      case kOpReduce:
        hipLaunchKernelGGL(chol_reduce_kernel, grid, dim3(256), 0, s_, sch.red.get(), op.task0, b);
        break;
      case kOpGatherS:
        hipLaunchKernelGGL(chol_gather_s_kernel, grid, dim3(256), 0, s_, sch.col.get(), op.task0, dp, d_S_.get());
        break;
      case kOpMirror:
        hipLaunchKernelGGL(chol_mirror_kernel, grid, dim3(256), 0, s_, sch.col.get(), op.task0, dp, d_S_.get());
        break;
      case kOpAsmV:
      case kOpGatherX:
      case kOpLoadV:
      case kOpScatterX: {   // one block per (supernode, group of kSolveColGroup right-hand sides)
        const SolveArgs& sa = *static_cast<const SolveArgs*>(solve_args);
        const dim3 g2(op.ntask, (sa.t + kSolveColGroup - 1) / kSolveColGroup);
        if (op.type == kOpLoadV)
          hipLaunchKernelGGL(chol_load_v_kernel, g2, dim3(256), 0, s_, sch.col.get(), op.task0, dp, sa);
        else if (op.type == kOpAsmV)
          hipLaunchKernelGGL(chol_asmv_kernel, g2, dim3(256), 0, s_, sch.col.get(), op.task0, dp, sa);
        else if (op.type == kOpGatherX)
          hipLaunchKernelGGL(chol_gather_x_kernel, g2, dim3(256), 0, s_, sch.col.get(), op.task0, dp, sa);
        else
          hipLaunchKernelGGL(chol_scatter_x_kernel, g2, dim3(256), 0, s_, sch.col.get(), op.task0, dp, sa);
        break;
      }
      case kOpFwdVec:
      case kOpCopyXS: {
        const SolveArgs& sa = *static_cast<const SolveArgs*>(solve_args);
        if (op.type == kOpFwdVec)
          hipLaunchKernelGGL(chol_fwd_vec_kernel, grid, dim3(64), 0, s_, sch.col.get(), op.task0, dp, sa);
        else
          hipLaunchKernelGGL(chol_copy_xs_kernel, grid, dim3(256), 0, s_, sch.col.get(), op.task0, sa);
        break;
      }
      case kOpBwdVecPart:
      case kOpBwdVecFin: {
        const SolveArgs& sa = *static_cast<const SolveArgs*>(solve_args);
        if (op.type == kOpBwdVecPart)
          hipLaunchKernelGGL(chol_bwd_vec_part_kernel, grid, dim3(256), 0, s_, sch.col.get(), op.task0, dp, sa, d_P_.get());
        else
          hipLaunchKernelGGL(chol_bwd_vec_fin_kernel, grid, dim3(64), 0, s_, sch.col.get(), op.task0, dp, sa, d_P_.get());
        break;
      }
      case kOpFSolve1:
      case kOpBSolve1: {
        const SolveArgs& sa = *static_cast<const SolveArgs*>(solve_args);
        Solve1Args a1{d_lvl_sup_.get(), (int)op.task0, d_F_.get(), d_Wd_.get(), d_woff_.get(), sa.V, sa.vofs, sa.b, sa.X};
        if (op.type == kOpFSolve1)
          hipLaunchKernelGGL(chol_fsolve1_kernel, grid, dim3(256), 0, s_, dp, a1);
        else
          hipLaunchKernelGGL(chol_bsolve1_kernel, grid, dim3(256), 0, s_, dp, a1);
        break;
      }
      default:
        Fatal("sparse Cholesky: unknown op %d", op.type);
    }
    HIP_CHECK(hipGetLastError());
  }
}

void SparseChol::Factor(const double* W) {
  // (the info counter is reset by the first assembly launch)
  HIP_CHECK(hipEventRecord(ev0_, s_));
  cur_W_ = W;
  Run(impl_->factor, nullptr, nullptr);
  HIP_CHECK(hipEventRecord(ev1_, s_));
  factored_ = true;
  timed_ = true;
}

float SparseChol::last_factor_ms() {
  if (!timed_) return 0.f;
  HIP_CHECK(hipEventSynchronize(ev1_));
  float ms = 0.f;
  HIP_CHECK(hipEventElapsedTime(&ms, ev0_, ev1_));
  return ms;
}

int SparseChol::Info() {
  int h = 0;
  HIP_CHECK(hipMemcpyAsync(&h, d_info_.get(), sizeof(int), hipMemcpyDeviceToHost, s_));
  HIP_CHECK(hipStreamSynchronize(s_));
  return h;
}

double SparseChol::LogDet() {
  const int nb = std::min(kRedBlocks, grid_for(n_, 256));
  hipLaunchKernelGGL(chol_logdet_kernel, dim3(nb), dim3(256), 0, s_, n_, d_dpos_.get(), d_F_.get(), d_red_.get());
  hipLaunchKernelGGL(chol_sum_parts_kernel, dim3(1), dim3(256), 0, s_, d_red_.get(), nb, 1, 0,
                     d_red_.get() + 2 * kRedBlocks);
  HIP_CHECK(hipGetLastError());
  double h = 0.;
  HIP_CHECK(hipMemcpyAsync(&h, d_red_.get() + 2 * kRedBlocks, sizeof(double), hipMemcpyDeviceToHost, s_));
  HIP_CHECK(hipStreamSynchronize(s_));
  return h;
}

void SparseChol::SolveCols(const double* b, double* x, int t, int mode) {
  if (!factored_) Fatal("sparse Cholesky: solve before a factorization");
  if (t <= 0) return;
  const std::pair<int, int> key(t, mode);
  Impl& I = *impl_;
  auto it = I.solve.find(key);
  if (it == I.solve.end()) {
    CholSchedule S;
    std::vector<int64_t> vofs;
    chol_solve_schedule(plan_, t, mode == 1, S, vofs, mode == 2);
    std::unique_ptr<SparseCholDev> dev(new SparseCholDev);
    dev->Upload(S);
    std::unique_ptr<DevBuf<int64_t>> dv(new DevBuf<int64_t>);
    upload(*dv, vofs);
    I.vofs_d[key] = std::move(dv);
    it = I.solve.emplace(key, std::move(dev)).first;
  }
  const SparseCholDev& sch = *it->second;
  if ((int64_t)I.V.size() < sch.y_doubles) I.V.alloc(sch.y_doubles);
  if (t == 1 && (int64_t)I.XS.size() < sch.y_doubles) I.XS.alloc(sch.y_doubles);
  SolveArgs a{I.V.get(), I.vofs_d[key]->get(), b, x, t, t == 1 ? I.XS.get() : nullptr, d_F_.get(), d_Wd_.get(),
              d_woff_.get()};
  Run(sch, I.V.get(), &a);
}

void SparseChol::Solve(const double* b, double* x) { SolveCols(b, x, 1, 0); }

void SparseChol::ForwardCols(const double* B, double* X, int nrhs) { SolveCols(B, X, nrhs, 1); }

void SparseChol::SolveMulti(const double* B, double* X, int nrhs) { SolveCols(B, X, nrhs, 0); }

void SparseChol::BackwardCols(const double* B, double* X, int nrhs) { SolveCols(B, X, nrhs, 2); }

void SparseChol::SelectedInverse(double* tr_bdb, double* tr_da, double* diagS) {
  if (!factored_) Fatal("sparse Cholesky: selected inverse before a factorization");
  if (d_S_.size() < (size_t)std::max<int64_t>(plan_.front_doubles, 1)) d_S_.alloc(std::max<int64_t>(plan_.front_doubles, 1));
  if ((int64_t)d_Y_.size() < impl_->selinv.y_doubles) d_Y_.alloc(std::max<int64_t>(impl_->selinv.y_doubles, 1));
  Run(impl_->selinv, d_Y_.get(), nullptr);
  const int nb = std::min(kRedBlocks, grid_for(n_, 256));
  hipLaunchKernelGGL(chol_trace_kernel, dim3(nb), dim3(256), 0, s_, n_, d_ecol_.get(), d_eoff_.get(), d_aval_.get(),
                     has_dA_ ? d_daval_.get() : nullptr, d_S_.get(), d_red_.get());
  for (int q = 0; q < 2; ++q)
    hipLaunchKernelGGL(chol_sum_parts_kernel, dim3(1), dim3(256), 0, s_, d_red_.get(), nb, 2, q,
                       d_red_.get() + 2 * kRedBlocks);
  if (diagS != nullptr)
    hipLaunchKernelGGL(chol_diag_s_kernel, dim3(grid_for(n_, 256)), dim3(256), 0, s_, n_, d_dpos_.get(),
                       d_perm_.get(), d_S_.get(), diagS);
  HIP_CHECK(hipGetLastError());
  double h[2] = {0., 0.};
  HIP_CHECK(hipMemcpyAsync(h, d_red_.get() + 2 * kRedBlocks, sizeof(h), hipMemcpyDeviceToHost, s_));
  HIP_CHECK(hipStreamSynchronize(s_));
  if (tr_bdb) *tr_bdb = h[0];
  if (tr_da) *tr_da = h[1];
}

}  // namespace gpb_amd

// ---- helpers of the Cholesky Laplace path
#include "lik_device.h"

namespace gpb_amd {
namespace {

__global__ void __launch_bounds__(256) chol_dmll_kernel(int n, int lik, double aux, const double* __restrict__ y,
                                                        const double* __restrict__ loc,
                                                        const double* __restrict__ offset, ObsMap obs,
                                                        const double* __restrict__ diagS, double* __restrict__ dmll) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  double dW;
  if (obs.ptr == nullptr) {
    dW = lik_dinfo(lik, aux, y ? y[i] : 0., offset ? loc[i] + offset[i] : loc[i]);
  } else {
    dW = 0.;
    for (int e = obs.ptr[i]; e < obs.ptr[i + 1]; ++e)
      dW += lik_dinfo(lik, aux, obs.y[e], obs.offset ? loc[i] + obs.offset[e] : loc[i]);
  }
  dmll[i] = 0.5 * diagS[i] * dW;
}

__global__ void __launch_bounds__(256) chol_pred_cols_kernel(int n, int mp, const int* __restrict__ nb,
                                                             const double* __restrict__ Bpo, double* __restrict__ cols) {
  const int p = blockIdx.x;   // the columns were zeroed before
  for (int r = threadIdx.x; r < mp; r += 256) {
    const int j = nb[(size_t)p * mp + r];
    if (j >= 0) cols[j + (size_t)p * n] = Bpo[(size_t)p * mp + r];
  }
}

__global__ void __launch_bounds__(256) chol_transpose_scale_kernel(int n, int np, const double* __restrict__ M,
                                                                   double scale, double* __restrict__ V, int ldv) {
  __shared__ double T[64][65];
  const int k0 = blockIdx.x * 64, p0 = blockIdx.y * 64;
  for (int e = threadIdx.x; e < 64 * 64; e += 256) {
    const int kk = e & 63, pp = e >> 6;
    if (k0 + kk < n && p0 + pp < np) T[kk][pp] = M[(k0 + kk) + (size_t)(p0 + pp) * n];
  }
  __syncthreads();
  for (int e = threadIdx.x; e < 64 * 64; e += 256) {
    const int pp = e & 63, kk = e >> 6;
    if (k0 + kk < n && p0 + pp < np) V[(p0 + pp) + (size_t)(k0 + kk) * ldv] = scale * T[kk][pp];
  }
}

}  // namespace

void launch_chol_dmll(int n, int lik, double aux, const double* y, const double* loc, const double* offset,
                      const ObsMap& obs, const double* diagS, double* dmll, hipStream_t s) {
  hipLaunchKernelGGL(chol_dmll_kernel, dim3((n + 255) / 256), dim3(256), 0, s, n, lik, aux, y, loc, offset, obs, diagS,
                     dmll);
  HIP_CHECK(hipGetLastError());
}

void launch_chol_pred_cols(int n, int np, int mp, const int* nb, const double* Bpo, double* cols, hipStream_t s) {
  if (np <= 0) return;
  HIP_CHECK(hipMemsetAsync(cols, 0, sizeof(double) * (size_t)n * np, s));
  hipLaunchKernelGGL(chol_pred_cols_kernel, dim3(np), dim3(256), 0, s, n, mp, nb, Bpo, cols);
  HIP_CHECK(hipGetLastError());
}

void launch_chol_transpose_scale(int n, int np, const double* M, double scale, double* V, int ldv, hipStream_t s) {
  if (n <= 0 || np <= 0) return;
  hipLaunchKernelGGL(chol_transpose_scale_kernel, dim3((n + 63) / 64, (np + 63) / 64), dim3(256), 0, s, n, np, M, scale,
                     V, ldv);
  HIP_CHECK(hipGetLastError());
}

}  // namespace gpb_amd
