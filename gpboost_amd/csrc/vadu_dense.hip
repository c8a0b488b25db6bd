// Dense head of the VADU preconditioner solves (the first K0 Vecchia rows).
//
// Reference replaced: the two sparse triangular solves of the VADU preconditioner
// P^-1 = B^-1 (D^-1 + W)^-1 B^-T (CG_utils.cpp:56-60, 131-136; likelihoods.h:11963-12041) on
// the rows 0..K0-1 of the Vecchia order.
//
// Why: in a random Vecchia ordering the first rows form the deep, thin end of the dependency
// DAG (row i depends on its m nearest EARLIER points, all over the domain while i is small):
// at n = 100k, m = 30 the first 2048 rows alone span 201 of the 388 levels of each solve, with
// ~10 rows per level. Solved level by level that is 2 x 201 dependent steps per application.
// Here the block is solved with dense algebra instead: per factor, B_00 (K0 x K0, unit lower)
// is inverted once, G = B_00^-1 (recursive TRTRI, fp64 MFMA GEMMs), and G^T is stored too (both
// products then read their operand coalesced); per application the head block of both solves
// is two triangular block products (fp64 MFMA), the rest of the rows see it through the
// partial sums of vadu_head.hip:
//   B^T solve:   S = diag(1/dw_0) G^T (R_0 - B_10^T Y_1 - ...)   (later rows folded in first)
//   lower solve: Z_0 = G S
// Same algebra, different rounding: G's entries carry a relative error ~cond(B_00) eps, which
// the tests bound. (Forming M = G diag(1/dw) G^T once per system would save a launch but square
// the condition number: 1e-6 relative error in P^-1 x for a Gaussian kernel at cond(B) ~ 2e5.)
//
// Layout: K0 x K0 matrices column-major (index = Vecchia row), leading dimension ld = K0 rounded
// up to 64, padded with the identity. The t-column blocks are row-major in the solve's storage
// order (row p at X[p * t]); the head-0 rows are reached through DenseHead::row.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "common.h"
#include "dense.h"
#include "latent_kernels.h"

namespace gpb_amd {
namespace {

typedef double double4_t __attribute__((ext_vector_type(4)));

// Bd = B_00 (unit lower): identity everywhere first (separate launch), then the row entries.
__global__ void __launch_bounds__(256) dense_head_identity_kernel(int ld, double* __restrict__ Bd) {
  const size_t total = (size_t)ld * ld;
  for (size_t e = (size_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (size_t)gridDim.x * 256) {
    const size_t i = e % ld, j = e / ld;
    Bd[e] = i == j ? 1. : 0.;
  }
}

__global__ void __launch_bounds__(256) dense_head_scatter_kernel(DenseHead d, double* __restrict__ Bd) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= d.K0 * d.m) return;
  const int j = d.col[e];
  if (j >= 0) Bd[(size_t)(e / d.m) + (size_t)j * d.ld] = d.val[e];
}

// Inverses of the 64 x 64 diagonal blocks of a unit lower triangular matrix, one wave per block:
// lane r computes column r of the inverse by forward substitution over an LDS copy of the block
// (zeros above the diagonal are written too, so W's upper part stays structurally zero).
__global__ void __launch_bounds__(64) unit_lower_diag_inv_kernel(int ld, const double* __restrict__ L,
                                                                 double* __restrict__ W) {
  __shared__ double Ls[64][65];
  const int j0 = blockIdx.x * 64;
  const int r = threadIdx.x;
  for (int c = 0; c < 64; ++c) Ls[r][c] = L[(size_t)(j0 + r) + (size_t)(j0 + c) * ld];
  __syncthreads();
  double x[64];
#pragma unroll
  for (int i = 0; i < 64; ++i) {
    double s = i == r ? 1. : 0.;
#pragma unroll
    for (int p = 0; p < i; ++p) s = fma(-Ls[i][p], x[p], s);
    x[i] = i >= r ? s : 0.;
  }
#pragma unroll
  for (int i = 0; i < 64; ++i) W[(size_t)(j0 + i) + (size_t)(j0 + r) * ld] = x[i];
}

// GT = G^T (both ld x ld column-major), 64 x 64 tiles through LDS
__global__ void __launch_bounds__(256) transpose_kernel(int ld, const double* __restrict__ G, double* __restrict__ GT) {
  __shared__ double tile[64][65];
  const int i0 = blockIdx.x * 64, j0 = blockIdx.y * 64;
  for (int e = threadIdx.x; e < 64 * 64; e += 256) {
    const int i = e & 63, j = e >> 6;
    tile[j][i] = G[(size_t)(i0 + i) + (size_t)(j0 + j) * ld];
  }
  __syncthreads();
  for (int e = threadIdx.x; e < 64 * 64; e += 256) {
    const int j = e & 63, i = e >> 6;
    GT[(size_t)(j0 + j) + (size_t)(i0 + i) * ld] = tile[j][i];
  }
}

// One triangular block product over the head-0 rows, t columns, compact row-major operands:
//   UPPER (A = G^T, upper): Y[i] = (sum_{k >= i} A(i, k) X[k]) / dw[row[i]]
//   !UPPER (A = G, lower):  Y[row[i]] = sum_{k <= i} A(i, k) X[k]   (scattered to the storage rows)
// Workgroup = 16 output rows x 32 columns (two 16 x 16 f64 MFMA tiles); the tile's k range (the
// structural zeros skipped) is split over 8 waves in whole trips, ascending k, loads of the
// next trip issued before the current trip's MFMAs; the partial tiles are combined through LDS
// in a fixed wave order (bitwise repeatable).
constexpr int kApplyWaves = 8;
#ifndef GPB_APPLY_U
#define GPB_APPLY_U 8
#endif
// k steps of 4 per trip: a trip is 4 kApplyU k values, 2 kApplyU MFMAs; the loads of the next
// trip are in flight during the current trip's MFMAs. Trips of 8 k (kApplyU = 2) left the
// products bound by one load round trip per 4 MFMAs (25 us per product at K0 = 2048).
constexpr int kApplyU = GPB_APPLY_U;
struct ApplyTrip {
  double a[kApplyU], b0[kApplyU], b1[kApplyU];
};
__device__ __forceinline__ void apply_load(const double* __restrict__ A, const double* __restrict__ X, int ld, int t,
                                           int ai, int kl, int cA, int cB, bool okA, bool okB, int k, int ke,
                                           ApplyTrip& tr) {
#pragma unroll
  for (int u = 0; u < kApplyU; ++u) {
    const int kk = k + 4 * u + kl;
    const bool ok = kk < ke;
    tr.a[u] = ok ? A[(size_t)ai + (size_t)kk * ld] : 0.;
    tr.b0[u] = (ok && okA) ? X[(size_t)kk * t + cA] : 0.;
    tr.b1[u] = (ok && okB) ? X[(size_t)kk * t + cB] : 0.;
  }
}
template <bool UPPER>
__global__ void __launch_bounds__(kApplyWaves * 64) dense_head_apply_kernel(DenseHead d, const double* __restrict__ A,
                                                                            const double* __restrict__ dw,
                                                                            const double* __restrict__ X,
                                                                            double* __restrict__ Y, int t) {
  __shared__ double red[kApplyWaves][2][4][64];
  const int K0 = d.K0, ld = d.ld;
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int i0 = blockIdx.x * 16;
  const int c0 = blockIdx.y * 32;
  const int kt0 = UPPER ? i0 : 0, kt1 = UPPER ? K0 : min(i0 + 16, K0);
  constexpr int trip = 4 * kApplyU;
  const int per = ((kt1 - kt0 + kApplyWaves * trip - 1) / (kApplyWaves * trip)) * trip;
  const int kb = kt0 + wave * per, ke = min(kb + per, kt1);
  const int ai = i0 + (lane & 15);
  const int kl = lane >> 4;
  const int cA = c0 + (lane & 15), cB = cA + 16;
  const bool okA = cA < t, okB = cB < t;
  double4_t acc0 = {0., 0., 0., 0.}, acc1 = {0., 0., 0., 0.};
  ApplyTrip cur, nxt;
  if (kb < ke) apply_load(A, X, ld, t, ai, kl, cA, cB, okA, okB, kb, ke, cur);
  for (int k = kb; k < ke; k += trip) {
    if (k + trip < ke) apply_load(A, X, ld, t, ai, kl, cA, cB, okA, okB, k + trip, ke, nxt);
#pragma unroll
    for (int u = 0; u < kApplyU; ++u) {
      acc0 = __builtin_amdgcn_mfma_f64_16x16x4f64(cur.a[u], cur.b0[u], acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f64_16x16x4f64(cur.a[u], cur.b1[u], acc1, 0, 0, 0);
    }
    cur = nxt;
  }
#pragma unroll
  for (int rg = 0; rg < 4; ++rg) {
    red[wave][0][rg][lane] = acc0[rg];
    red[wave][1][rg][lane] = acc1[rg];
  }
  __syncthreads();
  if (wave < 2) {   // wave q writes column tile q
    const int q = wave;
    const int c = c0 + 16 * q + (lane & 15);
#pragma unroll
    for (int rg = 0; rg < 4; ++rg) {
      double s = red[0][q][rg][lane];
#pragma unroll
      for (int w = 1; w < kApplyWaves; ++w) s += red[w][q][rg][lane];
      const int i = i0 + (lane >> 4) + 4 * rg;   // f64 MFMA C/D layout (as gemm_f64_kernel)
      if (i < K0 && c < t) {
        if (UPPER) Y[(size_t)i * t + c] = s / dw[d.row[i]];
        else Y[(size_t)d.row[i] * t + c] = s;
      }
    }
  }
}

}  // namespace

void dense_head_factor(const DenseHead& d, double* Bd, double* G, double* GT, double* T, hipStream_t s) {
  if (d.K0 <= 0) return;
  const int ld = d.ld;
  const int gid = (int)std::min<size_t>(((size_t)ld * ld + 255) / 256, 4096);
  hipLaunchKernelGGL(dense_head_identity_kernel, dim3(gid), dim3(256), 0, s, ld, Bd);
  hipLaunchKernelGGL(dense_head_scatter_kernel, dim3((d.K0 * d.m + 255) / 256), dim3(256), 0, s, d, Bd);
  hipLaunchKernelGGL(unit_lower_diag_inv_kernel, dim3(ld / 64), dim3(64), 0, s, ld, Bd, G);
  HIP_CHECK(hipGetLastError());
  // recursive TRTRI on 64-aligned halves: W21 = -W22 (L21 W11)
  struct Rec {
    static void run(int a, int b, int ld, const double* L, double* W, double* X, hipStream_t s) {
      if (b - a <= 64) return;
      const int mid = a + ((b - a) / 2 + 63) / 64 * 64;
      run(a, mid, ld, L, W, X, s);
      run(mid, b, ld, L, W, X, s);
      const int m2 = b - mid, m1 = mid - a;
      gemm_f64(s, m2, m1, m1, 1., L + mid + (size_t)a * ld, ld, 0, W + a + (size_t)a * ld, ld, 0, 0., X, ld, 0, 0, 0,
               1);
      gemm_f64(s, m2, m1, m2, -1., W + mid + (size_t)mid * ld, ld, 0, X, ld, 0, 0., W + mid + (size_t)a * ld, ld, 0, 1,
               0, 0);
    }
  };
  Rec::run(0, ld, ld, Bd, G, T, s);
  hipLaunchKernelGGL(transpose_kernel, dim3(ld / 64, ld / 64), dim3(256), 0, s, ld, G, GT);
  HIP_CHECK(hipGetLastError());
}

void launch_dense_head_apply(const DenseHead& d, const double* G, const double* GT, const double* dw, const double* X,
                             double* S, double* Y, int t, hipStream_t s) {
  if (d.K0 <= 0 || t <= 0) return;
  const dim3 grid(d.ld / 16, (t + 31) / 32);
  hipLaunchKernelGGL((dense_head_apply_kernel<true>), grid, dim3(kApplyWaves * 64), 0, s, d, GT, dw, X, S + (size_t)d.ld * t,
                     t);
  hipLaunchKernelGGL((dense_head_apply_kernel<false>), grid, dim3(kApplyWaves * 64), 0, s, d, G, dw,
                     S + (size_t)d.ld * t, Y, t);
  HIP_CHECK(hipGetLastError());
}

}  // namespace gpb_amd
