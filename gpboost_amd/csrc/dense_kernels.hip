// Dense Gaussian-process likelihood + gradient on gfx950 (gp_approx = "none").
//
// Reference path replaced (re_model_template.h):
//   CalcChol (:5902-5904, Eigen::LLT)              -> blocked right-looking POTRF, fp64 MFMA updates
//   CalcYAux (:9007) / logdet (:2875)              -> W = L^-1 (TRTRI), z = W y, q = |z|^2, 2 sum log L_ii
//   CalcPsiInv (:5987-6007, L^-1 then L^-T L^-1)   -> recursive TRTRI + out-of-place LAUUM (P = W^T W)
//   dense gradient (:1798-1818)                    -> one fused pass over the lower triangle of P that
//                                                     recomputes Sigma_ij and dSigma_ij from the coordinates
// Matrices are column-major with leading dimension ld (a multiple of 64), lower triangles only.
// Every GEMM-shaped step (TRSM-as-GEMM with the inverted diagonal block, panel and trailing
// updates, the TRTRI products and LAUUM) goes through one MFMA kernel:
//   C[M x N] = alpha * op(A) op(B) + beta * C,  64 x 64 output tile per 256-thread workgroup,
//   4 waves x (32 x 32) = 2 x 2 v_mfma_f64_16x16x4 tiles per wave, K staged through LDS in steps of 16
//   (large problems: 128 x 128 tiles, 4 x 4 MFMA tiles per wave, double-buffered K staging),
// with per-tile K ranges that skip the structural zeros of triangular operands and optional
// skipping of output tiles above the diagonal.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <string>
#include <vector>

#include "cov.h"
#include "dense.h"
#include "kernels.h"

namespace gpb_amd {
namespace {

typedef double double4_t __attribute__((ext_vector_type(4)));

constexpr int TM = 64, TN = 64, TK = 16;

struct GemmArgs {
  int M, N, K;
  double alpha, beta;
  const double* A; int lda; int transA;
  const double* B; int ldb; int transB;
  double* C; int ldc;
  int lower_out;     // skip output tiles entirely above the diagonal (local indices)
  int a_lower;       // op(A)[i][k] == 0 for k > i   -> k_end = min(K, m0 + TM); mask
  int a_upper;       // op(A)[i][k] == 0 for k < i   -> k_begin >= m0; mask
  int b_lower;       // op(B)[k][j] == 0 for k < j   -> k_begin >= n0; mask
};

__global__ void __launch_bounds__(256) gemm_f64_kernel(GemmArgs g) {
  __shared__ double As[TK][TM + 1];
  __shared__ double Bs[TK][TN + 1];
  const int m0 = blockIdx.y * TM, n0 = blockIdx.x * TN;
  if (g.lower_out && n0 > m0 + TM - 1) return;
  int k_begin = 0, k_end = g.K;
  if (g.a_lower) k_end = min(k_end, m0 + TM);
  if (g.a_upper) k_begin = max(k_begin, m0);
  if (g.b_lower) k_begin = max(k_begin, n0);
  k_begin = (k_begin / TK) * TK;

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = (wave >> 1) * 32, wn = (wave & 1) * 32;   // wave's 32x32 sub-tile
  double4_t acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[a][b] = (double4_t){0., 0., 0., 0.};

  for (int kk = k_begin; kk < k_end; kk += TK) {
    // stage op(A)[m0:m0+64, kk:kk+16] and op(B)[kk:kk+16, n0:n0+64]; 4 elements per thread each
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int idx = tid + e * 256;
      int i, k;
      if (g.transA) { k = idx & 15; i = idx >> 4; } else { i = idx & 63; k = idx >> 6; }
      const int gi = m0 + i, gk = kk + k;
      double v = 0.;
      if (gi < g.M && gk < k_end && gk >= k_begin && !(g.a_lower && gk > gi) && !(g.a_upper && gk < gi))
        v = g.transA ? g.A[(size_t)gk + (size_t)gi * g.lda] : g.A[(size_t)gi + (size_t)gk * g.lda];
      As[k][i] = v;
      int j, kb;
      if (g.transB) { j = idx & 63; kb = idx >> 6; } else { kb = idx & 15; j = idx >> 4; }
      const int gj = n0 + j, gkb = kk + kb;
      double w = 0.;
      if (gj < g.N && gkb < k_end && gkb >= k_begin && !(g.b_lower && gkb < gj))
        w = g.transB ? g.B[(size_t)gj + (size_t)gkb * g.ldb] : g.B[(size_t)gkb + (size_t)gj * g.ldb];
      Bs[kb][j] = w;
    }
    __syncthreads();
#pragma unroll
    for (int k4 = 0; k4 < TK; k4 += 4) {
      const int kl = k4 + (lane >> 4);
      double a0 = As[kl][wm + (lane & 15)], a1 = As[kl][wm + 16 + (lane & 15)];
      double b0 = Bs[kl][wn + (lane & 15)], b1 = Bs[kl][wn + 16 + (lane & 15)];
      acc[0][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b0, acc[0][0], 0, 0, 0);
      acc[0][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b1, acc[0][1], 0, 0, 0);
      acc[1][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b0, acc[1][0], 0, 0, 0);
      acc[1][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b1, acc[1][1], 0, 0, 0);
    }
    __syncthreads();
  }
  // epilogue: f64 MFMA C/D layout col = lane & 15, row = (lane >> 4) + 4 * reg
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int rg = 0; rg < 4; ++rg) {
        const int i = m0 + wm + a * 16 + (lane >> 4) + 4 * rg;
        const int j = n0 + wn + b * 16 + (lane & 15);
        if (i < g.M && j < g.N && !(g.lower_out && j > i)) {
          double* c = g.C + (size_t)i + (size_t)j * g.ldc;
          const double prev = (g.beta == 0.) ? 0. : g.beta * (*c);
          *c = prev + g.alpha * acc[a][b][rg];
        }
      }
}

// Pipelined tile GEMM: TBt x TBt output tile per 256-thread workgroup, each wave (TBt/2)^2 =
// WT x WT MFMA tiles, K staged in steps of TKB through two LDS buffers: the next step's operands
// are loaded into registers while the current step's MFMAs run, one barrier per step.
//   TBt = 128 (large updates: trailing SYRK, TRTRI / LAUUM products): 4 x 4 MFMA tiles per wave
//     (16 MFMAs per 8 LDS reads); K step 16 and two waves per SIMD: 64 KB of LDS and <= 256
//     registers let two workgroups share a CU, so one's barrier / store phase overlaps the
//     other's MFMAs (n = 20000: 0.339 -> 0.260 s per evaluation vs K step 32 at one workgroup per
//     CU; an XOR-swizzled unpadded LDS layout measured 6 % slower, profiles/r02/dense_ab_r02.log);
//   TBt = 64 (panel / TRSM steps and small products): 2 x 2 MFMA tiles per wave; the pipelined
//     staging replaces the load -> barrier -> MFMA -> barrier sequence whose global-load latency
//     was exposed every K step (~30 us per call at K = 64).
// Same masks, K ranges and summation order per output element for every TBt (k ascending in
// steps of 4 through the MFMA), so the tile size never changes a result bit.
#ifndef GPB_TKB
#define GPB_TKB 16
#endif
constexpr int TB = 128, TKB = GPB_TKB;

template <int TBt>
__device__ __forceinline__ void gemm_tile_body(const GemmArgs& g) {
  constexpr int WT = TBt / 32;   // MFMA tiles per wave and dimension
  __shared__ double As[2][TKB][TBt + 1];
  __shared__ double Bs[2][TKB][TBt + 1];
  const int m0 = blockIdx.y * TBt, n0 = blockIdx.x * TBt;
  if (g.lower_out && n0 > m0 + TBt - 1) return;
  int k_begin = 0, k_end = g.K;
  if (g.a_lower) k_end = min(k_end, m0 + TBt);
  if (g.a_upper) k_begin = max(k_begin, m0);
  if (g.b_lower) k_begin = max(k_begin, n0);
  k_begin = (k_begin / TKB) * TKB;

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = (wave >> 1) * (TBt / 2), wn = (wave & 1) * (TBt / 2);   // wave's sub-tile
  double4_t acc[WT][WT];
#pragma unroll
  for (int a = 0; a < WT; ++a)
#pragma unroll
    for (int b = 0; b < WT; ++b) acc[a][b] = (double4_t){0., 0., 0., 0.};

  constexpr int EPT = TKB * TBt / 256;   // staged elements per thread and operand
  double ra[EPT], rb[EPT];
  auto load = [&](int kk) {
#pragma unroll
    for (int e = 0; e < EPT; ++e) {
      const int idx = tid + e * 256;
      int i, k;
      if (g.transA) { k = idx & (TKB - 1); i = idx / TKB; } else { i = idx & (TBt - 1); k = idx / TBt; }
      const int gi = m0 + i, gk = kk + k;
      double v = 0.;
      if (gi < g.M && gk < k_end && gk >= k_begin && !(g.a_lower && gk > gi) && !(g.a_upper && gk < gi))
        v = g.transA ? g.A[(size_t)gk + (size_t)gi * g.lda] : g.A[(size_t)gi + (size_t)gk * g.lda];
      ra[e] = v;
      int j, kb;
      if (g.transB) { j = idx & (TBt - 1); kb = idx / TBt; } else { kb = idx & (TKB - 1); j = idx / TKB; }
      const int gj = n0 + j, gkb = kk + kb;
      double w = 0.;
      if (gj < g.N && gkb < k_end && gkb >= k_begin && !(g.b_lower && gkb < gj))
        w = g.transB ? g.B[(size_t)gj + (size_t)gkb * g.ldb] : g.B[(size_t)gkb + (size_t)gj * g.ldb];
      rb[e] = w;
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int e = 0; e < EPT; ++e) {
      const int idx = tid + e * 256;
      int i, k;
      if (g.transA) { k = idx & (TKB - 1); i = idx / TKB; } else { i = idx & (TBt - 1); k = idx / TBt; }
      As[buf][k][i] = ra[e];
      int j, kb;
      if (g.transB) { j = idx & (TBt - 1); kb = idx / TBt; } else { kb = idx & (TKB - 1); j = idx / TKB; }
      Bs[buf][kb][j] = rb[e];
    }
  };
  if (k_begin < k_end) {
    load(k_begin);
    store(0);
  }
  __syncthreads();
  int buf = 0;
  for (int kk = k_begin; kk < k_end; kk += TKB) {
    const bool more = kk + TKB < k_end;
    if (more) load(kk + TKB);   // in flight during this step's MFMAs
#pragma unroll
    for (int k4 = 0; k4 < TKB; k4 += 4) {
      const int kl = k4 + (lane >> 4);
      double a[WT], b[WT];
#pragma unroll
      for (int q = 0; q < WT; ++q) {
        a[q] = As[buf][kl][wm + 16 * q + (lane & 15)];
        b[q] = Bs[buf][kl][wn + 16 * q + (lane & 15)];
      }
#pragma unroll
      for (int p = 0; p < WT; ++p)
#pragma unroll
        for (int q = 0; q < WT; ++q) acc[p][q] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[p], b[q], acc[p][q], 0, 0, 0);
    }
    if (more) store(buf ^ 1);   // the other buffer: last read before the previous barrier
    __syncthreads();
    buf ^= 1;
  }
  // epilogue: the beta C reads of a row group of tiles are issued together (clamped addresses, unconditional), then
  // the masked stores -- one memory round trip per group instead of one per element
#pragma unroll
  for (int a = 0; a < WT; ++a) {
    double prev[WT][4];
    if (g.beta != 0.) {
#pragma unroll
      for (int b = 0; b < WT; ++b)
#pragma unroll
        for (int rg = 0; rg < 4; ++rg) {
          const int i = min(m0 + wm + a * 16 + (lane >> 4) + 4 * rg, g.M - 1);
          const int j = min(n0 + wn + b * 16 + (lane & 15), g.N - 1);
          prev[b][rg] = g.C[(size_t)i + (size_t)j * g.ldc];
        }
    } else {
#pragma unroll
      for (int b = 0; b < WT; ++b)
#pragma unroll
        for (int rg = 0; rg < 4; ++rg) prev[b][rg] = 0.;
    }
#pragma unroll
    for (int b = 0; b < WT; ++b)
#pragma unroll
      for (int rg = 0; rg < 4; ++rg) {
        const int i = m0 + wm + a * 16 + (lane >> 4) + 4 * rg;
        const int j = n0 + wn + b * 16 + (lane & 15);
        const double v = (g.beta == 0. ? 0. : g.beta * prev[b][rg]) + g.alpha * acc[a][b][rg];
        if (i < g.M && j < g.N && !(g.lower_out && j > i)) g.C[(size_t)i + (size_t)j * g.ldc] = v;
      }
  }
}

__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2))) gemm_f64_big_kernel(GemmArgs g) {
  gemm_tile_body<128>(g);
}

__global__ void __launch_bounds__(256) gemm_f64_pipe_kernel(GemmArgs g) { gemm_tile_body<64>(g); }

// Split-K form for long-K products with few output tiles (FITC's m x m Woodbury Gram over n
// observations): grid.z = K chunk; chunk z writes its partial product to C + z * cstride.
__global__ void __launch_bounds__(256) gemm_f64_splitk_kernel(GemmArgs g, int kchunk, long cstride) {
  GemmArgs h = g;
  const int k0 = blockIdx.z * kchunk;
  h.K = min(g.K - k0, kchunk);
  h.A = g.transA ? g.A + k0 : g.A + (size_t)k0 * g.lda;
  h.B = g.transB ? g.B + (size_t)k0 * g.ldb : g.B + k0;
  h.C = g.C + (size_t)blockIdx.z * cstride;
  gemm_tile_body<64>(h);
}
// the same with 128 x 128 tiles (the big kernel's body and occupancy; same chunks -> same bits)
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2)))
gemm_f64_splitk_big_kernel(GemmArgs g, int kchunk, long cstride) {
  GemmArgs h = g;
  const int k0 = blockIdx.z * kchunk;
  h.K = min(g.K - k0, kchunk);
  h.A = g.transA ? g.A + k0 : g.A + (size_t)k0 * g.lda;
  h.B = g.transB ? g.B + (size_t)k0 * g.ldb : g.B + k0;
  h.C = g.C + (size_t)blockIdx.z * cstride;
  gemm_tile_body<128>(h);
}

// Lower triangle (i >= j) of Psi = Sigma + I, tile-parallel, upper tiles skipped.
template <int COV>
__global__ void __launch_bounds__(256) build_psi_kernel(const double* __restrict__ X, int n, int d, int ld,
                                                        double var, double phi, double* __restrict__ A) {
  const int i0 = blockIdx.y * 64, j0 = blockIdx.x * 64;
  if (j0 > i0 + 63) return;
  const int ti = threadIdx.x & 63;
  for (int jj = threadIdx.x >> 6; jj < 64; jj += 4) {
    const int i = i0 + ti, j = j0 + jj;
    if (i >= n || j >= n || j > i) continue;
    double v;
    if (i == j) {
      v = var + 1.;
    } else {
      double s = 0.;
      for (int q = 0; q < d; ++q) { const double t = X[(size_t)i * d + q] - X[(size_t)j * d + q]; s += t * t; }
      double dc;
      cov_dcov<COV>(sqrt(s), var, phi, v, dc);
    }
    A[(size_t)i + (size_t)j * ld] = v;
  }
}

// Unblocked Cholesky of one (ib <= 64) diagonal block in LDS + its inverse.
// L overwrites the lower triangle of A's block; L^-1 (upper part zero) is written to Winv's block.
__global__ void __launch_bounds__(256) potrf_diag_kernel(double* A, int lda, int j0, int ib, double* Winv, int ldw,
                                                       int* info) {
  __shared__ double L[64][65];
  __shared__ double I[64][65];
  const int tid = threadIdx.x;
  for (int e = tid; e < 64 * 64; e += 256) {
    const int i = e & 63, j = e >> 6;
    L[i][j] = (i < ib && j < ib && j <= i) ? A[(size_t)(j0 + i) + (size_t)(j0 + j) * lda] : 0.;
    I[i][j] = 0.;
  }
  __syncthreads();
  for (int j = 0; j < ib; ++j) {
    if (tid == 0) {
      const double p = L[j][j];
      if (!(p > 0.)) { atomicAdd(info, 1); L[j][j] = 1.; }   // not positive definite
      else L[j][j] = sqrt(p);
    }
    __syncthreads();
    const double ljj = L[j][j];
    for (int i = j + 1 + tid; i < ib; i += 256) L[i][j] /= ljj;
    __syncthreads();
    const int w = ib - j - 1;
    for (int e = tid; e < w * w; e += 256) {
      const int i = j + 1 + e % w, c = j + 1 + e / w;
      if (c <= i) L[i][c] -= L[i][j] * L[c][j];
    }
    __syncthreads();
  }
  // column c of L^-1 by thread c (forward substitution), in LDS
  if (tid < ib) {
    const int c = tid;
    for (int i = c; i < ib; ++i) {
      double s = (i == c) ? 1. : 0.;
      for (int p = c; p < i; ++p) s -= L[i][p] * I[p][c];
      I[i][c] = s / L[i][i];
    }
  }
  __syncthreads();
  for (int e = tid; e < ib * ib; e += 256) {
    const int i = e % ib, j = e / ib;
    if (j <= i) A[(size_t)(j0 + i) + (size_t)(j0 + j) * lda] = L[i][j];
    Winv[(size_t)(j0 + i) + (size_t)(j0 + j) * ldw] = (j <= i) ? I[i][j] : 0.;
  }
}

// Same factorization and inverse by ONE wave (lane r owns row r in registers): the 256-thread
// form above pays three workgroup barriers and an integer-division loop per column, ~123 us
// per 64-block (313 blocks per n = 20000 evaluation). Here column j is broadcast through LDS
// inside the wave (no barrier needed beyond the wave's own LDS wait), every update is the same
// fma (c - l_rj * l_cj) in the same order, and column c of L^-1 is lane c's forward
// substitution over the LDS copy of L (terms p < c are exact zeros, so the sums equal the
// p = c.. form).
#ifndef GPB_DIAG_NOMASK
#define GPB_DIAG_NOMASK 1
#endif
__global__ void __launch_bounds__(64) potrf_diag_wave_kernel(double* A, int lda, int j0, int ib, double* Winv,
                                                             int ldw, int* info) {
  __shared__ double colb[2][64];
  __shared__ double Ls[64][65];
  const int r = threadIdx.x;
  double row[64];
#pragma unroll
  for (int c = 0; c < 64; ++c)
    row[c] = (r < ib && c < ib && c <= r) ? A[(size_t)(j0 + r) + (size_t)(j0 + c) * lda] : 0.;
#pragma unroll
  for (int j = 0; j < 64; ++j) {
    if (j < ib) {
      const double p = __shfl(row[j], j, 64);
      double d;
      if (!(p > 0.)) {   // not positive definite
        if (r == 0) atomicAdd(info, 1);
        d = 1.;
      } else {
        d = sqrt(p);
      }
      const double l = (r > j) ? row[j] / d : (r == j ? d : 0.);
      if (r >= j) row[j] = l;
      colb[j & 1][r] = l;
      __syncthreads();   // one wave: orders the LDS write before the reads
#if GPB_DIAG_NOMASK
      // no c <= r mask: lanes r < j have l = 0 here, and the entries c > r this updates (upper
      // part) are never read as L (the inverse reads p < i and the diagonal; stores mask c <= r)
#pragma unroll
      for (int c = j + 1; c < 64; ++c) row[c] = fma(-l, colb[j & 1][c], row[c]);
#else
#pragma unroll
      for (int c = j + 1; c < 64; ++c)
        if (c <= r) row[c] = fma(-l, colb[j & 1][c], row[c]);
#endif
    }
  }
#pragma unroll
  for (int c = 0; c < 64; ++c) {
    Ls[r][c] = row[c];
    if (r < ib && c < ib && c <= r) A[(size_t)(j0 + r) + (size_t)(j0 + c) * lda] = row[c];
  }
  __syncthreads();
  // column c = r of L^-1 by forward substitution
  double x[64];
#pragma unroll
  for (int i = 0; i < 64; ++i) {
    double s = (i == r) ? 1. : 0.;
#pragma unroll
    for (int p = 0; p < i; ++p) s -= Ls[i][p] * x[p];
    x[i] = (i >= r && i < ib) ? s / Ls[i][i] : 0.;
  }
  // Winv[i][c] = x_c[i]: lane c holds column c
#pragma unroll
  for (int i = 0; i < 64; ++i)
    if (i < ib && r < ib) Winv[(size_t)(j0 + i) + (size_t)(j0 + r) * ldw] = (r <= i) ? x[i] : 0.;
}

// The same factorization and inverse of one 64 x 64 diagonal block with four waves (the default; the
// one-wave kernel above runs every one of its ~19k instructions on one wave, so each pivot costs the
// whole step's issue time: 78 vs 52 us per block in scripts/microbench/diag_bench.hip, V0 vs V8).
// Wave w holds the columns c = 4k + w (k < 16) of all 64 rows (lane r = row r) in registers; pivot j's
// owner wave (j & 3) takes the pivot by v_readlane, scales its column (by 1 / sqrt(p) from the rsqrt estimate) and
// publishes L[:, j] (zero for rows <= j) to LDS; after ONE barrier every wave updates its columns c > j
// (registers whose columns are all <= j skipped at compile time, the published zeros make the rest
// branch-free). A partial block (ib < 64) is padded with the identity. Every element sees the same
// operations in the same order as in the one-wave kernel except the pivot scaling (multiplies by the Newton-refined
// 1 / sqrt(p) instead of the one-wave form's sqrt + division: within an ulp per entry); L^-1 by its code on
// wave 0 (a four-wave split of that substitution changed the rounding enough to move an ill-conditioned
// Gaussian-kernel FITC case past its 1e-9 reference bound).
__global__ void __launch_bounds__(256) potrf_diag_quad_kernel(double* A, int lda, int j0, int ib, double* Winv,
                                                              int ldw, int* info) {
  __shared__ double colb[2][64];
  __shared__ double Ls[64][65];
  const int r = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int rr = min(r, ib - 1);
  double col[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int c = 4 * k + w;
    const double v = A[(size_t)(j0 + rr) + (size_t)(j0 + min(c, ib - 1)) * lda];
    col[k] = (r < ib && c < ib) ? (c <= r ? v : 0.) : (r == c ? 1. : 0.);
  }
  bool bad = false;
#pragma unroll
  for (int j = 0; j < 64; ++j) {
    if (w == (j & 3)) {
      const int lo = __builtin_amdgcn_readlane(__double2loint(col[j >> 2]), j);
      const int hi = __builtin_amdgcn_readlane(__double2hiint(col[j >> 2]), j);
      const double p = __hiloint2double(hi, lo);
      bad = bad || !(p > 0.);   // not positive definite
      // y = 1 / sqrt(p) by the hardware estimate and two Newton steps, L_jj = p y, the column scaled by y
      // (multiplies instead of a square root and a division on the pivot chain)
      const double ps = p > 0. ? p : 1., h = 0.5 * ps;
      double y = __builtin_amdgcn_rsq(ps);
      y = y * fma(-h * y, y, 1.5);
      y = y * fma(-h * y, y, 1.5);
      const double l = r > j ? col[j >> 2] * y : (r == j ? ps * y : col[j >> 2]);
      col[j >> 2] = l;
      colb[j & 1][r] = r > j ? l : 0.;
    }
    __syncthreads();
    const double lr = colb[j & 1][r];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      if (4 * k + 3 <= j) continue;   // every column of register k is <= j
      col[k] = fma(-lr, colb[j & 1][4 * k + w], col[k]);
    }
  }
  if (bad && r == 0) atomicAdd(info, 1);
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int c = 4 * k + w;
    Ls[r][c] = col[k];
    if (c <= r && r < ib && c < ib) A[(size_t)(j0 + r) + (size_t)(j0 + c) * lda] = col[k];
  }
  __syncthreads();
  // L^-1 (column r on lane r) by the right-looking form of the one-wave kernel's forward substitution, on the
  // four waves: wave w keeps the partial sums acc_i of its rows i = 4k + w; step p: the owner of row p forms
  // x_p = acc_p / L_pp (its final entry) and publishes it, one barrier, every wave updates acc_i -= L_ip x_p for
  // its rows i > p. Each acc_i sees the same fmas in the same order (p ascending from delta_ir) as the one-wave
  // kernel's dot products, so the inverse is bit-identical, at one division + one fma of latency per step instead
  // of a dependent LDS-load + fma chain of length i per row on one wave.
  double acc[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) acc[k] = (4 * k + w == r) ? 1. : 0.;
#pragma unroll
  for (int p = 0; p < 64; ++p) {
    if (w == (p & 3)) {
      const double xp = (p >= r && p < ib) ? acc[p >> 2] / Ls[p][p] : 0.;
      acc[p >> 2] = xp;
      colb[p & 1][r] = xp;
    }
    __syncthreads();
    const double xp = colb[p & 1][r];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      if (4 * k + 3 <= p) continue;   // every row of register k is <= p
      const int i = 4 * k + w;
      if (i > p) acc[k] = fma(-Ls[i][p], xp, acc[k]);
    }
  }
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int i = 4 * k + w;
    if (i < ib && r < ib) Winv[(size_t)(j0 + i) + (size_t)(j0 + r) * ldw] = (r <= i) ? acc[k] : 0.;
  }
}

// one diagonal block: GPBOOST_AMD_DIAG_FORM = quad (default) | wave | old (A/B)
void launch_potrf_diag(hipStream_t s, double* A, int ld, int j0, int ib, double* W, int* info) {
  static const int form = [] {
    const char* e = std::getenv("GPBOOST_AMD_DIAG_FORM");
    if (std::getenv("GPBOOST_AMD_DIAG_OLD") != nullptr) return 2;
    if (e == nullptr || std::string(e) == "quad") return 0;
    if (std::string(e) == "wave") return 1;
    if (std::string(e) == "old") return 2;
    Fatal("GPBOOST_AMD_DIAG_FORM must be quad, wave or old (got '%s')", e);
    return 0;
  }();
  if (form == 0) hipLaunchKernelGGL(potrf_diag_quad_kernel, dim3(1), dim3(256), 0, s, A, ld, j0, ib, W, ld, info);
  else if (form == 1) hipLaunchKernelGGL(potrf_diag_wave_kernel, dim3(1), dim3(64), 0, s, A, ld, j0, ib, W, ld, info);
  else hipLaunchKernelGGL(potrf_diag_kernel, dim3(1), dim3(256), 0, s, A, ld, j0, ib, W, ld, info);
  HIP_CHECK(hipGetLastError());
}

// Cross-covariance C[i + p ld] = cov(|x_i - xp_p|) (n x np, column-major) and, when S is non-null,
// the prediction points' own covariance S[p + q np] (np x np, diagonal = var)
template <int COV>
__global__ void __launch_bounds__(256) build_cross_kernel(const double* __restrict__ X, const double* __restrict__ Xp,
                                                          int n, int np, int d, int ld, double var, double phi,
                                                          double* __restrict__ C) {
  const int i = blockIdx.x * 64 + (threadIdx.x & 63);
  const int p = blockIdx.y * 4 + (threadIdx.x >> 6);
  if (i >= n || p >= np) return;
  double s = 0.;
  for (int q = 0; q < d; ++q) {
    const double t = X[(size_t)i * d + q] - Xp[(size_t)p * d + q];
    s += t * t;
  }
  double c, dc;
  if (s == 0. && X == Xp && i == p) { c = var; } else { cov_dcov<COV>(sqrt(s), var, phi, c, dc); }
  C[(size_t)i + (size_t)p * ld] = c;
}

// Combined GP + grouped random effects: the grouped components' covariances sum_k tau_k [lev_k(a) == lev_k(b)]
struct GroupedTau {
  double t[8];
};

// A (lower triangle incl. the diagonal) += sum_k tau_k [lev_k(i) == lev_k(j)]
__global__ void __launch_bounds__(256) add_grouped_kernel(int n, int ld, int K, const int* __restrict__ lev,
                                                          GroupedTau tau, double* __restrict__ A) {
  const int i0 = blockIdx.y * 64, j0 = blockIdx.x * 64;
  if (j0 > i0 + 63) return;
  const int ti = threadIdx.x & 63;
  for (int jj = threadIdx.x >> 6; jj < 64; jj += 4) {
    const int i = i0 + ti, j = j0 + jj;
    if (i >= n || j >= n || j > i) continue;
    double v = 0.;
    for (int k = 0; k < K; ++k)
      if (lev[(size_t)k * n + i] == lev[(size_t)k * n + j]) v += tau.t[k];
    A[(size_t)i + (size_t)j * ld] += v;
  }
}

// C (n x np, ld) += sum_k tau_k [lev_k(i) == plev_k(p)] (cross-covariances to the prediction points), or with
// lev = plev (np x np, square) the prediction points' own grouped covariances
__global__ void __launch_bounds__(256) add_grouped_cross_kernel(int n, int np, int ld, int K, const int* __restrict__ lev,
                                                                const int* __restrict__ plev, GroupedTau tau,
                                                                double* __restrict__ C) {
  const int i = blockIdx.x * 64 + (threadIdx.x & 63);
  const int p = blockIdx.y * 4 + (threadIdx.x >> 6);
  if (i >= n || p >= np) return;
  double v = 0.;
  for (int k = 0; k < K; ++k)
    if (lev[(size_t)k * n + i] == plev[(size_t)k * np + p]) v += tau.t[k];
  C[(size_t)i + (size_t)p * ld] += v;
}

// per 64 x 64 tile of the lower triangle of P = Psi^-1: part[tile * K + k] = sum over the tile's entries with
// lev_k(i) == lev_k(j) of w P_ij (w = 1 on the diagonal, 2 below: the full symmetric sum); upper tiles write 0
__global__ void __launch_bounds__(256) grouped_trace_kernel(int n, int ld, int K, const int* __restrict__ lev,
                                                            const double* __restrict__ P, double* __restrict__ part) {
  __shared__ double red[4][8];
  const int i0 = blockIdx.y * 64, j0 = blockIdx.x * 64;
  const int tile = blockIdx.y * gridDim.x + blockIdx.x;
  double acc[8] = {0., 0., 0., 0., 0., 0., 0., 0.};
  if (j0 <= i0 + 63) {
    const int ti = threadIdx.x & 63;
    for (int jj = threadIdx.x >> 6; jj < 64; jj += 4) {
      const int i = i0 + ti, j = j0 + jj;
      if (i >= n || j >= n || j > i) continue;
      const double v = P[(size_t)i + (size_t)j * ld] * (i == j ? 1. : 2.);
#pragma unroll
      for (int k = 0; k < 8; ++k)
        if (k < K && lev[(size_t)k * n + i] == lev[(size_t)k * n + j]) acc[k] += v;
    }
  }
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    double s = acc[k];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    if (lane == 0) red[w][k] = s;
  }
  __syncthreads();
  if (threadIdx.x < K) {
    const int k = threadIdx.x;
    part[(size_t)tile * K + k] = (red[0][k] + red[1][k]) + (red[2][k] + red[3][k]);
  }
}

// 2 * sum log L_ii -> out (single block, fixed order)
__global__ void __launch_bounds__(256) logdet_kernel(const double* A, int lda, int n, double* out) {
  __shared__ double red[256];
  double s = 0.;
  for (int i = threadIdx.x; i < n; i += 256) s += log(A[(size_t)i + (size_t)i * lda]);
  red[threadIdx.x] = s;
  __syncthreads();
  for (int off = 128; off > 0; off >>= 1) {
    if ((int)threadIdx.x < off) red[threadIdx.x] += red[threadIdx.x + off];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[0] = 2. * red[0];
}

// z = W y for lower-triangular W: partial[cb][i] = sum_{j in column block cb, j <= i} W_ij y_j
__global__ void __launch_bounds__(256) trmv_lower_partial_kernel(const double* W, int ld, int n, const double* y,
                                                              double* partial) {
  const int i = blockIdx.y * 256 + threadIdx.x;
  const int cb = blockIdx.x;             // 256-column block
  if (cb * 256 > blockIdx.y * 256 + 255) return;
  __shared__ double ys[256];
  const int jc = cb * 256 + threadIdx.x;
  ys[threadIdx.x] = jc < n ? y[jc] : 0.;
  __syncthreads();
  if (i >= n) return;
  double s = 0.;
  const int jmax = min(min(cb * 256 + 256, n), i + 1);
  for (int j = cb * 256; j < jmax; ++j) s += W[(size_t)i + (size_t)j * ld] * ys[j - cb * 256];
  partial[(size_t)cb * n + i] = s;
}

__global__ void __launch_bounds__(256) trmv_lower_reduce_kernel(const double* partial, int n, double* z) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  double s = 0.;
  for (int cb = 0; cb <= i / 256; ++cb) s += partial[(size_t)cb * n + i];
  z[i] = s;
}

// out_j = sum_{i >= j} W_ij z_i (W^T z), one wave per column, coalesced down the column
__global__ void __launch_bounds__(256) trmv_lower_t_kernel(const double* W, int ld, int n, const double* z, double* out) {
  const int j = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (j >= n) return;
  double s = 0.;
  for (int i = j + lane; i < n; i += 64) s += W[(size_t)i + (size_t)j * ld] * z[i];
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
  if (lane == 0) out[j] = s;
}

// Fused gradient pass over the lower triangle of P = Psi^-1 (64 x 64 tiles):
// per tile partial sums of [tr(dPsi_var P), tr(dPsi_rng P), yaux^T dPsi_var yaux, yaux^T dPsi_rng yaux]
// with dPsi_var = Sigma (variance on the diagonal), dPsi_rng = dSigma/dlog(phi) (0 on the diagonal).
template <int COV>
__global__ void __launch_bounds__(256) dense_grad_kernel(const double* __restrict__ X, int n, int d, int ld,
                                                         double var, double phi, const double* __restrict__ P,
                                                         const double* __restrict__ yaux, double* __restrict__ part) {
  const int i0 = blockIdx.y * 64, j0 = blockIdx.x * 64;
  const int tile = blockIdx.y * gridDim.x + blockIdx.x;
  double s[4] = {0., 0., 0., 0.};
  if (j0 <= i0 + 63) {
    const int ti = threadIdx.x & 63;
    const int i = i0 + ti;
    double xi[3] = {0., 0., 0.};
    if (i < n) for (int q = 0; q < d; ++q) xi[q] = X[(size_t)i * d + q];
    const double yi = i < n ? yaux[i] : 0.;
    for (int jj = threadIdx.x >> 6; jj < 64; jj += 4) {
      const int j = j0 + jj;
      if (i >= n || j >= n || j > i) continue;
      const double pij = P[(size_t)i + (size_t)j * ld];
      double c, dc;
      if (i == j) {
        c = var; dc = 0.;
      } else {
        double ss = 0.;
        for (int q = 0; q < d; ++q) { const double t = xi[q] - X[(size_t)j * d + q]; ss += t * t; }
        cov_dcov<COV>(sqrt(ss), var, phi, c, dc);
      }
      const double w = (i == j) ? 1. : 2.;
      const double yy = w * yi * yaux[j];
      s[0] += w * c * pij;
      s[1] += w * dc * pij;
      s[2] += yy * c;
      s[3] += yy * dc;
    }
  }
  __shared__ double red[4][256];
  for (int q = 0; q < 4; ++q) red[q][threadIdx.x] = s[q];
  __syncthreads();
  for (int off = 128; off > 0; off >>= 1) {
    if ((int)threadIdx.x < off)
      for (int q = 0; q < 4; ++q) red[q][threadIdx.x] += red[q][threadIdx.x + off];
    __syncthreads();
  }
  if (threadIdx.x < 4) part[(size_t)tile * 4 + threadIdx.x] = red[threadIdx.x][0];
}

// Fisher information (GPB_GetCovPar calc_std_dev, re_model_template.h:9144-9236 dense branch):
// full derivative matrices of Sigma on the ORIGINAL scale (GetZSigmaZtGrad transf_scale = false,
// re_comp.h:1389-1438): D1 = dSigma/dsigma1^2 = correlation (1 on the diagonal), D2 = dSigma/drho
// = dscale * dcorr/dlog(phi) (0 on the diagonal; dscale = sigma1^2 dlog(phi)/drho).
template <int COV>
__global__ void __launch_bounds__(256) build_dsigma_kernel(const double* __restrict__ X, int n, int d, int ld,
                                                           double phi, double dscale, double* __restrict__ D1,
                                                           double* __restrict__ D2) {
  const int i0 = blockIdx.y * 64, j0 = blockIdx.x * 64;
  const int ti = threadIdx.x & 63;
  for (int jj = threadIdx.x >> 6; jj < 64; jj += 4) {
    const int i = i0 + ti, j = j0 + jj;
    if (i >= n || j >= n) continue;
    double c = 1., dc = 0.;
    if (i != j) {
      double s = 0.;
      for (int q = 0; q < d; ++q) { const double t = X[(size_t)i * d + q] - X[(size_t)j * d + q]; s += t * t; }
      cov_dcov<COV>(sqrt(s), 1., phi, c, dc);
    }
    D1[(size_t)i + (size_t)j * ld] = c;
    D2[(size_t)i + (size_t)j * ld] = dscale * dc;
  }
}

// Upper triangle of a symmetric matrix from its lower triangle (64 x 64 tiles above the diagonal).
__global__ void __launch_bounds__(256) mirror_lower_kernel(double* A, int n, int ld) {
  const int i0 = blockIdx.y * 64, j0 = blockIdx.x * 64;
  if (j0 < i0) return;
  const int ti = threadIdx.x & 63;
  for (int jj = threadIdx.x >> 6; jj < 64; jj += 4) {
    const int i = i0 + ti, j = j0 + jj;
    if (i < n && j < n && i < j) A[(size_t)i + (size_t)j * ld] = A[(size_t)j + (size_t)i * ld];
  }
}

// Per lower tile pair {T = (bi, bj), T' = (bj, bi)} of P (= Psi^-1, symmetric) and G_k = P D_k:
// partial sums of [sum P^2, sum P o G1, sum P o G2, sum G1 o G1^T, sum G1 o G2^T, sum G2 o G2^T] over
// both tiles (fixed order; the transposed tiles of G staged in LDS so every global read coalesces).
__global__ void __launch_bounds__(256) fisher_trace_kernel(const double* __restrict__ P, const double* __restrict__ G1,
                                                           const double* __restrict__ G2, int n, int ld,
                                                           double* __restrict__ part) {
  __shared__ double t1[64][65], t2[64][65];
  const int bi = blockIdx.y, bj = blockIdx.x;
  const int tile = bi * gridDim.x + bj;
  const int ti = threadIdx.x & 63;
  double s[6] = {0., 0., 0., 0., 0., 0.};
  if (bj <= bi) {
    const int i0 = bi * 64, j0 = bj * 64;
    // stage T' = rows j0.., cols i0.. of G1, G2 transposed: t[a][b] = G(j0 + b, i0 + a)
    for (int aa = threadIdx.x >> 6; aa < 64; aa += 4) {
      const int r = j0 + ti, c = i0 + aa;
      const bool ok = r < n && c < n;
      t1[aa][ti] = ok ? G1[(size_t)r + (size_t)c * ld] : 0.;
      t2[aa][ti] = ok ? G2[(size_t)r + (size_t)c * ld] : 0.;
    }
    __syncthreads();
    const bool diag = bi == bj;
    for (int jj = threadIdx.x >> 6; jj < 64; jj += 4) {
      const int i = i0 + ti, j = j0 + jj;
      if (i >= n || j >= n) continue;
      const double p = P[(size_t)i + (size_t)j * ld];   // lower tile (i >= j on diagonal tiles below)
      const double g1 = G1[(size_t)i + (size_t)j * ld], g2 = G2[(size_t)i + (size_t)j * ld];
      const double h1 = t1[ti][jj], h2 = t2[ti][jj];   // G(j, i)
      if (diag) {   // the tile is its own transpose: every (i, j) once
        const double pp = (i >= j) ? p : P[(size_t)j + (size_t)i * ld];
        s[0] += pp * pp;
        s[1] += pp * g1;
        s[2] += pp * g2;
        s[3] += g1 * h1;
        s[4] += g1 * h2;
        s[5] += g2 * h2;
      } else {      // (i, j) and (j, i)
        s[0] += 2. * p * p;
        s[1] += p * (g1 + h1);
        s[2] += p * (g2 + h2);
        s[3] += 2. * g1 * h1;
        s[4] += g1 * h2 + h1 * g2;
        s[5] += 2. * g2 * h2;
      }
    }
  }
  __syncthreads();
  double* red = &t1[0][0];   // reuse: 6 x 256
  for (int q = 0; q < 6; ++q) red[q * 256 + threadIdx.x] = s[q];
  __syncthreads();
  for (int off = 128; off > 0; off >>= 1) {
    if ((int)threadIdx.x < off)
      for (int q = 0; q < 6; ++q) red[q * 256 + threadIdx.x] += red[q * 256 + threadIdx.x + off];
    __syncthreads();
  }
  if (threadIdx.x < 6) part[(size_t)tile * 6 + threadIdx.x] = red[threadIdx.x * 256];
}

// diag_j = sum_{i >= j} W_ij^2 (diag(W^T W) = diag(Psi^-1) for W = L^-1), one wave per column
__global__ void __launch_bounds__(256) colnorm2_lower_kernel(const double* W, int ld, int n, double* diag) {
  const int j = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (j >= n) return;
  double s = 0.;
  for (int i = j + lane; i < n; i += 64) {
    const double w = W[(size_t)i + (size_t)j * ld];
    s += w * w;
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
  if (lane == 0) diag[j] = s;
}

// Inverses of the 64 x 64 diagonal blocks of a UNIT lower-triangular matrix (one wave per block, lane
// c = column c of the block inverse by forward substitution in LDS) into W's diagonal blocks (upper
// part zero), the input trtri_lower expects.
__global__ void __launch_bounds__(64) unit_lower_diag_inv_kernel(const double* A, int lda, int n, double* W, int ldw) {
  // column r of the inverse kept in LDS (X[i][r]), the block's L broadcast from LDS
  __shared__ double Ls[64][65];
  __shared__ double X[64][65];
  const int j0 = blockIdx.x * 64, ib = min(64, n - j0);
  const int r = threadIdx.x;
  for (int c = 0; c < 64; ++c)
    Ls[r][c] = (r < ib && c < ib && c < r) ? A[(size_t)(j0 + r) + (size_t)(j0 + c) * lda] : 0.;
  __syncthreads();
  for (int i = 0; i < 64; ++i) {
    double s = (i == r) ? 1. : 0.;
    for (int p = r; p < i; ++p) s -= Ls[i][p] * X[p][r];
    X[i][r] = (i >= r && i < ib) ? s : 0.;
  }
  for (int i = 0; i < ib; ++i)
    if (r < ib) W[(size_t)(j0 + i) + (size_t)(j0 + r) * ldw] = (r <= i) ? X[i][r] : 0.;
}

// A[:, j] *= d[j] for j < n (rows < m)
__global__ void __launch_bounds__(256) scale_cols_kernel(double* A, int lda, int m, int n, const double* d) {
  const int i = blockIdx.x * 256 + threadIdx.x, j = blockIdx.y;
  if (i < m && j < n) A[(size_t)i + (size_t)j * lda] *= d[j];
}

// A[i, i] += v for i < n
__global__ void __launch_bounds__(256) add_diag_kernel(double* A, int lda, int n, double v) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < n) A[(size_t)i + (size_t)i * lda] += v;
}

// out[i] = sum_c U[i + c ld]^2 / nsim + add[i] (fixed column order)
__global__ void __launch_bounds__(256) rowsq_kernel(const double* U, int ld, int n, int nsim, const double* add,
                                                   double* out) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  double s = 0.;
  for (int c = 0; c < nsim; ++c) {
    const double u = U[(size_t)i + (size_t)c * ld];
    s += u * u;
  }
  out[i] = (nsim > 0 ? s / nsim : 0.) + add[i];
}

// out[p] = sum_i T[i + p ld]^2 for i < n (one wave per column)
__global__ void __launch_bounds__(256) colnorm2_full_kernel(const double* T, int ld, int n, int np, double* out) {
  const int p = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (p >= np) return;
  double s = 0.;
  for (int i = lane; i < n; i += 64) {
    const double t = T[(size_t)i + (size_t)p * ld];
    s += t * t;
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
  if (lane == 0) out[p] = s;
}

__global__ void dot_kernel(const double* a, const double* b, int n, double* out) {
  __shared__ double red[256];
  double s = 0.;
  for (int i = threadIdx.x; i < n; i += 256) s += a[i] * b[i];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int off = 128; off > 0; off >>= 1) {
    if ((int)threadIdx.x < off) red[threadIdx.x] += red[threadIdx.x + off];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[0] = red[0];
}

void gemm(hipStream_t s, int M, int N, int K, double alpha, const double* A, int lda, int transA, const double* B,
          int ldb, int transB, double beta, double* C, int ldc, int lower_out = 0, int a_lower = 0, int a_upper = 0,
          int b_lower = 0) {
  if (M <= 0 || N <= 0) return;
  GemmArgs g{M, N, K, alpha, beta, A, lda, transA, B, ldb, transB, C, ldc, lower_out, a_lower, a_upper, b_lower};
  static const bool small_only = std::getenv("GPBOOST_AMD_GEMM64") != nullptr;   // A/B: 64 x 64 tiles only
  // large tiles only where they still give every CU two tiles (small problems keep the 64 x 64
  // form's parallelism: n = 2000 measured 7.6 ms vs 8.6 ms per evaluation with 128 x 128 tiles)
  if ((long)((M + TB - 1) / TB) * ((N + TB - 1) / TB) >= 512 && !small_only) {
    dim3 grid((N + TB - 1) / TB, (M + TB - 1) / TB);
    hipLaunchKernelGGL(gemm_f64_big_kernel, grid, dim3(256), 0, s, g);
    HIP_CHECK(hipGetLastError());
    return;
  }
  dim3 grid((N + TN - 1) / TN, (M + TM - 1) / TM);
  static const bool unpiped = std::getenv("GPBOOST_AMD_GEMM_UNPIPED") != nullptr;   // A/B: round-1 64-tile form
  if (unpiped)
    hipLaunchKernelGGL(gemm_f64_kernel, grid, dim3(256), 0, s, g);
  else
    hipLaunchKernelGGL(gemm_f64_pipe_kernel, grid, dim3(256), 0, s, g);
  HIP_CHECK(hipGetLastError());
}

template <typename F>
void dispatch_cov(int cov, F&& f) {
  switch (cov) {
    case kMatern05: f(std::integral_constant<int, kMatern05>{}); break;
    case kMatern15: f(std::integral_constant<int, kMatern15>{}); break;
    case kMatern25: f(std::integral_constant<int, kMatern25>{}); break;
    case kGaussian: f(std::integral_constant<int, kGaussian>{}); break;
    default: Fatal("unsupported covariance type %d", cov);
  }
}

}  // namespace

void gemm_f64(hipStream_t s, int M, int N, int K, double alpha, const double* A, int lda, int transA, const double* B,
              int ldb, int transB, double beta, double* C, int ldc, int lower_out, int a_lower, int a_upper,
              int b_lower) {
  gemm(s, M, N, K, alpha, A, lda, transA, B, ldb, transB, beta, C, ldc, lower_out, a_lower, a_upper, b_lower);
}

int gemm_f64_splitk(hipStream_t s, int M, int N, int K, const double* A, int lda, int transA, const double* B, int ldb,
                    int transB, double* C, int ldc, long cstride, int target_blocks, int max_chunks) {
  if (M <= 0 || N <= 0 || K <= 0) return 0;
  const long tiles = (long)((M + TN - 1) / TN) * ((N + TN - 1) / TN);
  int chunks = (int)std::max<long>(1, std::min<long>((target_blocks + tiles - 1) / tiles, (K + 255) / 256));
  chunks = std::max(1, std::min(chunks, max_chunks));
  int kchunk = (K + chunks - 1) / chunks;
  kchunk = (kchunk + TKB - 1) / TKB * TKB;
  chunks = (K + kchunk - 1) / kchunk;
  GemmArgs g{M, N, K, 1., 0., A, lda, transA, B, ldb, transB, C, ldc, 0, 0, 0, 0};
  // 128-tiles once both dimensions fill them (GPBOOST_AMD_SPLITK_TILE=64 keeps the 64-tile form: A/B)
  static const bool tile64 = [] {
    const char* e = std::getenv("GPBOOST_AMD_SPLITK_TILE");
    return e != nullptr && std::string(e) == "64";
  }();
  if (!tile64 && M >= TB && N >= TB) {
    dim3 grid((N + TB - 1) / TB, (M + TB - 1) / TB, chunks);
    hipLaunchKernelGGL(gemm_f64_splitk_big_kernel, grid, dim3(256), 0, s, g, kchunk, cstride);
  } else {
    dim3 grid((N + TN - 1) / TN, (M + TM - 1) / TM, chunks);
    hipLaunchKernelGGL(gemm_f64_splitk_kernel, grid, dim3(256), 0, s, g, kchunk, cstride);
  }
  HIP_CHECK(hipGetLastError());
  return chunks;
}

DenseSolver::DenseSolver(int n, int d, const double* d_X, hipStream_t stream)
    : n_(n), d_(d), ld_(((n + 63) / 64) * 64), d_X_(d_X), stream_(stream) {
  const size_t nn = (size_t)ld_ * (size_t)ld_;
  A_.alloc(nn);
  W_.alloc(nn);
  T_.alloc((size_t)ld_ * (size_t)(ld_ / 2 + 64));
  HIP_CHECK(hipMemsetAsync(A_.get(), 0, nn * sizeof(double), stream_));
  HIP_CHECK(hipMemsetAsync(W_.get(), 0, nn * sizeof(double), stream_));
  const int nb = (n + 255) / 256;
  vec_.alloc((size_t)4 * ld_ + (size_t)nb * n);
  const int tiles = ((n + 63) / 64) * ((n + 63) / 64);
  red_.alloc((size_t)tiles * 4 + 16);
  info_.alloc(1);
  HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&h_red_), 16 * sizeof(double), hipHostMallocDefault));
  for (auto& e : ev_) HIP_CHECK(hipEventCreate(&e));
}

DenseSolver::~DenseSolver() {
  if (h_red_) (void)hipHostFree(h_red_);
  for (auto& e : ev_) if (e) (void)hipEventDestroy(e);
  for (auto& e : ev_la_) if (e) (void)hipEventDestroy(e);
  if (s_chain_) (void)hipStreamDestroy(s_chain_);
  if (s_rest_) (void)hipStreamDestroy(s_rest_);
}

void chol_lower(hipStream_t s, double* A, double* W, int n, int ld, int* info) {
  // two-level right-looking Cholesky: 256-wide outer panels, 64-wide inner steps
  constexpr int NBO = 256, NBI = 64;
  for (int J0 = 0; J0 < n; J0 += NBO) {
    const int jb = std::min(NBO, n - J0);
    for (int j0 = J0; j0 < J0 + jb; j0 += NBI) {
      const int ib = std::min(NBI, J0 + jb - j0);
      launch_potrf_diag(s, A, ld, j0, ib, W, info);
      const int r0 = j0 + ib;
      if (r0 < n) {
        // L21 = A21 * L11^-T  (in place: each 64-row tile reads its whole K = ib range first)
        gemm(s, n - r0, ib, ib, 1., A + r0 + (size_t)j0 * ld, ld, 0, W + j0 + (size_t)j0 * ld, ld, 1, 0.,
             A + r0 + (size_t)j0 * ld, ld, 0, 0, 0, 0);
      }
      if (r0 < J0 + jb) {
        // remaining panel columns: A[r0:n, r0:J0+jb] -= L[r0:n, j0:r0] L[r0:J0+jb, j0:r0]^T
        gemm(s, n - r0, J0 + jb - r0, ib, -1., A + r0 + (size_t)j0 * ld, ld, 0, A + r0 + (size_t)j0 * ld, ld, 1,
             1., A + r0 + (size_t)r0 * ld, ld, 1, 0, 0, 0);
      }
    }
    const int t0 = J0 + jb;
    if (t0 < n) {
      // trailing SYRK: A[t0:n, t0:n] -= L[t0:n, J0:t0] L[t0:n, J0:t0]^T  (lower tiles only)
      gemm(s, n - t0, n - t0, jb, -1., A + t0 + (size_t)J0 * ld, ld, 0, A + t0 + (size_t)J0 * ld, ld, 1, 1.,
           A + t0 + (size_t)t0 * ld, ld, 1, 0, 0, 0);
    }
  }
}

void trtri_lower(hipStream_t s, const double* L, double* W, double* X, int a, int b, int ld) {
  // W[a:b, a:b] = L[a:b, a:b]^-1 (lower); diagonal 64-blocks were inverted by chol_lower.
  if (b - a <= 64) return;
  const int half = ((b - a) / 2 + 63) / 64 * 64;
  const int mid = a + half;
  trtri_lower(s, L, W, X, a, mid, ld);
  trtri_lower(s, L, W, X, mid, b, ld);
  const int m2 = b - mid, m1 = mid - a;
  // X = L21 * W11   (W11 lower)
  gemm(s, m2, m1, m1, 1., L + mid + (size_t)a * ld, ld, 0, W + a + (size_t)a * ld, ld, 0, 0., X, ld, 0, 0, 0, 1);
  // W21 = -W22 * X  (W22 lower)
  gemm(s, m2, m1, m2, -1., W + mid + (size_t)mid * ld, ld, 0, X, ld, 0, 0., W + mid + (size_t)a * ld, ld, 0, 1, 0, 0);
}

void launch_logdet_chol(hipStream_t s, const double* L, int ld, int n, double* out) {
  hipLaunchKernelGGL(logdet_kernel, dim3(1), dim3(256), 0, s, L, ld, n, out);
  HIP_CHECK(hipGetLastError());
}

void DenseSolver::Potrf() { chol_lower(stream_, A_.get(), W_.get(), n_, ld_, info_.get()); }

void vecchia_latent_dense_pred(hipStream_t s, int N, int n, const double* B, const double* D, const double* y,
                               bool want_var, bool want_cov, double* mean, double* var, double* cov) {
  // Sigma = B^-1 diag(D) B^-T over all N points (observed first), then the Gaussian conditional of
  // the last np = N - n points given y = (latent at the observed points) + N(0, I):
  //   mean = Sigma_po (Sigma_oo + I)^-1 y,  cov = Sigma_pp - Sigma_po (Sigma_oo + I)^-1 Sigma_op
  const int np = N - n;
  if (np <= 0 || n <= 0) Fatal("vecchia_latent_dense_pred: empty observed or prediction set");
  const int ld = (N + 63) / 64 * 64, ldo = (n + 63) / 64 * 64;
  const size_t NN = (size_t)ld * ld;
  DevBuf<double> dB(NN), W(NN), S(NN), T((size_t)ld * (ld / 2 + 64)), dD(N), Aoo((size_t)ldo * ldo),
      Woo((size_t)ldo * ldo), v((size_t)3 * ldo), Tm((size_t)ldo * np);
  DevBuf<int> info(1);
  HIP_CHECK(hipMemsetAsync(W.get(), 0, NN * sizeof(double), s));
  HIP_CHECK(hipMemsetAsync(Woo.get(), 0, (size_t)ldo * ldo * sizeof(double), s));
  HIP_CHECK(hipMemsetAsync(info.get(), 0, sizeof(int), s));
  HIP_CHECK(hipMemcpy2DAsync(dB.get(), sizeof(double) * ld, B, sizeof(double) * N, sizeof(double) * N, N,
                             hipMemcpyHostToDevice, s));
  HIP_CHECK(hipMemcpyAsync(dD.get(), D, sizeof(double) * N, hipMemcpyHostToDevice, s));
  // W = B^-1 (unit lower: diagonal-block inverses, then the recursive TRTRI)
  hipLaunchKernelGGL(unit_lower_diag_inv_kernel, dim3((N + 63) / 64), dim3(64), 0, s, dB.get(), ld, N, W.get(), ld);
  trtri_lower(s, dB.get(), W.get(), T.get(), 0, N, ld);
  // S = (W diag(D)) W^T
  HIP_CHECK(hipMemcpyAsync(dB.get(), W.get(), NN * sizeof(double), hipMemcpyDeviceToDevice, s));
  hipLaunchKernelGGL(scale_cols_kernel, dim3((N + 255) / 256, N), dim3(256), 0, s, dB.get(), ld, N, N, dD.get());
  gemm(s, N, N, N, 1., dB.get(), ld, 0, W.get(), ld, 1, 0., S.get(), ld, 0, 1, 0, 0);
  // Aoo = Sigma_oo + I = L L^T, Woo = L^-1
  HIP_CHECK(hipMemcpy2DAsync(Aoo.get(), sizeof(double) * ldo, S.get(), sizeof(double) * ld, sizeof(double) * n, n,
                             hipMemcpyDeviceToDevice, s));
  hipLaunchKernelGGL(add_diag_kernel, dim3((n + 255) / 256), dim3(256), 0, s, Aoo.get(), ldo, n, 1.);
  chol_lower(s, Aoo.get(), Woo.get(), n, ldo, info.get());
  trtri_lower(s, Aoo.get(), Woo.get(), T.get(), 0, n, ldo);
  // mean = Sigma_po Woo^T Woo y
  double* dy = v.get();
  double* z = dy + ldo;
  double* x = z + ldo;
  HIP_CHECK(hipMemcpyAsync(dy, y, sizeof(double) * n, hipMemcpyHostToDevice, s));
  gemm(s, n, 1, n, 1., Woo.get(), ldo, 0, dy, ldo, 0, 0., z, ldo, 0, 1, 0, 0);
  hipLaunchKernelGGL(trmv_lower_t_kernel, dim3((n + 3) / 4), dim3(256), 0, s, Woo.get(), ldo, n, z, x);
  DevBuf<double> dm(np);
  gemm(s, np, 1, n, 1., S.get() + n, ld, 0, x, ldo, 0, 0., dm.get(), np);
  HIP_CHECK(hipMemcpyAsync(mean, dm.get(), sizeof(double) * np, hipMemcpyDeviceToHost, s));
  if (want_var || want_cov) {
    // Tm = Woo Sigma_op (n x np); cov = Sigma_pp - Tm^T Tm
    gemm(s, n, np, n, 1., Woo.get(), ldo, 0, S.get() + (size_t)n * ld, ld, 0, 0., Tm.get(), ldo, 0, 1, 0, 0);
    DevBuf<double> C((size_t)np * np);
    HIP_CHECK(hipMemcpy2DAsync(C.get(), sizeof(double) * np, S.get() + n + (size_t)n * ld, sizeof(double) * ld,
                               sizeof(double) * np, np, hipMemcpyDeviceToDevice, s));
    gemm(s, np, np, n, -1., Tm.get(), ldo, 1, Tm.get(), ldo, 0, 1., C.get(), np);
    std::vector<double> h((size_t)np * np);
    HIP_CHECK(hipMemcpyAsync(h.data(), C.get(), sizeof(double) * h.size(), hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipStreamSynchronize(s));
    if (want_cov) std::copy(h.begin(), h.end(), cov);
    if (want_var)
      for (int p = 0; p < np; ++p) var[p] = h[(size_t)p * np + p];
  }
  HIP_CHECK(hipGetLastError());
  int h_info = 0;
  HIP_CHECK(hipMemcpyAsync(&h_info, info.get(), sizeof(int), hipMemcpyDeviceToHost, s));
  HIP_CHECK(hipStreamSynchronize(s));
  if (h_info != 0) Fatal("the observed covariance plus nugget is not positive definite (Cholesky failed)");
}

void latent_pred_moments(hipStream_t s, int np, const double* Bp, const double* Dp, const double* d_V, int nsim,
                         bool want_var, bool want_cov, double* var, double* cov) {
  // W = Bp^-1 (identity when Bp is null), U = W V; var = rowsum(U^2) / nsim + diag(W diag(Dp) W^T);
  // cov = U U^T / nsim + W diag(Dp) W^T (PredictLaplaceApproxVecchia, likelihoods.h:6713-6749).
  // nsim = 0 (d_V unused): the Gaussian likelihood's W diag(Dp) W^T alone (Vecchia_utils.cpp:1977-2006)
  const int ld = (np + 63) / 64 * 64;
  const size_t NN = (size_t)ld * ld;
  DevBuf<double> W, dB, T, U, dD(np), det(np), out(np);
  HIP_CHECK(hipMemcpyAsync(dD.get(), Dp, sizeof(double) * np, hipMemcpyHostToDevice, s));
  const double* Uptr = d_V;
  int ldu = np;
  if (Bp != nullptr) {
    W.alloc(NN);
    dB.alloc(NN);
    T.alloc((size_t)ld * (ld / 2 + 64));
    if (nsim > 0) U.alloc((size_t)ld * nsim);
    HIP_CHECK(hipMemsetAsync(W.get(), 0, NN * sizeof(double), s));
    HIP_CHECK(hipMemcpy2DAsync(dB.get(), sizeof(double) * ld, Bp, sizeof(double) * np, sizeof(double) * np, np,
                               hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(unit_lower_diag_inv_kernel, dim3((np + 63) / 64), dim3(64), 0, s, dB.get(), ld, np, W.get(), ld);
    trtri_lower(s, dB.get(), W.get(), T.get(), 0, np, ld);
    if (nsim > 0) gemm(s, np, nsim, np, 1., W.get(), ld, 0, d_V, np, 0, 0., U.get(), ld, 0, 1, 0, 0);
    Uptr = U.get();
    ldu = ld;
  }
  DevBuf<double> WD, C;
  if (Bp != nullptr && (want_var || want_cov)) {
    WD.alloc(NN);   // W diag(Dp)
    HIP_CHECK(hipMemcpyAsync(WD.get(), W.get(), NN * sizeof(double), hipMemcpyDeviceToDevice, s));
    hipLaunchKernelGGL(scale_cols_kernel, dim3((np + 255) / 256, np), dim3(256), 0, s, WD.get(), ld, np, np, dD.get());
  }
  if (want_var) {
    if (Bp != nullptr) {   // diag(W diag(Dp) W^T)_i = sum_k W_ik^2 Dp_k = rowsum(W diag(sqrt Dp))^2: by the GEMM
      C.alloc(NN);
      gemm(s, np, np, np, 1., WD.get(), ld, 0, W.get(), ld, 1, 0., C.get(), ld, 0, 1, 0, 0);
      HIP_CHECK(hipMemcpy2DAsync(det.get(), sizeof(double), C.get(), sizeof(double) * (ld + 1), sizeof(double), np,
                                 hipMemcpyDeviceToDevice, s));
    } else {
      HIP_CHECK(hipMemcpyAsync(det.get(), dD.get(), sizeof(double) * np, hipMemcpyDeviceToDevice, s));
    }
    hipLaunchKernelGGL(rowsq_kernel, dim3((np + 255) / 256), dim3(256), 0, s, Uptr, ldu, np, nsim, det.get(), out.get());
    HIP_CHECK(hipMemcpyAsync(var, out.get(), sizeof(double) * np, hipMemcpyDeviceToHost, s));
  }
  if (want_cov) {
    DevBuf<double> Cv((size_t)np * np);
    if (Bp != nullptr) {
      gemm(s, np, np, np, 1., WD.get(), ld, 0, W.get(), ld, 1, 0., Cv.get(), np, 0, 1, 0, 0);
    } else {
      HIP_CHECK(hipMemsetAsync(Cv.get(), 0, sizeof(double) * np * np, s));
      HIP_CHECK(hipMemcpy2DAsync(Cv.get(), sizeof(double) * (np + 1), dD.get(), sizeof(double), sizeof(double), np,
                                 hipMemcpyDeviceToDevice, s));
    }
    if (nsim > 0) gemm(s, np, np, nsim, 1. / nsim, Uptr, ldu, 0, Uptr, ldu, 1, 1., Cv.get(), np);
    HIP_CHECK(hipMemcpyAsync(cov, Cv.get(), sizeof(double) * np * np, hipMemcpyDeviceToHost, s));
  }
  HIP_CHECK(hipGetLastError());
  HIP_CHECK(hipStreamSynchronize(s));
}

void spd_solve_inverse(hipStream_t s, int n, const double* A, const double* b, double* x, double* diag, double* inv) {
  // A = L L^T (POTRF), W = L^-1 (TRTRI), x = W^T (W b), diag(A^-1) = column norms^2 of W,
  // A^-1 = W^T W (MFMA GEMM)
  if (n <= 0) return;
  const int ld = (n + 63) / 64 * 64;
  const size_t nn = (size_t)ld * ld;
  DevBuf<double> dA(nn), dW(nn), T((size_t)ld * (ld / 2 + 64)), v((size_t)3 * ld);
  DevBuf<int> info(1);
  HIP_CHECK(hipMemsetAsync(dW.get(), 0, nn * sizeof(double), s));
  HIP_CHECK(hipMemsetAsync(info.get(), 0, sizeof(int), s));
  HIP_CHECK(hipMemcpy2DAsync(dA.get(), sizeof(double) * ld, A, sizeof(double) * n, sizeof(double) * n, n,
                             hipMemcpyHostToDevice, s));
  chol_lower(s, dA.get(), dW.get(), n, ld, info.get());
  trtri_lower(s, dA.get(), dW.get(), T.get(), 0, n, ld);
  double* db = v.get();
  double* z = db + ld;
  double* dx = z + ld;
  if (b != nullptr) {
    HIP_CHECK(hipMemcpyAsync(db, b, sizeof(double) * n, hipMemcpyHostToDevice, s));
    gemm(s, n, 1, n, 1., dW.get(), ld, 0, db, ld, 0, 0., z, ld, 0, 1, 0, 0);                          // z = W b
    hipLaunchKernelGGL(trmv_lower_t_kernel, dim3((n + 3) / 4), dim3(256), 0, s, dW.get(), ld, n, z, dx);  // W^T z
    HIP_CHECK(hipMemcpyAsync(x, dx, sizeof(double) * n, hipMemcpyDeviceToHost, s));
  }
  if (diag != nullptr) {
    hipLaunchKernelGGL(colnorm2_lower_kernel, dim3((n + 3) / 4), dim3(256), 0, s, dW.get(), ld, n, z);
    HIP_CHECK(hipMemcpyAsync(diag, z, sizeof(double) * n, hipMemcpyDeviceToHost, s));
  }
  if (inv != nullptr) {
    gemm(s, n, n, n, 1., dW.get(), ld, 1, dW.get(), ld, 0, 0., dA.get(), ld, 0, 0, 1, 1);   // full W^T W
    HIP_CHECK(hipMemcpy2DAsync(inv, sizeof(double) * n, dA.get(), sizeof(double) * ld, sizeof(double) * n, n,
                               hipMemcpyDeviceToHost, s));
  }
  HIP_CHECK(hipGetLastError());
  int h_info = 0;
  HIP_CHECK(hipMemcpyAsync(&h_info, info.get(), sizeof(int), hipMemcpyDeviceToHost, s));
  HIP_CHECK(hipStreamSynchronize(s));
  if (h_info != 0) Fatal("matrix is not positive definite (Cholesky failed)");
}

// The same factorization with one panel of lookahead: after panel J's inner steps, the trailing
// update is split into the next panel's columns (on the chain stream, immediately) and the rest
// (on a second stream), so panel J+1's diagonal factorizations, TRSMs and panel updates run
// while the bulk of panel J's SYRK is still in flight. Every output element receives the same
// products in the same order as Potrf() (per-element K order is tile-size independent), so the
// factor is bitwise identical.
void DenseSolver::PotrfLookahead() {
  const int n = n_, ld = ld_;
  double* A = A_.get();
  double* W = W_.get();
  constexpr int NBO = 256, NBI = 64;
  if (!s_chain_) {
    int lo = 0, hi = 0;
    HIP_CHECK(hipDeviceGetStreamPriorityRange(&lo, &hi));
    HIP_CHECK(hipStreamCreateWithPriority(&s_chain_, hipStreamNonBlocking, hi));
    HIP_CHECK(hipStreamCreateWithPriority(&s_rest_, hipStreamNonBlocking, lo));
    for (auto& e : ev_la_) HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  }
  hipEvent_t ev_in = ev_la_[0], ev_panel = ev_la_[1], ev_rest = ev_la_[2];
  HIP_CHECK(hipEventRecord(ev_in, stream_));
  HIP_CHECK(hipStreamWaitEvent(s_chain_, ev_in, 0));
  HIP_CHECK(hipStreamWaitEvent(s_rest_, ev_in, 0));
  bool rest_pending = false;
  for (int J0 = 0; J0 < n; J0 += NBO) {
    const int jb = std::min(NBO, n - J0);
    for (int j0 = J0; j0 < J0 + jb; j0 += NBI) {
      const int ib = std::min(NBI, J0 + jb - j0);
      launch_potrf_diag(s_chain_, A, ld, j0, ib, W, info_.get());
      const int r0 = j0 + ib;
      if (r0 < n)
        gemm(s_chain_, n - r0, ib, ib, 1., A + r0 + (size_t)j0 * ld, ld, 0, W + j0 + (size_t)j0 * ld, ld, 1, 0.,
             A + r0 + (size_t)j0 * ld, ld, 0, 0, 0, 0);
      if (r0 < J0 + jb)
        gemm(s_chain_, n - r0, J0 + jb - r0, ib, -1., A + r0 + (size_t)j0 * ld, ld, 0, A + r0 + (size_t)j0 * ld, ld, 1,
             1., A + r0 + (size_t)r0 * ld, ld, 1, 0, 0, 0);
    }
    const int t0 = J0 + jb;
    if (t0 >= n) break;
    const int nb = std::min(NBO, n - t0);   // the next panel's columns
    // the previous rest update wrote these columns: wait for it before touching them
    if (rest_pending) HIP_CHECK(hipStreamWaitEvent(s_chain_, ev_rest, 0));
    HIP_CHECK(hipEventRecord(ev_panel, s_chain_));   // panel J final
    gemm(s_chain_, n - t0, nb, jb, -1., A + t0 + (size_t)J0 * ld, ld, 0, A + t0 + (size_t)J0 * ld, ld, 1, 1.,
         A + t0 + (size_t)t0 * ld, ld, 1, 0, 0, 0);
    const int t1 = t0 + nb;
    if (t1 < n) {
      HIP_CHECK(hipStreamWaitEvent(s_rest_, ev_panel, 0));
      gemm(s_rest_, n - t1, n - t1, jb, -1., A + t1 + (size_t)J0 * ld, ld, 0, A + t1 + (size_t)J0 * ld, ld, 1, 1.,
           A + t1 + (size_t)t1 * ld, ld, 1, 0, 0, 0);
      HIP_CHECK(hipEventRecord(ev_rest, s_rest_));
      rest_pending = true;
    }
  }
  HIP_CHECK(hipEventRecord(ev_panel, s_chain_));
  HIP_CHECK(hipStreamWaitEvent(stream_, ev_panel, 0));
  HIP_CHECK(hipEventRecord(ev_rest, s_rest_));
  HIP_CHECK(hipStreamWaitEvent(stream_, ev_rest, 0));
}

void DenseSolver::Trtri(int a, int b) { trtri_lower(stream_, A_.get(), W_.get(), T_.get(), a, b, ld_); }

void DenseSolver::Eval(int cov_type, double var, double phi, const double* d_y, bool want_grad, double* sums,
                       double* kernel_ms) {
  const int n = n_, ld = ld_, d = d_;
  double* A = A_.get();
  double* W = W_.get();
  double* z = vec_.get();
  double* yaux = z + ld;
  double* partial = z + 2 * (size_t)ld;
  double* dred = red_.get();
  HIP_CHECK(hipMemsetAsync(info_.get(), 0, sizeof(int), stream_));
  HIP_CHECK(hipEventRecord(ev_[0], stream_));
  const int nt = (n + 63) / 64;
  dispatch_cov(cov_type, [&](auto c) {
    hipLaunchKernelGGL((build_psi_kernel<decltype(c)::value>), dim3(nt, nt), dim3(256), 0, stream_, d_X_, n, d, ld, var,
                       phi, A);
  });
  HIP_CHECK(hipGetLastError());
  AddGrouped();
  static const bool no_lookahead = std::getenv("GPBOOST_AMD_DENSE_NO_LOOKAHEAD") != nullptr;   // A/B
  if (!no_lookahead)
    PotrfLookahead();
  else
    Potrf();
  HIP_CHECK(hipEventRecord(ev_[1], stream_));
  hipLaunchKernelGGL(logdet_kernel, dim3(1), dim3(256), 0, stream_, A, ld, n, dred + 0);
  Trtri(0, n);
  // z = W y, q = |z|^2
  const int nb = (n + 255) / 256;
  hipLaunchKernelGGL(trmv_lower_partial_kernel, dim3(nb, nb), dim3(256), 0, stream_, W, ld, n, d_y, partial);
  hipLaunchKernelGGL(trmv_lower_reduce_kernel, dim3(nb), dim3(256), 0, stream_, partial, n, z);
  hipLaunchKernelGGL(dot_kernel, dim3(1), dim3(256), 0, stream_, z, z, n, dred + 1);
  HIP_CHECK(hipGetLastError());
  int ngrad = 0;
  if (want_grad) {
    // y_aux = W^T z ; P = W^T W (lower) into A (L no longer needed)
    hipLaunchKernelGGL(trmv_lower_t_kernel, dim3((n + 3) / 4), dim3(256), 0, stream_, W, ld, n, z, yaux);
    gemm(stream_, n, n, n, 1., W, ld, 1, W, ld, 0, 0., A, ld, 1, 0, 1, 1);
    dispatch_cov(cov_type, [&](auto c) {
      hipLaunchKernelGGL((dense_grad_kernel<decltype(c)::value>), dim3(nt, nt), dim3(256), 0, stream_, d_X_, n, d, ld,
                         var, phi, A, yaux, dred + 16);
    });
    HIP_CHECK(hipGetLastError());
    ngrad = nt * nt;
    launch_sum_blocks(dred + 16, ngrad, 4, dred + 2, stream_);
  }
  HIP_CHECK(hipMemcpyAsync(h_red_, dred, sizeof(double) * 6, hipMemcpyDeviceToHost, stream_));
  int info = 0;
  HIP_CHECK(hipMemcpyAsync(&info, info_.get(), sizeof(int), hipMemcpyDeviceToHost, stream_));
  HIP_CHECK(hipEventRecord(ev_[2], stream_));
  HIP_CHECK(hipStreamSynchronize(stream_));
  if (info != 0) Fatal("the covariance matrix is not positive definite (Cholesky failed)");
  float ms0 = 0.f, ms1 = 0.f;
  HIP_CHECK(hipEventElapsedTime(&ms0, ev_[0], ev_[1]));
  HIP_CHECK(hipEventElapsedTime(&ms1, ev_[0], ev_[2]));
  kernel_ms[0] = ms0;
  kernel_ms[1] = ms1;
  sums[0] = h_red_[0];
  sums[1] = h_red_[1];
  if (want_grad) {
    // s1_k = -1/2 y_aux^T dPsi_k y_aux ; s2_k = tr(dPsi_k Psi^-1)   (re_model_template.h:1813-1814)
    sums[2] = -0.5 * h_red_[4];
    sums[3] = -0.5 * h_red_[5];
    sums[4] = h_red_[2];
    sums[5] = h_red_[3];
  } else {
    sums[2] = sums[3] = sums[4] = sums[5] = 0.;
  }
}

void DenseSolver::Fisher(int cov_type, double var, double phi, double dscale, double* sums6) {
  // P = Psi^-1 as in Eval's gradient branch, then G_k = P D_k (two MFMA GEMMs) and the traces
  const int n = n_, ld = ld_, d = d_;
  double* A = A_.get();
  double* W = W_.get();
  HIP_CHECK(hipMemsetAsync(info_.get(), 0, sizeof(int), stream_));
  const int nt = (n + 63) / 64;
  dispatch_cov(cov_type, [&](auto c) {
    hipLaunchKernelGGL((build_psi_kernel<decltype(c)::value>), dim3(nt, nt), dim3(256), 0, stream_, d_X_, n, d, ld, var,
                       phi, A);
  });
  HIP_CHECK(hipGetLastError());
  AddGrouped();
  PotrfLookahead();
  Trtri(0, n);
  gemm(stream_, n, n, n, 1., W, ld, 1, W, ld, 0, 0., A, ld, 1, 0, 1, 1);   // P = W^T W (lower)
  hipLaunchKernelGGL(mirror_lower_kernel, dim3(nt, nt), dim3(256), 0, stream_, A, n, ld);
  DevBuf<double> D2((size_t)ld * ld), G1((size_t)ld * ld), G2((size_t)ld * ld), part((size_t)nt * nt * 6);
  dispatch_cov(cov_type, [&](auto c) {
    hipLaunchKernelGGL((build_dsigma_kernel<decltype(c)::value>), dim3(nt, nt), dim3(256), 0, stream_, d_X_, n, d, ld,
                       phi, dscale, W, D2.get());   // D1 into W (L^-1 is no longer needed)
  });
  HIP_CHECK(hipGetLastError());
  gemm(stream_, n, n, n, 1., A, ld, 0, W, ld, 0, 0., G1.get(), ld);
  gemm(stream_, n, n, n, 1., A, ld, 0, D2.get(), ld, 0, 0., G2.get(), ld);
  hipLaunchKernelGGL(fisher_trace_kernel, dim3(nt, nt), dim3(256), 0, stream_, A, G1.get(), G2.get(), n, ld, part.get());
  HIP_CHECK(hipGetLastError());
  double* dred = red_.get();
  launch_sum_blocks(part.get(), nt * nt, 6, dred + 8, stream_);
  HIP_CHECK(hipMemcpyAsync(h_red_, dred + 8, sizeof(double) * 6, hipMemcpyDeviceToHost, stream_));
  int info = 0;
  HIP_CHECK(hipMemcpyAsync(&info, info_.get(), sizeof(int), hipMemcpyDeviceToHost, stream_));
  HIP_CHECK(hipStreamSynchronize(stream_));
  if (info != 0) Fatal("the covariance matrix is not positive definite (Cholesky failed)");
  for (int q = 0; q < 6; ++q) sums6[q] = h_red_[q];
}

void DenseSolver::SetGrouped(int K, const int* d_lev, const double* tau) {
  if (K < 0 || K > 8) Fatal("the dense GP + grouped random effects path supports at most 8 grouped effects, got %d", K);
  gK_ = K;
  g_lev_ = d_lev;
  for (int k = 0; k < 8; ++k) g_tau_[k] = k < K ? tau[k] : 0.;
}

void DenseSolver::SetGroupedPred(int np, const int* d_plev) {
  gnp_ = np;
  g_plev_ = d_plev;
}

void DenseSolver::AddGrouped() {
  if (gK_ == 0) return;
  GroupedTau t;
  for (int k = 0; k < 8; ++k) t.t[k] = g_tau_[k];
  const int nt = (n_ + 63) / 64;
  hipLaunchKernelGGL(add_grouped_kernel, dim3(nt, nt), dim3(256), 0, stream_, n_, ld_, gK_, g_lev_, t, A_.get());
  HIP_CHECK(hipGetLastError());
}

void DenseSolver::GroupedTraces(double* s2, double* yaux) {
  if (gK_ == 0) Fatal("GroupedTraces without grouped effects");
  const int n = n_, ld = ld_, nt = (n + 63) / 64, K = gK_;
  const int tiles = nt * nt;
  g_part_.alloc((size_t)tiles * K + K);
  double* out = g_part_.get() + (size_t)tiles * K;
  hipLaunchKernelGGL(grouped_trace_kernel, dim3(nt, nt), dim3(256), 0, stream_, n, ld, K, g_lev_, A_.get(),
                     g_part_.get());
  HIP_CHECK(hipGetLastError());
  launch_sum_blocks(g_part_.get(), tiles, K, out, stream_);
  HIP_CHECK(hipMemcpyAsync(s2, out, sizeof(double) * K, hipMemcpyDeviceToHost, stream_));
  HIP_CHECK(hipMemcpyAsync(yaux, vec_.get() + ld, sizeof(double) * n, hipMemcpyDeviceToHost, stream_));
  HIP_CHECK(hipStreamSynchronize(stream_));
  for (int k = 0; k < K; ++k) s2[k] *= g_tau_[k];
}

void DenseSolver::Factor(int cov_type, double var, double phi) {
  const int n = n_, ld = ld_, d = d_;
  HIP_CHECK(hipMemsetAsync(info_.get(), 0, sizeof(int), stream_));
  const int nt = (n + 63) / 64;
  dispatch_cov(cov_type, [&](auto c) {
    hipLaunchKernelGGL((build_psi_kernel<decltype(c)::value>), dim3(nt, nt), dim3(256), 0, stream_, d_X_, n, d, ld, var,
                       phi, A_.get());
  });
  HIP_CHECK(hipGetLastError());
  AddGrouped();
  PotrfLookahead();
  Trtri(0, n);
}

void DenseSolver::Predict(int cov_type, double var, double phi, const double* d_y, const double* Xp, int np,
                          bool want_var, bool want_cov, double* mean, double* pvar, double* pcov) {
  // CalcPred (re_model_template.h CalcPred, gp_approx = "none", Gaussian): with Psi = L L^T, W = L^-1,
  // T = W Sigma_op: mean = T^T (W y), cov = Sigma_pp - T^T T (variances: var - column norms of T)
  const int n = n_, ld = ld_, d = d_;
  Factor(cov_type, var, phi);
  DevBuf<double> dXp((size_t)np * d), C((size_t)ld * np), T((size_t)ld * np), z(ld), m(np), v(np);
  HIP_CHECK(hipMemcpyAsync(dXp.get(), Xp, sizeof(double) * np * d, hipMemcpyHostToDevice, stream_));
  dispatch_cov(cov_type, [&](auto c) {
    hipLaunchKernelGGL((build_cross_kernel<decltype(c)::value>), dim3((n + 63) / 64, (np + 3) / 4), dim3(256), 0,
                       stream_, d_X_, dXp.get(), n, np, d, ld, var, phi, C.get());
  });
  HIP_CHECK(hipGetLastError());
  GroupedTau gt;
  for (int k = 0; k < 8; ++k) gt.t[k] = g_tau_[k];
  if (gK_ > 0) {
    if (gnp_ != np || g_plev_ == nullptr) Fatal("prediction group levels missing for the combined model");
    hipLaunchKernelGGL(add_grouped_cross_kernel, dim3((n + 63) / 64, (np + 3) / 4), dim3(256), 0, stream_, n, np, ld, gK_,
                       g_lev_, g_plev_, gt, C.get());
    HIP_CHECK(hipGetLastError());
  }
  gemm(stream_, n, np, n, 1., W_.get(), ld, 0, C.get(), ld, 0, 0., T.get(), ld, 0, 1, 0, 0);
  gemm(stream_, n, 1, n, 1., W_.get(), ld, 0, d_y, ld, 0, 0., z.get(), ld, 0, 1, 0, 0);
  gemm(stream_, np, 1, n, 1., T.get(), ld, 1, z.get(), ld, 0, 0., m.get(), np);
  HIP_CHECK(hipMemcpyAsync(mean, m.get(), sizeof(double) * np, hipMemcpyDeviceToHost, stream_));
  if (want_var) {
    hipLaunchKernelGGL(colnorm2_full_kernel, dim3((np + 3) / 4), dim3(256), 0, stream_, T.get(), ld, n, np, v.get());
    HIP_CHECK(hipMemcpyAsync(pvar, v.get(), sizeof(double) * np, hipMemcpyDeviceToHost, stream_));
  }
  if (want_cov) {
    DevBuf<double> S((size_t)np * np);
    dispatch_cov(cov_type, [&](auto c) {
      hipLaunchKernelGGL((build_cross_kernel<decltype(c)::value>), dim3((np + 63) / 64, (np + 3) / 4), dim3(256), 0,
                         stream_, dXp.get(), dXp.get(), np, np, d, np, var, phi, S.get());
    });
    if (gK_ > 0)
      hipLaunchKernelGGL(add_grouped_cross_kernel, dim3((np + 63) / 64, (np + 3) / 4), dim3(256), 0, stream_, np, np, np,
                         gK_, g_plev_, g_plev_, gt, S.get());
    gemm(stream_, np, np, n, -1., T.get(), ld, 1, T.get(), ld, 0, 1., S.get(), np);
    HIP_CHECK(hipMemcpyAsync(pcov, S.get(), sizeof(double) * np * np, hipMemcpyDeviceToHost, stream_));
  }
  CheckInfo();
  double gvar = 0.;   // every grouped effect adds its variance to the prior variance of a prediction point
  for (int k = 0; k < gK_; ++k) gvar += g_tau_[k];
  if (want_var)
    for (int p = 0; p < np; ++p) pvar[p] = var + gvar - pvar[p];
}

void DenseSolver::CheckInfo() {
  int info = 0;
  HIP_CHECK(hipMemcpyAsync(&info, info_.get(), sizeof(int), hipMemcpyDeviceToHost, stream_));
  HIP_CHECK(hipStreamSynchronize(stream_));
  if (info != 0) Fatal("the covariance matrix is not positive definite (Cholesky failed)");
}

void DenseSolver::Gram(int cov_type, double var, double phi, const double* Z, int c, double* G) {
  // [X | y]^T Psi^-1 [X | y] = (W Z)^T (W Z), W = L^-1 (CalcXTPsiInvX, re_model_template.h:9125-9132)
  const int n = n_, ld = ld_;
  Factor(cov_type, var, phi);
  DevBuf<double> dZ((size_t)ld * c), WZ((size_t)ld * c), dG((size_t)c * c);
  HIP_CHECK(hipMemsetAsync(dZ.get(), 0, sizeof(double) * dZ.size(), stream_));
  HIP_CHECK(hipMemcpy2DAsync(dZ.get(), sizeof(double) * ld, Z, sizeof(double) * n, sizeof(double) * n, c,
                             hipMemcpyHostToDevice, stream_));
  gemm(stream_, n, c, n, 1., W_.get(), ld, 0, dZ.get(), ld, 0, 0., WZ.get(), ld, 0, 1, 0, 0);
  gemm(stream_, c, c, n, 1., WZ.get(), ld, 1, WZ.get(), ld, 0, 0., dG.get(), c);
  HIP_CHECK(hipMemcpyAsync(G, dG.get(), sizeof(double) * c * c, hipMemcpyDeviceToHost, stream_));
  CheckInfo();
}

void DenseSolver::PsiInvDiag(int cov_type, double var, double phi, const double* d_y, double* yaux, double* diag) {
  const int n = n_, ld = ld_;
  Factor(cov_type, var, phi);
  double* W = W_.get();
  double* z = vec_.get();
  double* ya = z + ld;
  double* partial = z + 2 * (size_t)ld;
  DevBuf<double> dg(n);
  const int nb = (n + 255) / 256;
  hipLaunchKernelGGL(trmv_lower_partial_kernel, dim3(nb, nb), dim3(256), 0, stream_, W, ld, n, d_y, partial);
  hipLaunchKernelGGL(trmv_lower_reduce_kernel, dim3(nb), dim3(256), 0, stream_, partial, n, z);
  hipLaunchKernelGGL(trmv_lower_t_kernel, dim3((n + 3) / 4), dim3(256), 0, stream_, W, ld, n, z, ya);
  hipLaunchKernelGGL(colnorm2_lower_kernel, dim3((n + 3) / 4), dim3(256), 0, stream_, W, ld, n, dg.get());
  HIP_CHECK(hipGetLastError());
  HIP_CHECK(hipMemcpyAsync(yaux, ya, sizeof(double) * n, hipMemcpyDeviceToHost, stream_));
  HIP_CHECK(hipMemcpyAsync(diag, dg.get(), sizeof(double) * n, hipMemcpyDeviceToHost, stream_));
  CheckInfo();
}

}  // namespace gpb_amd
