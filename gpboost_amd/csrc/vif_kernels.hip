// Full-scale Vecchia approximation (vif.h gives the model and the reference lines). Per evaluation
// (n points, m inducing points, nn neighbours, ld ldm):
//   low-rank part   K_mn, K_mm, L = chol(K_mm,s), V = L^-1 K_mn                  FitcSolver::Prior (MFMA GEMM)
//   derivatives     A = K_mm,s^-1 K_mn, P_k = L^-1 (dK_mn,k - 1/2 dK_mm,k A)       four MFMA GEMMs
//   residual rows   per point: the Gram blocks V_S^T V_S, V_S^T P_k,S of its neighbour set S through LDS,
//                   the residual covariances, one Cholesky + 3 solves             vif_rows_kernel (one WG / row)
//   Woodbury        BK = B K_mn^T (sparse over m-vectors), M = K_mm,s + BK^T D^-1 BK  split-K MFMA Gram
//   y_aux, traces   B / B^T vector products, m-vector solves with the inverse Cholesky factor, column dots
// The gradient's m x m traces come from tr(M^-1 X^T Y) = sum_i (M^-1 X_i) . Y_i with M^-1 X formed by
// one MFMA GEMM per matrix (re_model_template.h:2041-2079 forms the m x m products instead).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <limits>
#include <cstdlib>
#include <string>
#include <type_traits>

#include "cov.h"
#include "dense.h"
#include "fitc.h"
#include "latent_kernels.h"
#include "kernels.h"
#include "vif.h"

namespace gpb_amd {
namespace {

constexpr int kT = 256;
constexpr int kCh = 32;      // m-rows per LDS staging chunk in the row kernel
constexpr int kMaxNn = 64;        // neighbours per row without derivatives (prediction rows; LDS of the row kernel)
constexpr int kMaxNnGrad = 48;    // with the two derivative blocks (the likelihood's rows)
constexpr int kNv = 16;      // n-vector scratch slots
constexpr int kMv = 12;      // m-vector scratch slots

template <class F>
void dispatch_cov_vif(int cov, F&& f) {
  switch (cov) {
    case kMatern05: f(std::integral_constant<int, kMatern05>{}); break;
    case kMatern15: f(std::integral_constant<int, kMatern15>{}); break;
    case kMatern25: f(std::integral_constant<int, kMatern25>{}); break;
    case kGaussian: f(std::integral_constant<int, kGaussian>{}); break;
    default: Fatal("unsupported covariance type %d", cov);
  }
}

__device__ __forceinline__ double wsum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// LDS ordering among the lanes of one wave (its LDS operations execute in order; the fences keep the
// compiler from moving them across)
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ double dist_pts(const double* X, int d, int a, int b) {
  double s = 0.;
  for (int q = 0; q < d; ++q) {
    const double t = X[(size_t)a * d + q] - X[(size_t)b * d + q];
    s += t * t;
  }
  return sqrt(s);
}

// Work item of block b in a grid of 8 * chunk blocks: without an order the block index itself; with one, the
// blocks dealt to one XCD (b, b + 8, ...: the hardware's round-robin) take one contiguous run of the spatial
// (Morton) order, so the neighbour columns the rows gather stay in that XCD's L2. -1: padding block.
__device__ __forceinline__ int vif_row_slot(const int* ord, int chunk, int nitems) {
  const int b = blockIdx.x;
  if (!ord) return b;
  const int pos = (b & 7) * chunk + (b >> 3);
  return pos < nitems ? ord[pos] : -1;
}

// In-place Cholesky of the k x k matrix C (row stride ld, lower) by one wave, row-oriented (left-looking):
// step j forms L_jj from row j's dot product, then every lane t > j forms L_tj = (C_tj - L_t . L_j) / L_jj
// from its own row; the dot products read rows written in earlier steps only, so their LDS loads pipeline.
__device__ __forceinline__ void wave_chol(double* C, int ld, int k, int lane) {
  for (int j = 0; j < k; ++j) {
    if (lane == j) {
      double sacc = C[j * ld + j];
      for (int q = 0; q < j; ++q) sacc -= C[j * ld + q] * C[j * ld + q];
      C[j * ld + j] = sqrt(sacc);
    }
    wave_sync();
    if (lane > j && lane < k) {
      double sacc = C[lane * ld + j];
      for (int q = 0; q < j; ++q) sacc -= C[lane * ld + q] * C[j * ld + q];
      C[lane * ld + j] = sacc / C[j * ld + j];
    }
    wave_sync();
  }
}

// dK_mn / dlog(phi) (m x n, ld ldm)
template <int COV>
__global__ void __launch_bounds__(kT) vif_dkmn_kernel(const double* __restrict__ X, const double* __restrict__ Z, int n,
                                                     int m, int d, int ldm, double var, double phi,
                                                     double* __restrict__ dK) {
  const int j = blockIdx.x * 64 + (threadIdx.x & 63);
  const int i = blockIdx.y * 4 + (threadIdx.x >> 6);
  if (i >= n || j >= m) return;
  double s = 0.;
  for (int q = 0; q < d; ++q) {
    const double t = X[(size_t)i * d + q] - Z[(size_t)j * d + q];
    s += t * t;
  }
  double c, dc;
  cov_dcov<COV>(sqrt(s), var, phi, c, dc);
  dK[(size_t)j + (size_t)i * ldm] = dc;
}

struct VifRowsArgs {
  const double* X;
  const int* nbr;
  int n, d, nn, mi, ldm;
  const double* V;
  const double* P0;
  const double* P1;
  double var, phi;
  int r1;   // doubles of the staging / residual-matrix region
  int i0;   // first row (prediction rows follow the n observed points); nbr / Bv / D are indexed by i - i0
  double nugget;   // 1 (Gaussian likelihood, transformed scale) or 0 (latent form of the non-Gaussian likelihoods)
  double cjit;     // multiplier of the neighbour matrix's diagonal: 1, or JITTER_MULT_VECCHIA without a nugget
  const int* ord;   // nullable: rows in spatial order, processed XCD-chunked (vif_row_slot)
  int chunk;        // ceil(rows / 8) with ord
  double* Bv;
  double* D;
  double* dBv0;
  double* dBv1;
  double* dD0;
  double* dD1;
};

// Residual Vecchia row i (Vecchia_utils.cpp:1405-1617, full_scale_vecchia branches), transformed scale:
//   C = k(N, N) + I - V_N^T V_N,  c = k(N, i) - V_N^T V_i,  d0 = 1 + var - |V_i|^2
//   A = C^-1 c,  B(i, N) = -A,  D_i = d0 - A . c
// and per parameter k (log var, log phi), with P_k = L^-1 (dK_k - 1/2 dK_mm,k A) so that
// dK_a . A_b + A_a . (dK_b - dK_mm A_b) = V_a . P_b + P_a . V_b:
//   dC = dk(N, N) - (G + G^T),  dc = dk(N, i) - (V_N . P_i + P_N . V_i),  dd0 = [k = var] var - 2 V_i . P_i
//   dA = C^-1 (dc - dC A),  dB(i, N) = -dA,  dD_i = dd0 - (dA . c + A . dc)
// One 256-thread workgroup per row: the Gram blocks of the neighbour set S = N + {i} accumulate over
// m-chunks staged in LDS; then one wave factors the k x k matrix and solves (right-hand sides in
// registers, pivots broadcast by lane shuffles).
template <int COV, bool GRAD>
__global__ void __launch_bounds__(kT) vif_rows_kernel(VifRowsArgs a) {
  extern __shared__ double lds[];
  __shared__ int idx[kMaxNn + 1];
  __shared__ double vecs[4][kMaxNn];   // c, dc0, dc1, A
  __shared__ double scal[4];
  constexpr int G = GRAD ? 3 : 1;
  const int ir = vif_row_slot(a.ord, a.chunk, a.n - a.i0), tid = threadIdx.x;
  if (ir < 0) return;
  const int i = a.i0 + ir;
  const int nn = a.nn, k = min(i, nn), S = k + 1;
  if (tid < k) idx[tid] = a.nbr[(size_t)ir * nn + tid];
  if (tid == k) idx[k] = i;
  double* st = lds;            // staging [g][q][a] (kCh x Sp each), later C, dC0, dC1 (k x k each)
  double* gram = lds + a.r1;   // [g][a][b] = V_a . M^g_b, S x S each
  // Gram blocks in 4 x 4 register tiles (8 LDS reads per 16 FMAs); the staging rows are padded to
  // Sp = round_up(S, 4) + 2 doubles so that the tiles of one wave fall on distinct banks
  const int Sp = ((S + 3) & ~3) + 2, T4 = (S + 3) >> 2, NT = G * T4 * T4;
  for (int t = tid; t < G * kCh * (Sp - S); t += kT) {
    const int w = Sp - S;
    const int gq = t / w;
    st[gq * Sp + S + (t - gq * w)] = 0.;
  }
  __syncthreads();
  double acc[2][16];
#pragma unroll
  for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
    for (int j = 0; j < 16; ++j) acc[s2][j] = 0.;
  for (int q0 = 0; q0 < a.mi; q0 += kCh) {
    const int tot = G * S * kCh;
    for (int t = tid; t < tot; t += kT) {
      const int g = t / (S * kCh);
      const int r = t - g * S * kCh;
      const int p = r / kCh;
      const int q = r - p * kCh;
      const double* M = g == 0 ? a.V : (g == 1 ? a.P0 : a.P1);
      st[(g * kCh + q) * Sp + p] = q0 + q < a.mi ? M[(size_t)idx[p] * a.ldm + q0 + q] : 0.;
    }
    __syncthreads();
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      const int tile = tid + s2 * kT;
      if (tile < NT) {
        const int g = tile / (T4 * T4);
        const int r = tile - g * T4 * T4;
        const int pa = r / T4, pb = r - pa * T4;
        const double* L = st + 4 * pa;
        const double* R = st + (size_t)g * kCh * Sp + 4 * pb;
        for (int q = 0; q < kCh; ++q) {
          const double l0 = L[q * Sp], l1 = L[q * Sp + 1], l2 = L[q * Sp + 2], l3 = L[q * Sp + 3];
          const double r0 = R[q * Sp], r1 = R[q * Sp + 1], r2 = R[q * Sp + 2], r3 = R[q * Sp + 3];
          acc[s2][0] = fma(l0, r0, acc[s2][0]);
          acc[s2][1] = fma(l0, r1, acc[s2][1]);
          acc[s2][2] = fma(l0, r2, acc[s2][2]);
          acc[s2][3] = fma(l0, r3, acc[s2][3]);
          acc[s2][4] = fma(l1, r0, acc[s2][4]);
          acc[s2][5] = fma(l1, r1, acc[s2][5]);
          acc[s2][6] = fma(l1, r2, acc[s2][6]);
          acc[s2][7] = fma(l1, r3, acc[s2][7]);
          acc[s2][8] = fma(l2, r0, acc[s2][8]);
          acc[s2][9] = fma(l2, r1, acc[s2][9]);
          acc[s2][10] = fma(l2, r2, acc[s2][10]);
          acc[s2][11] = fma(l2, r3, acc[s2][11]);
          acc[s2][12] = fma(l3, r0, acc[s2][12]);
          acc[s2][13] = fma(l3, r1, acc[s2][13]);
          acc[s2][14] = fma(l3, r2, acc[s2][14]);
          acc[s2][15] = fma(l3, r3, acc[s2][15]);
        }
      }
    }
    __syncthreads();
  }
#pragma unroll
  for (int s2 = 0; s2 < 2; ++s2) {
    const int tile = tid + s2 * kT;
    if (tile < NT) {
      const int g = tile / (T4 * T4);
      const int r = tile - g * T4 * T4;
      const int pa = r / T4, pb = r - pa * T4;
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const int p = 4 * pa + (j >> 2), b = 4 * pb + (j & 3);
        if (p < S && b < S) gram[g * S * S + p * S + b] = acc[s2][j];
      }
    }
  }
  __syncthreads();
  const int SS = S * S;
  double* C = st;
  double* dC0 = st + k * k;
  double* dC1 = st + 2 * k * k;
  for (int e = tid; e < k * k; e += kT) {
    const int p = e / k, b = e - p * k;
    double c = a.var, dc = 0.;
    if (p != b) cov_dcov<COV>(dist_pts(a.X, a.d, idx[p], idx[b]), a.var, a.phi, c, dc);
    C[e] = p == b ? (a.nugget + c - gram[p * S + b]) * a.cjit : c - gram[p * S + b];
    if (GRAD) {
      dC0[e] = c - (gram[SS + p * S + b] + gram[SS + b * S + p]);
      dC1[e] = dc - (gram[2 * SS + p * S + b] + gram[2 * SS + b * S + p]);
    }
  }
  for (int p = tid; p < k; p += kT) {
    double c, dc;
    cov_dcov<COV>(dist_pts(a.X, a.d, idx[p], i), a.var, a.phi, c, dc);
    vecs[0][p] = c - gram[p * S + k];
    if (GRAD) {
      vecs[1][p] = c - (gram[SS + p * S + k] + gram[SS + k * S + p]);
      vecs[2][p] = dc - (gram[2 * SS + p * S + k] + gram[2 * SS + k * S + p]);
    }
  }
  if (tid == 0) {
    scal[0] = a.nugget + a.var - gram[k * S + k];
    if (GRAD) {
      scal[1] = a.var - 2. * gram[SS + k * S + k];
      scal[2] = -2. * gram[2 * SS + k * S + k];
    }
  }
  __syncthreads();
  // From here one wave: the Cholesky factor in LDS (lane = row), the right-hand sides in registers with
  // the pivot entries broadcast by lane shuffles; wave-scope ordering instead of workgroup barriers.
  if (tid >= 64) return;
  const int lane = tid;
  wave_chol(C, k, k, lane);
  // L L^T x = b for the lane-distributed right-hand sides x[0 .. NR)
  auto solve = [&](double* x, int nr) {
    for (int j = 0; j < k; ++j) {
      const double ljj = C[j * k + j];
      const double lij = lane < k ? C[lane * k + j] : 0.;
      for (int r = 0; r < nr; ++r) {
        const double xj = __shfl(x[r], j, 64) / ljj;
        if (lane == j) x[r] = xj;
        else if (lane > j) x[r] -= lij * xj;
      }
    }
    for (int j = k - 1; j >= 0; --j) {
      const double ljj = C[j * k + j];
      const double lji = lane < j ? C[j * k + lane] : 0.;
      for (int r = 0; r < nr; ++r) {
        const double xj = __shfl(x[r], j, 64) / ljj;
        if (lane == j) x[r] = xj;
        else if (lane < j) x[r] -= lji * xj;
      }
    }
  };
  double xa[1] = {lane < k ? vecs[0][lane] : 0.};
  solve(xa, 1);   // A
  double xd[2] = {0., 0.};
  if (GRAD) {
    // r_k = dc_k - dC_k A, then dA_k = C^-1 r_k
    if (lane < k) vecs[3][lane] = xa[0];
    wave_sync();
    if (lane < k) {
      double r0 = vecs[1][lane], r1 = vecs[2][lane];
      for (int b = 0; b < k; ++b) {
        const double ab = vecs[3][b];
        r0 -= dC0[lane * k + b] * ab;
        r1 -= dC1[lane * k + b] * ab;
      }
      xd[0] = r0;
      xd[1] = r1;
    }
    solve(xd, 2);
  }
  {
    // D_i = d0 - A . c; dD_k = dd0_k - (dA_k . c + A . dc_k) (wave sums in a fixed order)
    const int p = lane;
    double s0 = 0., s1 = 0., s2 = 0.;
    if (p < k) {
      s0 = xa[0] * vecs[0][p];
      if (GRAD) {
        s1 = xd[0] * vecs[0][p] + xa[0] * vecs[1][p];
        s2 = xd[1] * vecs[0][p] + xa[0] * vecs[2][p];
      }
    }
    s0 = wsum(s0);
    if (GRAD) {
      s1 = wsum(s1);
      s2 = wsum(s2);
    }
    const size_t row = (size_t)ir * nn;
    if (p < nn) {
      a.Bv[row + p] = p < k ? -xa[0] : 0.;
      if (GRAD) {
        a.dBv0[row + p] = p < k ? -xd[0] : 0.;
        a.dBv1[row + p] = p < k ? -xd[1] : 0.;
      }
    }
    if (p == 0) {
      a.D[ir] = scal[0] - s0;
      if (GRAD) {
        a.dD0[ir] = scal[1] - s1;
        a.dD1[ir] = scal[2] - s2;
      }
    }
  }
}

typedef double vif_double4 __attribute__((ext_vector_type(4)));
typedef double vif_double2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ double readlane_d(double v, int l) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), l);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), l);
  return __hiloint2double(hi, lo);
}

// (row, column) of entry e of a lower triangle stored row by row (e < 528)
__device__ __forceinline__ void tri_rc(int e, int& p, int& b) {
  p = (int)((sqrtf(8.f * (float)e + 1.f) - 1.f) * 0.5f);
  if ((p + 1) * (p + 2) / 2 <= e) ++p;
  if (p * (p + 1) / 2 > e) --p;
  b = e - p * (p + 1) / 2;
}

// The same row factor for neighbour sets of at most 32 points (nn <= 31, the reference's default 30) with
// the Gram blocks on the fp64 MFMA: one wave per row, V_S^T [V P_0 P_1]_S as 16x16x4 tiles. The m-range is
// walked in chunks of 8: lane (kq, m0) loads entries 2 kq, 2 kq + 1 of the chunk of columns S[m0] and
// S[16 + m0] as one 16-byte load per matrix (the k-slot kq of MFMA step e takes entry 2 kq + e; any
// assignment of the m entries to k-slots gives the same Gram), the next chunk's loads are issued before the
// current chunk's MFMAs, no branches in the loop (the tail chunk reads the zero-masked padding of the ld-m
// column). V^T V is symmetric: its (1, 0) block is stored from the transposed (0, 1) accumulator (11 MFMAs
// per k-step with the derivative blocks). LDS: the V^T V block becomes the residual matrix C in place (lower
// triangle); one scratch matrix takes G_1 = V^T P_0, then G_2 = V^T P_1 for the transposed sums, and finally
// dC_0 (lower triangle) and dC_1 (upper triangle, diagonal in column 32): two 32 x 33 matrices per wave.
template <int COV, bool GRAD>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2))) vif_rows_mfma_kernel(VifRowsArgs a) {
  constexpr int LD = 33;   // row stride of the 32 x 32 blocks
  constexpr int G = GRAD ? 3 : 1;
  __shared__ double C[32 * LD];
  __shared__ double X[GRAD ? 32 * LD : 1];
  __shared__ int idx[32];
  __shared__ double vecs[3][32];   // c, dc0, dc1
  __shared__ double rdg[32];       // 1 / L_jj
  const int ir = vif_row_slot(a.ord, a.chunk, a.n - a.i0), lane = threadIdx.x;
  if (ir < 0) return;
  const int i = a.i0 + ir;
  const int nn = a.nn, k = min(i, nn);
  if (lane < 32) idx[lane] = lane < k ? a.nbr[(size_t)ir * nn + lane] : i;
  wave_sync();
  const int m0 = lane & 15, kq = lane >> 4;
  const size_t o0 = (size_t)idx[m0] * a.ldm + 2 * kq, o1 = (size_t)idx[16 + m0] * a.ldm + 2 * kq;
  vif_double4 acc[G][2][2];
#pragma unroll
  for (int g = 0; g < G; ++g)
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
      for (int y = 0; y < 2; ++y) acc[g][x][y] = vif_double4{0., 0., 0., 0.};
  typedef vif_double2 Buf[G][2];
  auto load = [&](Buf& buf, int ch) {
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const double* M = g == 0 ? a.V : (g == 1 ? a.P0 : a.P1);
      buf[g][0] = *reinterpret_cast<const vif_double2*>(M + o0 + 8 * ch);
      buf[g][1] = *reinterpret_cast<const vif_double2*>(M + o1 + 8 * ch);
    }
  };
  auto step = [&](Buf& buf) {
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const double v0 = buf[0][0][e], v1 = buf[0][1][e];
      acc[0][0][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(v0, v0, acc[0][0][0], 0, 0, 0);
      acc[0][0][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(v0, v1, acc[0][0][1], 0, 0, 0);
      acc[0][1][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(v1, v1, acc[0][1][1], 0, 0, 0);
#pragma unroll
      for (int g = 1; g < G; ++g) {
        const double p0 = buf[g][0][e], p1 = buf[g][1][e];
        acc[g][0][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(v0, p0, acc[g][0][0], 0, 0, 0);
        acc[g][0][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(v0, p1, acc[g][0][1], 0, 0, 0);
        acc[g][1][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(v1, p0, acc[g][1][0], 0, 0, 0);
        acc[g][1][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(v1, p1, acc[g][1][1], 0, 0, 0);
      }
    }
  };
  auto mask = [&](Buf& buf, int ch) {   // entries beyond m: the column's padding (ld m is a multiple of 64), zeroed
    const int q = 8 * ch + 2 * kq;
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
      for (int x = 0; x < 2; ++x)
#pragma unroll
        for (int e = 0; e < 2; ++e)
          if (q + e >= a.mi) buf[g][x][e] = 0.;
  };
  // ping-pong over two register buffers (no copies): chunk ch + 1 is in flight while chunk ch is multiplied
  const int nch = (a.mi + 7) >> 3, nfull = a.mi >> 3;
  Buf cur, nxt;
  load(cur, 0);
  int ch = 0;
  for (; ch + 1 < nfull; ch += 2) {
    load(nxt, ch + 1);
    step(cur);
    load(cur, min(ch + 2, nch - 1));
    step(nxt);
  }
  if (ch < nfull) {   // odd number of full chunks: cur holds the last one
    if (ch + 1 < nch) load(nxt, ch + 1);
    step(cur);
    if (ch + 1 < nch) {
      mask(nxt, ch + 1);
      step(nxt);
    }
  } else if (ch < nch) {   // cur holds the tail chunk
    mask(cur, ch);
    step(cur);
  }
  // C/D layout: row = (lane >> 4) + 4 r, col = lane & 15 within each 16 x 16 tile
  auto store = [&](double* W, const vif_double4 (&t)[2][2], bool sym) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      W[(kq + 4 * r) * LD + m0] = t[0][0][r];
      W[(kq + 4 * r) * LD + 16 + m0] = t[0][1][r];
      W[(16 + kq + 4 * r) * LD + 16 + m0] = t[1][1][r];
      if (sym) W[(16 + m0) * LD + kq + 4 * r] = t[0][1][r];
      else W[(16 + kq + 4 * r) * LD + m0] = t[1][0][r];
    }
  };
  store(C, acc[0], true);
  if (GRAD) store(X, acc[GRAD ? 1 : 0], false);
  wave_sync();
  const double var = a.var, phi = a.phi;
  // c, dc_k (column k of the blocks) and the diagonal terms, before C overwrites the V^T V block
  double cs = 0., dcs = 0., d0 = 0., dd0 = 0., dd1 = 0.;
  if (lane < k) {
    cov_dcov<COV>(dist_pts(a.X, a.d, idx[lane], i), var, phi, cs, dcs);
    vecs[0][lane] = cs - C[lane * LD + k];
    if (GRAD) vecs[1][lane] = cs - (X[lane * LD + k] + X[k * LD + lane]);
  }
  d0 = a.nugget + var - C[k * LD + k];
  if (GRAD) dd0 = var - 2. * X[k * LD + k];
  // the lower triangle of C in place; dC_0 and the base derivative covariances in registers
  const int nl = k * (k + 1) / 2;
  double dv0[8], dcv[8];
#pragma unroll
  for (int t = 0; t < 8; ++t) {
    const int e = lane + 64 * t;
    dv0[t] = 0.;
    dcv[t] = 0.;
    if (e < nl) {
      int p, b;
      tri_rc(e, p, b);
      double c = var, dc = 0.;
      if (p != b) cov_dcov<COV>(dist_pts(a.X, a.d, idx[p], idx[b]), var, phi, c, dc);
      C[p * LD + b] = p == b ? (a.nugget + c - C[p * LD + b]) * a.cjit : c - C[p * LD + b];
      if (GRAD) {
        dv0[t] = c - (X[p * LD + b] + X[b * LD + p]);
        dcv[t] = dc;
      }
    }
  }
  wave_sync();
  if (GRAD) {
    store(X, acc[GRAD ? 2 : 0], false);
    wave_sync();
    if (lane < k) vecs[2][lane] = dcs - (X[lane * LD + k] + X[k * LD + lane]);
    dd1 = -2. * X[k * LD + k];
    double dv1[8];
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      const int e = lane + 64 * t;
      dv1[t] = 0.;
      if (e < nl) {
        int p, b;
        tri_rc(e, p, b);
        dv1[t] = dcv[t] - (X[p * LD + b] + X[b * LD + p]);
      }
    }
    wave_sync();
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      const int e = lane + 64 * t;
      if (e < nl) {
        int p, b;
        tri_rc(e, p, b);
        X[p * LD + b] = dv0[t];
        X[p == b ? p * LD + 32 : b * LD + p] = dv1[t];
      }
    }
  }
  wave_sync();
  // Cholesky of C in registers, right-looking: lane p < 32 holds row p (lower part; the rows / columns >= k padded
  // with the identity, so all 32 steps run unconditionally), the column entries L(c, j) broadcast by readlane
  const int pl = min(lane, 31);
  double rw[32];
#pragma unroll
  for (int c = 0; c < 32; ++c) {
    const double v = C[pl * LD + c];
    rw[c] = (lane < k && c < k) ? (c <= lane ? v : 0.) : (c == lane ? 1. : 0.);
  }
  // pivot j: y = 1 / sqrt(p) by the hardware estimate and two Newton steps, L_jj = p y, the column scaled by y
  // (multiplies instead of a square root and a division on the pivot chain; y is also the solves' 1 / L_jj)
  double yd = 1.;
#pragma unroll
  for (int j = 0; j < 32; ++j) {
    const double p = readlane_d(rw[j], j), h = 0.5 * p;
    double y = __builtin_amdgcn_rsq(p);
    y = y * fma(-h * y, y, 1.5);
    y = y * fma(-h * y, y, 1.5);
    rw[j] = lane > j ? rw[j] * y : (lane == j ? p * y : 0.);
    yd = lane == j ? y : yd;
#pragma unroll
    for (int c = j + 1; c < 32; ++c) rw[c] = fma(-rw[j], readlane_d(rw[j], c), rw[c]);
  }
  // the factor's rows back to LDS (the backward sweep reads its columns), 1 / L_jj
#pragma unroll
  for (int c = 0; c < 32; ++c)
    if (lane < 32) C[lane * LD + c] = rw[c];
  if (lane < 32) rdg[lane] = yd;
  wave_sync();
  // L L^T x = b for lane-distributed right-hand sides (lane p holds entry p; zero beyond k)
  auto solve = [&](double* x, int nr) {
#pragma unroll
    for (int j = 0; j < 32; ++j) {
      const double rjj = rdg[j];
      for (int r = 0; r < nr; ++r) {
        const double xj = readlane_d(x[r], j) * rjj;
        x[r] = lane == j ? xj : (lane > j ? fma(-rw[j], xj, x[r]) : x[r]);
      }
    }
#pragma unroll
    for (int j = 31; j >= 0; --j) {
      const double rjj = rdg[j];
      const double lji = C[j * LD + pl];   // L(j, lane), used for lane < j
      for (int r = 0; r < nr; ++r) {
        const double xj = readlane_d(x[r], j) * rjj;
        x[r] = lane == j ? xj : (lane < j ? fma(-lji, xj, x[r]) : x[r]);
      }
    }
  };
  double xa[1] = {lane < k ? vecs[0][lane] : 0.};
  solve(xa, 1);
  double xd[2] = {0., 0.};
  if (GRAD) {
    // r_k = dc_k - dC_k A (dC_0 from the lower triangle of X, dC_1 from the upper one, both symmetric; A_b by readlane)
    double r0 = lane < k ? vecs[1][lane] : 0., r1 = lane < k ? vecs[2][lane] : 0.;
#pragma unroll
    for (int b = 0; b < 32; ++b) {
      if (b < k) {
        const double ab = readlane_d(xa[0], b);
        const double u = X[pl * LD + b], w = X[b * LD + pl];
        const double e0 = b <= lane ? u : w;
        const double e1 = b < lane ? w : (b > lane ? u : X[pl * LD + 32]);
        r0 = fma(-e0, ab, r0);
        r1 = fma(-e1, ab, r1);
      }
    }
    xd[0] = lane < k ? r0 : 0.;
    xd[1] = lane < k ? r1 : 0.;
    solve(xd, 2);
  }
  double s0 = 0., s1 = 0., s2 = 0.;
  if (lane < k) {
    s0 = xa[0] * vecs[0][lane];
    if (GRAD) {
      s1 = xd[0] * vecs[0][lane] + xa[0] * vecs[1][lane];
      s2 = xd[1] * vecs[0][lane] + xa[0] * vecs[2][lane];
    }
  }
  s0 = wsum(s0);
  if (GRAD) {
    s1 = wsum(s1);
    s2 = wsum(s2);
  }
  const size_t row = (size_t)ir * nn;
  if (lane < nn) {
    a.Bv[row + lane] = lane < k ? -xa[0] : 0.;
    if (GRAD) {
      a.dBv0[row + lane] = lane < k ? -xd[0] : 0.;
      a.dBv1[row + lane] = lane < k ? -xd[1] : 0.;
    }
  }
  if (lane == 0) {
    a.D[ir] = d0 - s0;
    if (GRAD) {
      a.dD0[ir] = dd0 - s1;
      a.dD1[ir] = dd1 - s2;
    }
  }
}

// out[:, i] = (self in[:, i] + sum_r coef[i nn + r] in[:, nbr[i nn + r]]) (/ D_i); out2 (nullable) gets
// the same column divided by D_i: one wave per column (i wave-uniform: the neighbour list and the coefficients are
// scalar loads), lane l holds entries 4 l .. 4 l + 3 of a 256-entry slice (two 16-byte loads per neighbour; ld m
// is a multiple of 64, so the slice stays inside the column; entries >= m are not stored)
__device__ __forceinline__ void vif_store4(double* dst, int q, int m, vif_double2 a, vif_double2 b) {
  if (q + 3 < m) {
    reinterpret_cast<vif_double2*>(dst + q)[0] = a;
    reinterpret_cast<vif_double2*>(dst + q)[1] = b;
  } else {
    if (q < m) dst[q] = a[0];
    if (q + 1 < m) dst[q + 1] = a[1];
    if (q + 2 < m) dst[q + 2] = b[0];
  }
}

__global__ void __launch_bounds__(kT) vif_brow_kernel(const double* __restrict__ in, const int* __restrict__ nbr,
                                                     const double* __restrict__ coef, const double* __restrict__ D,
                                                     int n, int nn, int m, int ldm, double self, int div,
                                                     double* __restrict__ out, double* __restrict__ out2,
                                                     const int* __restrict__ ord, int chunk) {
  const int lane = threadIdx.x & 63;
  const int b = ord ? (blockIdx.x & 7) * chunk + (blockIdx.x >> 3) : blockIdx.x;
  int i = b * 4 + (threadIdx.x >> 6);
  if (i >= n) return;
  if (ord) i = ord[i];
  i = __builtin_amdgcn_readfirstlane(i);
  const int k = min(i, nn);
  const int* nb = nbr + (size_t)i * nn;
  const double* cf = coef + (size_t)i * nn;
  const double inv = (div || out2) ? 1. / D[i] : 1.;
  for (int q = 4 * lane; q < m; q += 256) {
    vif_double2 s0 = {0., 0.}, s1 = {0., 0.};
    if (self != 0.) {
      const vif_double2* src = reinterpret_cast<const vif_double2*>(in + (size_t)i * ldm + q);
      s0 = self * src[0];
      s1 = self * src[1];
    }
#pragma unroll 8
    for (int r = 0; r < k; ++r) {
      const double c = cf[r];
      const vif_double2* src = reinterpret_cast<const vif_double2*>(in + (size_t)nb[r] * ldm + q);
      const vif_double2 x0 = src[0], x1 = src[1];
      s0[0] = fma(c, x0[0], s0[0]);
      s0[1] = fma(c, x0[1], s0[1]);
      s1[0] = fma(c, x1[0], s1[0]);
      s1[1] = fma(c, x1[1], s1[1]);
    }
    const vif_double2 d0 = s0 * inv, d1 = s1 * inv;
    if (div) vif_store4(out + (size_t)i * ldm, q, m, d0, d1);
    else vif_store4(out + (size_t)i * ldm, q, m, s0, s1);
    if (out2) vif_store4(out2 + (size_t)i * ldm, q, m, d0, d1);
  }
}

// out[:, j] = self in[:, j] + sum over rows i with j among their neighbours of coef(i, j) in[:, i] (coefT: the
// factor's values in column order), the same wave / lane layout
__global__ void __launch_bounds__(kT) vif_bcol_kernel(const double* __restrict__ in, const int* __restrict__ tptr,
                                                     const int* __restrict__ trow, const double* __restrict__ coefT,
                                                     int n, int m, int ldm, double self, double* __restrict__ out,
                                                     const int* __restrict__ ord, int chunk) {
  const int lane = threadIdx.x & 63;
  const int b = ord ? (blockIdx.x & 7) * chunk + (blockIdx.x >> 3) : blockIdx.x;
  int j = b * 4 + (threadIdx.x >> 6);
  if (j >= n) return;
  if (ord) j = ord[j];
  j = __builtin_amdgcn_readfirstlane(j);
  const int t0 = tptr[j], t1 = tptr[j + 1];
  for (int q = 4 * lane; q < m; q += 256) {
    vif_double2 s0 = {0., 0.}, s1 = {0., 0.};
    if (self != 0.) {
      const vif_double2* src = reinterpret_cast<const vif_double2*>(in + (size_t)j * ldm + q);
      s0 = self * src[0];
      s1 = self * src[1];
    }
#pragma unroll 8
    for (int t = t0; t < t1; ++t) {
      const double c = coefT[t];
      const vif_double2* src = reinterpret_cast<const vif_double2*>(in + (size_t)trow[t] * ldm + q);
      const vif_double2 x0 = src[0], x1 = src[1];
      s0[0] = fma(c, x0[0], s0[0]);
      s0[1] = fma(c, x0[1], s0[1]);
      s1[0] = fma(c, x1[0], s1[0]);
      s1[1] = fma(c, x1[1], s1[1]);
    }
    vif_store4(out + (size_t)j * ldm, q, m, s0, s1);
  }
}

__global__ void __launch_bounds__(kT) vif_bvec_kernel(const double* __restrict__ x, const int* __restrict__ nbr,
                                                     const double* __restrict__ coef, const double* __restrict__ D,
                                                     int n, int nn, double self, double* __restrict__ out) {
  const int i = blockIdx.x * kT + threadIdx.x;
  if (i >= n) return;
  const int k = min(i, nn);
  double s = self != 0. ? self * x[i] : 0.;
  for (int r = 0; r < k; ++r) s = fma(coef[(size_t)i * nn + r], x[nbr[(size_t)i * nn + r]], s);
  out[i] = D ? s / D[i] : s;
}

// out_j = self x_j + sum over column j's entries of coefT[t] x[trow[t]] (coefT: the values in column order):
// 16 lanes per column stride its entry list (contiguous trow / coefT reads), fixed-order shuffle sum
__global__ void __launch_bounds__(kT) vif_btvec_kernel(const double* __restrict__ x, const int* __restrict__ tptr,
                                                      const int* __restrict__ trow, const double* __restrict__ coefT,
                                                      int n, double self, double* __restrict__ out) {
  const int sub = threadIdx.x & 15;
  const int j = blockIdx.x * (kT / 16) + (threadIdx.x >> 4);
  if (j >= n) return;
  double s = 0.;
  for (int t = tptr[j] + sub; t < tptr[j + 1]; t += 16) s = fma(coefT[t], x[trow[t]], s);
#pragma unroll
  for (int o = 8; o > 0; o >>= 1) s += __shfl_xor(s, o, 16);
  if (sub == 0) out[j] = self != 0. ? fma(self, x[j], s) : s;
}

// coefT[t] = coef[tslot[t]] (the row-major factor values in column order)
__global__ void __launch_bounds__(kT) vif_gather_kernel(int nnz, const int* __restrict__ tslot,
                                                       const double* __restrict__ coef, double* __restrict__ coefT) {
  const int t = blockIdx.x * kT + threadIdx.x;
  if (t < nnz) coefT[t] = coef[tslot[t]];
}

// part[b ldm + j] = sum_{i in chunk b} M[j, i] x_i
__global__ void __launch_bounds__(kT) vif_gemv_part_kernel(const double* __restrict__ M, const double* __restrict__ x,
                                                          int n, int m, int ldm, double* __restrict__ part) {
  const int i0 = blockIdx.x * 64, i1 = min(n, i0 + 64);
  for (int j = threadIdx.x; j < m; j += kT) {
    double acc = 0.;
    for (int i = i0; i < i1; ++i) acc = fma(M[(size_t)i * ldm + j], x[i], acc);
    part[(size_t)blockIdx.x * ldm + j] = acc;
  }
}

__global__ void __launch_bounds__(kT) vif_gemv_reduce_kernel(const double* __restrict__ part, int nb, int m, int ldm,
                                                            double* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int j = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (j >= m) return;
  double s = 0.;
  for (int b = lane; b < nb; b += 64) s += part[(size_t)b * ldm + j];
  s = wsum(s);
  if (lane == 0) out[j] = s;
}

// out_i = M[:, i] . w (w != nullptr) or M[:, i] . M2[:, i]
__global__ void __launch_bounds__(kT) vif_coldot_kernel(const double* __restrict__ M, const double* __restrict__ w,
                                                       const double* __restrict__ M2, int n, int m, int ldm,
                                                       double* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (i >= n) return;
  double s = 0.;
  for (int q = lane; q < m; q += 64) s = fma(M[(size_t)i * ldm + q], w ? w[q] : M2[(size_t)i * ldm + q], s);
  s = wsum(s);
  if (lane == 0) out[i] = s;
}

// z_i = (-dD_i u_i + e_i) / D_i
__global__ void __launch_bounds__(kT) vif_zvec_kernel(int n, const double* __restrict__ dD, const double* __restrict__ u,
                                                     const double* __restrict__ e, const double* __restrict__ D,
                                                     double* __restrict__ z) {
  const int i = blockIdx.x * kT + threadIdx.x;
  if (i >= n) return;
  z[i] = (e[i] - dD[i] * u[i]) / D[i];
}

__global__ void __launch_bounds__(kT) vif_add_kernel(int n, const double* __restrict__ a, const double* __restrict__ b,
                                                    double* __restrict__ out) {
  const int i = blockIdx.x * kT + threadIdx.x;
  if (i < n) out[i] = a[i] + b[i];
}

__global__ void __launch_bounds__(kT) vif_sub_kernel(int n, const double* __restrict__ a, const double* __restrict__ b,
                                                    double* __restrict__ out) {
  const int i = blockIdx.x * kT + threadIdx.x;
  if (i < n) out[i] = a[i] - b[i];
}

// Per-block partial sums of up to 8 elementwise terms; op 0: a (b) (c) (nullable factors), 1: log a,
// 2: a (b) / c, 3: a b^2 / c^2, 4: a b / c^2
struct VifTerms {
  const double* a[8];
  const double* b[8];
  const double* c[8];
  int op[8];
};

__global__ void __launch_bounds__(kT) vif_sum_kernel(int n, int nt, VifTerms T, double* __restrict__ part) {
  __shared__ double red[kT / 64][8];
  double acc[8];
#pragma unroll
  for (int t = 0; t < 8; ++t) acc[t] = 0.;
  for (int i = blockIdx.x * kT + threadIdx.x; i < n; i += gridDim.x * kT) {
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      if (t >= nt) break;
      const double av = T.a[t][i];
      const double bv = T.b[t] ? T.b[t][i] : 1.;
      const double cv = T.c[t] ? T.c[t][i] : 1.;
      double v;
      switch (T.op[t]) {
        case 1: v = log(av); break;
        case 2: v = av * bv / cv; break;
        case 3: v = av * bv * bv / (cv * cv); break;
        case 4: v = av * bv / (cv * cv); break;
        default: v = av * bv * cv;
      }
      acc[t] += v;
    }
  }
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
#pragma unroll
  for (int t = 0; t < 8; ++t) {
    if (t >= nt) break;
    const double s = wsum(acc[t]);
    if (lane == 0) red[w][t] = s;
  }
  __syncthreads();
  if (threadIdx.x < nt) {
    const int t = threadIdx.x;
    part[(size_t)blockIdx.x * nt + t] = (red[0][t] + red[1][t]) + (red[2][t] + red[3][t]);
  }
}

// staging / residual-matrix region (doubles) for neighbour sets of up to nn + 1 points
int rows_r1(int nn, bool grad) {
  const int G = grad ? 3 : 1, S = nn + 1, Sp = ((S + 3) & ~3) + 2;
  return std::max(G * kCh * Sp, G * nn * nn);
}

size_t rows_lds_bytes(int nn, bool grad) {
  const int G = grad ? 3 : 1, S = nn + 1;
  return sizeof(double) * ((size_t)rows_r1(nn, grad) + (size_t)G * S * S);
}

// Prediction rows (full_scale_vecchia): mo_p = sum over observed neighbours of B(p, j) r_j (the Bpo r of the
// mean) and column p of Q^T = (Bpo K_nm)^T, one wave per prediction point (Vecchia_utils.cpp:1904, 1917-1921)
__global__ void __launch_bounds__(64) vif_pred_bpo_kernel(int np, int n, int mp, const int* __restrict__ nbr,
                                                          const double* __restrict__ Bv, const double* __restrict__ r,
                                                          const double* __restrict__ Kmn, int m, int ldm,
                                                          double* __restrict__ mo, double* __restrict__ Qt) {
  const int p = blockIdx.x, lane = threadIdx.x;
  const int* nb = nbr + (size_t)p * mp;
  const double* bv = Bv + (size_t)p * mp;
  double s = 0.;
  for (int j = lane; j < mp; j += 64)
    if (nb[j] >= 0 && nb[j] < n) s = fma(bv[j], r[nb[j]], s);
  s = wsum(s);
  if (lane == 0) mo[p] = s;
  for (int q = lane; q < m; q += 64) {
    double t = 0.;
    for (int j = 0; j < mp; ++j)
      if (nb[j] >= 0 && nb[j] < n) t = fma(bv[j], Kmn[(size_t)nb[j] * ldm + q], t);
    Qt[(size_t)p * ldm + q] = t;
  }
}

// var_p = (KP - PPV + 2 Q)_p . Sig_p + (PPV - 2 Q)_p . S2_p + Q_p . S3_p (Vecchia_utils.cpp:1966-1973), columns
// of m x np matrices (ld ldm)
__global__ void __launch_bounds__(kT) vif_pred_var_kernel(int np, int m, int ldm, const double* __restrict__ KP,
                                                          const double* __restrict__ PPV, const double* __restrict__ Q,
                                                          const double* __restrict__ Sig, const double* __restrict__ S2,
                                                          const double* __restrict__ S3, double* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int p = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (p >= np) return;
  const size_t o = (size_t)p * ldm;
  double s = 0.;
  for (int q = lane; q < m; q += 64) {
    const double kp = KP[o + q], pv = PPV[o + q], qq = Q[o + q];
    s += (kp - pv + 2. * qq) * Sig[o + q] + (pv - 2. * qq) * S2[o + q] + qq * S3[o + q];
  }
  s = wsum(s);
  if (lane == 0) out[p] = s;
}

__global__ void __launch_bounds__(kT) vif_sum_parts_kernel(const double* __restrict__ part, int chunks, long stride,
                                                           int m, int ldm, double* __restrict__ out) {
  const int q = blockIdx.x * kT + threadIdx.x;
  if (q >= m * m) return;
  const int i = q % m, j = q / m;
  double s = 0.;
  for (int c = 0; c < chunks; ++c) s += part[(size_t)c * stride + i + (size_t)j * ldm];
  out[i + (size_t)j * ldm] = s;
}

}  // namespace

VifSolver::VifSolver(int n, int d, const double* d_X, const std::vector<double>& Z, const std::vector<int>& nbr, int nn,
                     hipStream_t stream)
    : n_(n), d_(d), nn_(nn), s_(stream), d_X_(d_X) {
  if (nn < 1) Fatal("full_scale_vecchia needs num_neighbors >= 1");
  if (nn > kMaxNnGrad)
    Fatal("num_neighbors = %d > %d is not supported for gp_approx = 'full_scale_vecchia' by gpboost_amd", nn, kMaxNnGrad);
  if ((long)nbr.size() != (long)n * nn) Fatal("VifSolver: neighbour lists of the wrong size");
  F_.reset(new FitcSolver(n, d, d_X, Z, stream));
  m_ = F_->m_;
  ldm_ = F_->ldm_;
  const size_t mn = (size_t)ldm_ * n;
  for (DevBuf<double>* b : {&dK_, &P0_, &P1_, &BK_}) b->alloc(mn);
  for (DevBuf<double>* b : {&Bv_, &dBv0_, &dBv1_}) b->alloc((size_t)n * nn);
  for (DevBuf<double>* b : {&D_, &dD0_, &dD1_}) b->alloc(n);
  vec_.alloc((size_t)kNv * n);
  mvec_.alloc((size_t)kMv * ldm_);
  HIP_CHECK(hipMemsetAsync(mvec_.get(), 0, sizeof(double) * kMv * ldm_, stream));
  const int nbg = (n + 63) / 64, nbs = 512;
  part_.alloc(std::max<size_t>((size_t)nbg * ldm_, (size_t)nbs * 8));
  red_.alloc(64);
  HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&h_red_), 64 * sizeof(double), hipHostMallocDefault));
  nbr_.alloc((size_t)n * nn);
  HIP_CHECK(hipMemcpyAsync(nbr_.get(), nbr.data(), sizeof(int) * nbr.size(), hipMemcpyHostToDevice, stream));
  // B^T lists: for every column j the rows i (ascending) that hold j among their neighbours, with the slot
  std::vector<int> tptr(n + 1, 0);
  for (int i = 0; i < n; ++i)
    for (int r = 0; r < std::min(i, nn); ++r) ++tptr[nbr[(size_t)i * nn + r] + 1];
  for (int j = 0; j < n; ++j) tptr[j + 1] += tptr[j];
  const int nnz = tptr[n];
  std::vector<int> trow(std::max(nnz, 1)), tslot(std::max(nnz, 1)), fill(tptr.begin(), tptr.end() - 1);
  for (int i = 0; i < n; ++i)
    for (int r = 0; r < std::min(i, nn); ++r) {
      const int j = nbr[(size_t)i * nn + r];
      trow[fill[j]] = i;
      tslot[fill[j]] = i * nn + r;
      ++fill[j];
    }
  nnz_ = nnz;
  for (DevBuf<double>* b : {&BvT_, &dBvT0_, &dBvT1_}) b->alloc(std::max(nnz, 1));
  tptr_.alloc(n + 1);
  trow_.alloc(trow.size());
  tslot_.alloc(tslot.size());
  HIP_CHECK(hipMemcpyAsync(tptr_.get(), tptr.data(), sizeof(int) * (n + 1), hipMemcpyHostToDevice, stream));
  HIP_CHECK(hipMemcpyAsync(trow_.get(), trow.data(), sizeof(int) * trow.size(), hipMemcpyHostToDevice, stream));
  HIP_CHECK(hipMemcpyAsync(tslot_.get(), tslot.data(), sizeof(int) * tslot.size(), hipMemcpyHostToDevice, stream));
  // processing order of the row and B-product kernels: the points along a Morton curve of their (first two)
  // coordinates, so that rows worked on together share neighbour columns in L2 (the results do not depend on
  // it: every row / column is computed by one wave); GPBOOST_AMD_VIF_ORDER=0 keeps the index order
  const char* ordenv = std::getenv("GPBOOST_AMD_VIF_ORDER");
  if (!(ordenv && std::string(ordenv) == "0") && n > 1) {
    std::vector<double> hx((size_t)n * d);
    HIP_CHECK(hipMemcpyAsync(hx.data(), d_X, sizeof(double) * hx.size(), hipMemcpyDeviceToHost, stream));
    HIP_CHECK(hipStreamSynchronize(stream));
    const int dd = std::min(d, 2);
    double lo[2] = {0., 0.}, hi[2] = {0., 0.};
    for (int q = 0; q < dd; ++q) {
      lo[q] = hi[q] = hx[q];
      for (int i = 0; i < n; ++i) {
        lo[q] = std::min(lo[q], hx[(size_t)i * d + q]);
        hi[q] = std::max(hi[q], hx[(size_t)i * d + q]);
      }
    }
    std::vector<std::pair<uint64_t, int>> key(n);
    for (int i = 0; i < n; ++i) {
      uint64_t code = 0;
      uint32_t c[2] = {0, 0};
      for (int q = 0; q < dd; ++q) {
        const double w = hi[q] > lo[q] ? (hx[(size_t)i * d + q] - lo[q]) / (hi[q] - lo[q]) : 0.;
        c[q] = (uint32_t)std::min(65535., std::max(0., w * 65536.));
      }
      for (int bit = 15; bit >= 0; --bit)
        for (int q = 0; q < dd; ++q) code = (code << 1) | ((c[q] >> bit) & 1u);
      key[i] = {code, i};
    }
    std::sort(key.begin(), key.end());
    std::vector<int> ord(n);
    for (int i = 0; i < n; ++i) ord[i] = key[i].second;
    ord_.alloc(n);
    HIP_CHECK(hipMemcpyAsync(ord_.get(), ord.data(), sizeof(int) * n, hipMemcpyHostToDevice, stream));
  }
  lds_bytes_ = rows_lds_bytes(nn, true);
  for (int cov : {kMatern05, kMatern15, kMatern25, kGaussian})
    dispatch_cov_vif(cov, [&](auto c) {
      constexpr int COV = decltype(c)::value;
      HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&vif_rows_kernel<COV, true>),
                                    hipFuncAttributeMaxDynamicSharedMemorySize, (int)rows_lds_bytes(nn, true)));
      HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&vif_rows_kernel<COV, false>),
                                    hipFuncAttributeMaxDynamicSharedMemorySize, (int)rows_lds_bytes(nn, false)));
    });
  for (auto& e : ev_) HIP_CHECK(hipEventCreate(&e));
  HIP_CHECK(hipStreamSynchronize(stream));
}

VifSolver::~VifSolver() {
  if (h_red_) (void)hipHostFree(h_red_);
  for (auto& e : ev_) if (e) (void)hipEventDestroy(e);
}

void VifSolver::Rows(int cov_type, double var, double phi, bool grad) {
  VifRowsArgs a{};
  a.X = d_X_;
  a.nbr = nbr_.get();
  a.n = n_; a.d = d_; a.nn = nn_; a.mi = m_; a.ldm = ldm_;
  a.V = F_->V_.get(); a.P0 = P0_.get(); a.P1 = P1_.get();
  a.var = var; a.phi = phi;
  a.nugget = latent_ ? 0. : 1.;
  a.cjit = latent_ ? 1. + 1e-10 : 1.;   // JITTER_MULT_VECCHIA (utils.h:36; Vecchia_utils.cpp:1546-1548)
  a.r1 = rows_r1(nn_, grad);
  a.Bv = Bv_.get(); a.D = D_.get(); a.dBv0 = dBv0_.get(); a.dBv1 = dBv1_.get(); a.dD0 = dD0_.get(); a.dD1 = dD1_.get();
  a.ord = ord_.size() ? ord_.get() : nullptr;
  a.chunk = (n_ + 7) / 8;
  const int grid = a.ord ? 8 * a.chunk : n_;
  const size_t lds = rows_lds_bytes(nn_, grad);
  const char* form = std::getenv("GPBOOST_AMD_VIF_ROWS");   // "lds": the LDS-staged VALU form (A/B)
  const bool lds_form = form != nullptr && std::string(form) == "lds";
  const bool mfma = nn_ <= 31 && !lds_form;   // neighbour sets of <= 32 points: the MFMA Gram form
  dispatch_cov_vif(cov_type, [&](auto c) {
    constexpr int COV = decltype(c)::value;
    if (mfma) {
      if (grad) hipLaunchKernelGGL((vif_rows_mfma_kernel<COV, true>), dim3(grid), dim3(64), 0, s_, a);
      else hipLaunchKernelGGL((vif_rows_mfma_kernel<COV, false>), dim3(grid), dim3(64), 0, s_, a);
    } else if (grad) {
      hipLaunchKernelGGL((vif_rows_kernel<COV, true>), dim3(grid), dim3(kT), lds, s_, a);
    } else {
      hipLaunchKernelGGL((vif_rows_kernel<COV, false>), dim3(grid), dim3(kT), lds, s_, a);
    }
  });
  HIP_CHECK(hipGetLastError());
}

void VifSolver::BRow(const double* in, const double* coef, double self, bool div, double* out, double* out_div) {
  const int* ord = ord_.size() ? ord_.get() : nullptr;
  const int nb = (n_ + 3) / 4, chunk = (nb + 7) / 8;
  hipLaunchKernelGGL(vif_brow_kernel, dim3(ord ? 8 * chunk : nb), dim3(kT), 0, s_, in, nbr_.get(), coef, D_.get(), n_,
                     nn_, m_, ldm_, self, div ? 1 : 0, out, out_div, ord, chunk);
  HIP_CHECK(hipGetLastError());
}

void VifSolver::BCol(const double* in, const double* coefT, double self, double* out) {
  const int* ord = ord_.size() ? ord_.get() : nullptr;
  const int nb = (n_ + 3) / 4, chunk = (nb + 7) / 8;
  hipLaunchKernelGGL(vif_bcol_kernel, dim3(ord ? 8 * chunk : nb), dim3(kT), 0, s_, in, tptr_.get(), trow_.get(),
                     coefT, n_, m_, ldm_, self, out, ord, chunk);
  HIP_CHECK(hipGetLastError());
}

void VifSolver::BVec(const double* x, const double* coef, double self, double* out) {
  hipLaunchKernelGGL(vif_bvec_kernel, dim3((n_ + kT - 1) / kT), dim3(kT), 0, s_, x, nbr_.get(), coef,
                     static_cast<const double*>(nullptr), n_, nn_, self, out);
  HIP_CHECK(hipGetLastError());
}

void VifSolver::BtVec(const double* x, const double* coefT, double self, double* out) {
  hipLaunchKernelGGL(vif_btvec_kernel, dim3((n_ + kT / 16 - 1) / (kT / 16)), dim3(kT), 0, s_, x, tptr_.get(),
                     trow_.get(), coefT, n_, self, out);
  HIP_CHECK(hipGetLastError());
}

void VifSolver::Gemv(const double* M, const double* x, double* out) {
  const int nb = (n_ + 63) / 64;
  hipLaunchKernelGGL(vif_gemv_part_kernel, dim3(nb), dim3(kT), 0, s_, M, x, n_, m_, ldm_, part_.get());
  hipLaunchKernelGGL(vif_gemv_reduce_kernel, dim3((m_ + 3) / 4), dim3(kT), 0, s_, part_.get(), nb, m_, ldm_, out);
  HIP_CHECK(hipGetLastError());
}

void VifSolver::PredBpo(int np, int mp, const int* dnb, const double* Bvp, const double* r, const double* M, double* mo,
                        double* Qt) {
  hipLaunchKernelGGL(vif_pred_bpo_kernel, dim3(np), dim3(64), 0, s_, np, n_, mp, dnb, Bvp, r, M, m_, ldm_, mo, Qt);
  HIP_CHECK(hipGetLastError());
}

void VifSolver::ColDotN(const double* M, const double* w, const double* M2, int cols, double* out) {
  hipLaunchKernelGGL(vif_coldot_kernel, dim3((cols + 3) / 4), dim3(kT), 0, s_, M, w, M2, cols, m_, ldm_, out);
  HIP_CHECK(hipGetLastError());
}

void VifSolver::ColDot(const double* M, const double* w, const double* M2, double* out) {
  hipLaunchKernelGGL(vif_coldot_kernel, dim3((n_ + 3) / 4), dim3(kT), 0, s_, M, w, M2, n_, m_, ldm_, out);
  HIP_CHECK(hipGetLastError());
}

void VifSolver::Prepare(int cov_type, double var, double phi, bool want_grad, double* red, double* M_copy) {
  FitcSolver& F = *F_;
  const int n = n_, m = m_, ldm = ldm_;
  const size_t mn = (size_t)ldm * n;
  // low-rank part (CalcSigmaComps): K_mn, K_mm, K_mm,s, dK_mm, L, L^-1, V = L^-1 K_mn, K_mm,s^-1; red[0] =
  // log det K_mm,s
  F.Prior(cov_type, var, phi, red);
  if (want_grad) {
    dispatch_cov_vif(cov_type, [&](auto c) {
      constexpr int COV = decltype(c)::value;
      hipLaunchKernelGGL((vif_dkmn_kernel<COV>), dim3((m + 63) / 64, (n + 3) / 4), dim3(kT), 0, s_, d_X_, F.dZ_.get(),
                         n, m, d_, ldm, var, phi, dK_.get());
    });
    HIP_CHECK(hipGetLastError());
    // A = L^-T V; P_0 = L^-1 (K_mn - 1/2 K_mm A), P_1 = L^-1 (dK_mn - 1/2 dK_mm A) (Kd_ as the staging)
    gemm_f64(s_, m, n, m, 1., F.Li_.get(), ldm, 1, F.V_.get(), ldm, 0, 0., F.A_.get(), ldm, 0, 0, 1, 0);
    HIP_CHECK(hipMemcpyAsync(F.Kd_.get(), F.Kmn_.get(), sizeof(double) * mn, hipMemcpyDeviceToDevice, s_));
    gemm_f64(s_, m, n, m, -0.5, F.Kmm_.get(), ldm, 0, F.A_.get(), ldm, 0, 1., F.Kd_.get(), ldm);
    gemm_f64(s_, m, n, m, 1., F.Li_.get(), ldm, 0, F.Kd_.get(), ldm, 0, 0., P0_.get(), ldm, 0, 1, 0, 0);
    HIP_CHECK(hipMemcpyAsync(F.Kd_.get(), dK_.get(), sizeof(double) * mn, hipMemcpyDeviceToDevice, s_));
    gemm_f64(s_, m, n, m, -0.5, F.dKmm_.get(), ldm, 0, F.A_.get(), ldm, 0, 1., F.Kd_.get(), ldm);
    gemm_f64(s_, m, n, m, 1., F.Li_.get(), ldm, 0, F.Kd_.get(), ldm, 0, 0., P1_.get(), ldm, 0, 1, 0, 0);
  }
  // residual Vecchia factor (CalcCovFactorGradientVecchia), its values also in column order for B^T
  Rows(cov_type, var, phi, want_grad);
  if (nnz_ > 0) {
    const int nbt = (nnz_ + kT - 1) / kT;
    hipLaunchKernelGGL(vif_gather_kernel, dim3(nbt), dim3(kT), 0, s_, nnz_, tslot_.get(), Bv_.get(), BvT_.get());
    if (want_grad) {
      hipLaunchKernelGGL(vif_gather_kernel, dim3(nbt), dim3(kT), 0, s_, nnz_, tslot_.get(), dBv0_.get(), dBvT0_.get());
      hipLaunchKernelGGL(vif_gather_kernel, dim3(nbt), dim3(kT), 0, s_, nnz_, tslot_.get(), dBv1_.get(), dBvT1_.get());
    }
    HIP_CHECK(hipGetLastError());
  }
  // Woodbury matrix M = K_mm,s + BK^T D^-1 BK (CalcCovFactorFITC_FSA): BK_ = B K, Kd_ = D^-1 B K
  BRow(F.Kmn_.get(), Bv_.get(), 1., false, BK_.get(), F.Kd_.get());
  const long mm = (long)ldm * ldm;
  const int chunks = gemm_f64_splitk(s_, m, m, n, BK_.get(), ldm, 0, F.Kd_.get(), ldm, 1, F.part_.get(), ldm, mm, 2048,
                                     F.max_chunks_);
  fitc_wsum(s_, F.part_.get(), chunks, mm, m, ldm, F.Ks_.get(), F.W_.get());
  if (M_copy != nullptr)
    HIP_CHECK(hipMemcpyAsync(M_copy, F.W_.get(), sizeof(double) * mm, hipMemcpyDeviceToDevice, s_));
  chol_lower(s_, F.W_.get(), F.Wi_.get(), m, ldm, F.info_.get());
  launch_logdet_chol(s_, F.W_.get(), ldm, m, red + 1);
  trtri_lower(s_, F.W_.get(), F.Wi_.get(), F.T_.get(), 0, m, ldm);
  fitc_lower_t(s_, F.Wi_.get(), m, ldm, F.WiT_.get());
}

void VifSolver::Eval(int cov_type, double var, double phi, const double* d_y, bool want_grad, double* sums,
                     double* kernel_ms) {
  if (latent_) Fatal("VifSolver::Eval is the Gaussian likelihood's evaluation (the model is latent)");
  FitcSolver& F = *F_;
  const int n = n_, m = m_, ldm = ldm_;
  double* red = red_.get();
  HIP_CHECK(hipEventRecord(ev_[0], s_));
  Prepare(cov_type, var, phi, want_grad, red);
  HIP_CHECK(hipEventRecord(ev_[1], s_));
  // y_aux = R^-1 y - R^-1 K M^-1 K^T R^-1 y with R^-1 = B^T D^-1 B (CalcYAux :8910-8925)
  double* v = vec_.get();
  double* u = v;                      // D^-1 B y (vecchia_y)
  double* ry = v + (size_t)n;         // R^-1 y
  double* kw = v + 2 * (size_t)n;     // K s
  double* t1 = v + 3 * (size_t)n;
  double* rk = v + 4 * (size_t)n;     // R^-1 K s
  double* yaux = v + 5 * (size_t)n;
  double* mv = mvec_.get();
  double* mt = mv;                    // K^T R^-1 y
  double* ms = mv + ldm;              // w = M^-1 K^T R^-1 y
  double* mtmp = mv + 2 * (size_t)ldm;
  hipLaunchKernelGGL(vif_bvec_kernel, dim3((n + kT - 1) / kT), dim3(kT), 0, s_, d_y, nbr_.get(), Bv_.get(), D_.get(), n,
                     nn_, 1., u);
  BtVec(u, BvT_.get(), 1., ry);
  Gemv(F.Kmn_.get(), ry, mt);
  fitc_chol_solve(s_, F.Wi_.get(), F.WiT_.get(), mt, m, ldm, mtmp, ms);
  ColDot(F.Kmn_.get(), ms, nullptr, kw);
  hipLaunchKernelGGL(vif_bvec_kernel, dim3((n + kT - 1) / kT), dim3(kT), 0, s_, kw, nbr_.get(), Bv_.get(), D_.get(), n,
                     nn_, 1., t1);
  BtVec(t1, BvT_.get(), 1., rk);
  hipLaunchKernelGGL(vif_sub_kernel, dim3((n + kT - 1) / kT), dim3(kT), 0, s_, n, ry, rk, yaux);
  HIP_CHECK(hipGetLastError());
  const int nbs = std::min(512, (n + kT - 1) / kT);
  {
    VifTerms T{};
    T.a[0] = D_.get(); T.op[0] = 1;                      // sum log D
    T.a[1] = d_y; T.b[1] = yaux; T.op[1] = 0;            // y^T y_aux
    hipLaunchKernelGGL(vif_sum_kernel, dim3(nbs), dim3(kT), 0, s_, n, 2, T, part_.get());
    launch_sum_blocks(part_.get(), nbs, 2, red + 2, s_);
  }
  double* mv_a = mv + 3 * (size_t)ldm;    // a = K_mm,s^-1 K^T y_aux
  double* mv_g[2] = {mv + 4 * (size_t)ldm, mv + 5 * (size_t)ldm};   // dK_k^T y_aux
  double* mv_k[2] = {mv + 6 * (size_t)ldm, mv + 7 * (size_t)ldm};   // K^T vgy_k
  if (want_grad) {
    // the gradient (CalcGradPars_FITC_FSA_GaussLikelihood_Cluster_i, re_model_template.h:1985-2232): M^-1 for
    // the m x m traces, then per parameter the quadratic and trace sums
    gemm_f64(s_, m, m, m, 1., F.Wi_.get(), ldm, 1, F.Wi_.get(), ldm, 0, 0., F.Winv_.get(), ldm, 0, 0, 1, 1);
    double* mt2 = mv + 8 * (size_t)ldm;
    Gemv(F.Kmn_.get(), yaux, mt2);
    fitc_chol_solve(s_, F.Li_.get(), F.LiT_.get(), mt2, m, ldm, mtmp, mv_a);
    HIP_CHECK(hipMemcpyAsync(mv_g[0], mt2, sizeof(double) * m, hipMemcpyDeviceToDevice, s_));
    Gemv(dK_.get(), yaux, mv_g[1]);
    for (int p = 0; p < 2; ++p)
      fitc_mm_terms(s_, F.Kinv_.get(), F.Winv_.get(), F.Kmm_.get(), p == 0 ? F.Kmm_.get() : F.dKmm_.get(), mv_a, m, ldm,
                    F.part_.get(), red + 8 + 6 * p);
    // X = B^T D^-1 B K (A_), Xw = M^-1 X (V_), Bw = M^-1 BK (P0_)
    BCol(F.Kd_.get(), BvT_.get(), 1., F.A_.get());
    gemm_f64(s_, m, n, m, 1., F.Winv_.get(), ldm, 0, F.A_.get(), ldm, 0, 0., F.V_.get(), ldm);
    gemm_f64(s_, m, n, m, 1., F.Winv_.get(), ldm, 0, BK_.get(), ldm, 0, 0., P0_.get(), ldm);
    double* bkw = v + 6 * (size_t)n;   // (B K w)_i
    double* cg = v + 7 * (size_t)n;    // BK_i . Bw_i
    ColDot(BK_.get(), ms, nullptr, bkw);
    ColDot(BK_.get(), nullptr, P0_.get(), cg);
    for (int p = 0; p < 2; ++p) {
      const double* dBv = p == 0 ? dBv0_.get() : dBv1_.get();
      const double* dD = p == 0 ? dD0_.get() : dD1_.get();
      double* dby = v + 8 * (size_t)n;
      double* zp = v + 9 * (size_t)n;
      double* btz = v + 10 * (size_t)n;
      double* vgy = v + 11 * (size_t)n;
      double* dbkw = v + 12 * (size_t)n;
      double* cxw = v + 13 * (size_t)n;
      double* cf = v + 14 * (size_t)n;
      // vecchia_grad_y = dB^T u - B^T D^-1 (dD o u) + B^T D^-1 dB y (:2084-2085)
      BVec(d_y, dBv, 0., dby);
      hipLaunchKernelGGL(vif_zvec_kernel, dim3((n + kT - 1) / kT), dim3(kT), 0, s_, n, dD, u, dby, D_.get(), zp);
      BtVec(zp, BvT_.get(), 1., btz);
      BtVec(u, p == 0 ? dBvT0_.get() : dBvT1_.get(), 0., vgy);
      hipLaunchKernelGGL(vif_add_kernel, dim3((n + kT - 1) / kT), dim3(kT), 0, s_, n, vgy, btz, vgy);
      HIP_CHECK(hipGetLastError());
      Gemv(F.Kmn_.get(), vgy, mv_k[p]);
      BVec(kw, dBv, 0., dbkw);                                             // dB K w
      ColDot(F.V_.get(), nullptr, p == 0 ? F.Kmn_.get() : dK_.get(), cxw);  // (M^-1 X_i) . dK_k,i
      BRow(F.Kmn_.get(), dBv, 0., false, P1_.get());                      // dB K
      ColDot(P1_.get(), nullptr, P0_.get(), cf);                           // (dB K)_i . (M^-1 BK)_i
      VifTerms T{};
      T.a[0] = d_y; T.b[0] = vgy; T.op[0] = 0;                      // y . vgy
      T.a[1] = dbkw; T.b[1] = bkw; T.c[1] = D_.get(); T.op[1] = 2;  // w^T F w
      T.a[2] = dD; T.b[2] = bkw; T.c[2] = D_.get(); T.op[2] = 3;    // sum dD (D^-1 BK w)^2
      T.a[3] = dD; T.c[3] = D_.get(); T.op[3] = 2;                  // sum dD / D
      T.a[4] = cxw; T.op[4] = 0;                                     // tr(M^-1 E)
      T.a[5] = cf; T.c[5] = D_.get(); T.op[5] = 2;                  // tr(M^-1 F)
      T.a[6] = dD; T.b[6] = cg; T.c[6] = D_.get(); T.op[6] = 4;     // tr(M^-1 G)
      hipLaunchKernelGGL(vif_sum_kernel, dim3(nbs), dim3(kT), 0, s_, n, 7, T, part_.get());
      launch_sum_blocks(part_.get(), nbs, 7, red + 20 + 8 * p, s_);
    }
  }
  HIP_CHECK(hipMemcpyAsync(h_red_, red, sizeof(double) * 36, hipMemcpyDeviceToHost, s_));
  std::vector<double> hm(want_grad ? (size_t)6 * m : 0);
  if (want_grad) {
    const double* srcs[6] = {mv_a, mv_g[0], mv_g[1], mv_k[0], mv_k[1], ms};
    for (int k = 0; k < 6; ++k)
      HIP_CHECK(hipMemcpyAsync(hm.data() + (size_t)k * m, srcs[k], sizeof(double) * m, hipMemcpyDeviceToHost, s_));
  }
  int info = 0;
  HIP_CHECK(hipMemcpyAsync(&info, F.info_.get(), sizeof(int), hipMemcpyDeviceToHost, s_));
  HIP_CHECK(hipEventRecord(ev_[2], s_));
  HIP_CHECK(hipStreamSynchronize(s_));
  float ms0 = 0.f, ms1 = 0.f;
  HIP_CHECK(hipEventElapsedTime(&ms0, ev_[0], ev_[1]));
  HIP_CHECK(hipEventElapsedTime(&ms1, ev_[0], ev_[2]));
  kernel_ms[0] = ms0;
  kernel_ms[1] = ms1;
  const double nan = std::numeric_limits<double>::quiet_NaN();
  if (info != 0) {
    for (int k = 0; k < 6; ++k) sums[k] = nan;
    return;
  }
  // log det Psi = log det M - log det K_mm,s + sum log D (re_model_template.h:2700-2710)
  sums[0] = h_red_[1] - h_red_[0] + h_red_[2];
  sums[1] = h_red_[3];
  if (!want_grad) {
    for (int k = 2; k < 6; ++k) sums[k] = nan;
    return;
  }
  auto dot = [&](int x, int y) {
    double s = 0.;
    for (int j = 0; j < m; ++j) s += hm[(size_t)x * m + j] * hm[(size_t)y * m + j];
    return s;
  };
  for (int p = 0; p < 2; ++p) {
    const double* mmt = h_red_ + 8 + 6 * p;   // [tr Kinv Kmm, tr Winv Kmm, tr Kinv dK_mm, tr Winv dK_mm, ., a dK_mm a]
    const double* g = h_red_ + 20 + 8 * p;
    // / error_var part (:2040-2041, 2086-2089)
    const double quad = 0.5 * mmt[5] - dot(1 + p, 0) + 0.5 * g[0] - dot(3 + p, 5) + g[1] - 0.5 * g[2];
    // trace part (:2037-2038, 2085, 2215-2218): -1/2 tr(K_mm,s^-1 dK_mm) + 1/2 sum dD / D + 1/2 tr(M^-1 dM)
    const double tr = -0.5 * mmt[2] + 0.5 * g[3] + 0.5 * (2. * g[4] + 2. * g[5] - g[6] + mmt[3]);
    sums[2 + p] = quad;
    sums[4 + p] = 2. * tr;
  }
}

void VifSolver::GetFactor(double* D, double* Bv) const {
  HIP_CHECK(hipMemcpyAsync(D, D_.get(), sizeof(double) * n_, hipMemcpyDeviceToHost, s_));
  HIP_CHECK(hipMemcpyAsync(Bv, Bv_.get(), sizeof(double) * n_ * nn_, hipMemcpyDeviceToHost, s_));
  HIP_CHECK(hipStreamSynchronize(s_));
}

// The prediction points' residual Vecchia rows (Vecchia_utils.cpp:1807-1896, no derivatives): KP = K_mp (m x np),
// Va = [V | V_p] with V_p = L^-1 K_mp (chol_ip_cross_cov_pred, :1698-1699), Bvp (np x mp), Dp (np) from the row
// kernel at the row offset n (the latent form without a nugget when latent_), dnb the neighbour lists on the device.
void VifSolver::PredRows(int cov_type, double var, double phi, const double* Xp, int np, const int* nbr, int mp,
                         DevBuf<double>& KP, DevBuf<double>& Va, DevBuf<double>& Bvp, DevBuf<double>& Dp,
                         DevBuf<int>& dnb) {
  if (mp < 1 || mp > kMaxNn) Fatal("num_neighbors_pred = %d is not supported for gp_approx = 'full_scale_vecchia' (1..%d)",
                                   mp, kMaxNn);
  FitcSolver& F = *F_;
  const int n = n_, m = m_, ldm = ldm_, d = d_;
  const int na = n + np;
  DevBuf<double> Xa((size_t)na * d);
  KP.alloc((size_t)ldm * np);
  Va.alloc((size_t)ldm * na);
  Bvp.alloc((size_t)np * mp);
  Dp.alloc(np);
  dnb.alloc((size_t)np * mp);
  HIP_CHECK(hipMemcpyAsync(Xa.get(), d_X_, sizeof(double) * (size_t)n * d, hipMemcpyDeviceToDevice, s_));
  HIP_CHECK(hipMemcpyAsync(Xa.get() + (size_t)n * d, Xp, sizeof(double) * (size_t)np * d, hipMemcpyHostToDevice, s_));
  HIP_CHECK(hipMemcpyAsync(dnb.get(), nbr, sizeof(int) * (size_t)np * mp, hipMemcpyHostToDevice, s_));
  HIP_CHECK(hipMemsetAsync(KP.get(), 0, sizeof(double) * KP.size(), s_));
  fitc_kmn(s_, cov_type, Xa.get() + (size_t)n * d, F.dZ_.get(), np, m, d, ldm, var, phi, KP.get());   // K_mp
  HIP_CHECK(hipMemcpyAsync(Va.get(), F.V_.get(), sizeof(double) * (size_t)ldm * n, hipMemcpyDeviceToDevice, s_));
  HIP_CHECK(hipMemsetAsync(Va.get() + (size_t)ldm * n, 0, sizeof(double) * (size_t)ldm * np, s_));
  gemm_f64(s_, m, np, m, 1., F.Li_.get(), ldm, 0, KP.get(), ldm, 0, 0., Va.get() + (size_t)ldm * n, ldm, 0, 1, 0, 0);
  VifRowsArgs a{};
  a.X = Xa.get();
  a.nbr = dnb.get();
  a.n = na; a.d = d; a.nn = mp; a.mi = m; a.ldm = ldm;
  a.V = Va.get(); a.P0 = nullptr; a.P1 = nullptr;
  a.var = var; a.phi = phi;
  a.nugget = latent_ ? 0. : 1.;
  a.cjit = latent_ ? 1. + 1e-10 : 1.;
  a.r1 = rows_r1(mp, false);
  a.i0 = n;
  a.Bv = Bvp.get(); a.D = Dp.get();
  const size_t lds = rows_lds_bytes(mp, false);
  dispatch_cov_vif(cov_type, [&](auto c) {
    constexpr int COV = decltype(c)::value;
    if (mp <= 31) {
      hipLaunchKernelGGL((vif_rows_mfma_kernel<COV, false>), dim3(np), dim3(64), 0, s_, a);
    } else {
      HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&vif_rows_kernel<COV, false>),
                                    hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
      hipLaunchKernelGGL((vif_rows_kernel<COV, false>), dim3(np), dim3(kT), lds, s_, a);
    }
  });
  HIP_CHECK(hipGetLastError());
}

void VifSolver::Predict(int cov_type, double var, double phi, const double* d_y, const double* Xp, int np,
                        const int* nbr, int mp, bool cond_all, double* mean, double* pvar, double* pcov) {
  if (np <= 0) return;
  if (mp < 1 || mp > kMaxNn) Fatal("num_neighbors_pred = %d is not supported for gp_approx = 'full_scale_vecchia' (1..%d)",
                                   mp, kMaxNn);
  if (cond_all && pcov != nullptr && np > 20000)
    Fatal("order_obs_first_cond_all with predict_cov_mat is limited to num_data_pred <= 20000 in gpboost_amd");
  FitcSolver& F = *F_;
  const int n = n_, m = m_, ldm = ldm_;
  double sums[6], kms[2];
  Eval(cov_type, var, phi, d_y, false, sums, kms);   // factor, Woodbury M, w = M^-1 K^T R^-1 y, kw = K w
  if (std::isnan(sums[0])) Fatal("full_scale_vecchia prediction: the Woodbury matrix is not positive definite");
  const double* w = mvec_.get() + ldm;
  const double* kw = vec_.get() + 2 * (size_t)n;
  DevBuf<double> KP, Va, Bvp, Dp, r(n), mo(np), Qt((size_t)ldm * np), kpw(np);
  DevBuf<int> dnb;
  PredRows(cov_type, var, phi, Xp, np, nbr, mp, KP, Va, Bvp, Dp, dnb);
  // mean = -Bpo (y - K w) [Bp^-1] + K_pm w (:1903-1908)
  hipLaunchKernelGGL(vif_sub_kernel, dim3((n + kT - 1) / kT), dim3(kT), 0, s_, n, d_y, kw, r.get());
  hipLaunchKernelGGL(vif_pred_bpo_kernel, dim3(np), dim3(64), 0, s_, np, n, mp, dnb.get(), Bvp.get(), r.get(),
                     F.Kmn_.get(), m, ldm, mo.get(), Qt.get());
  hipLaunchKernelGGL(vif_coldot_kernel, dim3((np + 3) / 4), dim3(kT), 0, s_, KP.get(), w,
                     static_cast<const double*>(nullptr), np, m, ldm, kpw.get());
  HIP_CHECK(hipGetLastError());
  std::vector<double> hmo(np), hkpw(np), hD(np), hB((size_t)np * mp);
  HIP_CHECK(hipMemcpyAsync(hmo.data(), mo.get(), sizeof(double) * np, hipMemcpyDeviceToHost, s_));
  HIP_CHECK(hipMemcpyAsync(hkpw.data(), kpw.get(), sizeof(double) * np, hipMemcpyDeviceToHost, s_));
  HIP_CHECK(hipMemcpyAsync(hD.data(), Dp.get(), sizeof(double) * np, hipMemcpyDeviceToHost, s_));
  HIP_CHECK(hipMemcpyAsync(hB.data(), Bvp.get(), sizeof(double) * hB.size(), hipMemcpyDeviceToHost, s_));
  HIP_CHECK(hipStreamSynchronize(s_));
  // Bp x = b (unit lower; its off-diagonal entries are the rows' values at earlier prediction points)
  auto bp_solve = [&](double* x, size_t stride, int width) {
    for (int p = 0; p < np; ++p)
      for (int j = 0; j < mp; ++j) {
        const int q = nbr[(size_t)p * mp + j];
        if (q < n) continue;
        const double b = hB[(size_t)p * mp + j];
        for (int c = 0; c < width; ++c) x[(size_t)p * stride + c] -= b * x[(size_t)(q - n) * stride + c];
      }
  };
  std::vector<double> mu(np);
  for (int p = 0; p < np; ++p) mu[p] = -hmo[p];
  if (cond_all) bp_solve(mu.data(), 1, 1);
  for (int p = 0; p < np; ++p) mean[p] = mu[p] + hkpw[p];
  if (pvar == nullptr && pcov == nullptr) return;
  // Bp^-1 (dense, cond_all) for the Bp^-1 Dp Bp^-T part and Bp^-1 (Bpo K) (:1935-1948)
  std::vector<double> Binv;
  if (cond_all) {
    Binv.assign((size_t)np * np, 0.);   // row-major: row p = e_p^T Bp^-1
    for (int p = 0; p < np; ++p) Binv[(size_t)p * np + p] = 1.;
    bp_solve(Binv.data(), np, np);
    std::vector<double> hQ((size_t)ldm * np);
    HIP_CHECK(hipMemcpyAsync(hQ.data(), Qt.get(), sizeof(double) * hQ.size(), hipMemcpyDeviceToHost, s_));
    HIP_CHECK(hipStreamSynchronize(s_));
    bp_solve(hQ.data(), ldm, m);   // rows of Q = columns of Q^T (ld ldm)
    HIP_CHECK(hipMemcpyAsync(Qt.get(), hQ.data(), sizeof(double) * hQ.size(), hipMemcpyHostToDevice, s_));
  }
  // G = V (B^T D^-1 B K_nm) (m x m; :1910-1915), PPV^T = G^T V_p; Sig = K_mm,s^-1 K_mp; M^-1 PPV^T, M^-1 Q^T
  BRow(F.Kmn_.get(), Bv_.get(), 1., false, BK_.get(), F.Kd_.get());
  BCol(F.Kd_.get(), BvT_.get(), 1., F.A_.get());
  const long mm = (long)ldm * ldm;
  const int chunks = gemm_f64_splitk(s_, m, m, n, F.V_.get(), ldm, 0, F.A_.get(), ldm, 1, F.part_.get(), ldm, mm, 2048,
                                     F.max_chunks_);
  DevBuf<double> G(mm), PPV((size_t)ldm * np), Sig((size_t)ldm * np), S2((size_t)ldm * np), S3((size_t)ldm * np);
  hipLaunchKernelGGL(vif_sum_parts_kernel, dim3((m * m + kT - 1) / kT), dim3(kT), 0, s_, F.part_.get(), chunks, mm, m,
                     ldm, G.get());
  HIP_CHECK(hipGetLastError());
  for (auto* b : {&PPV, &Sig, &S2, &S3}) HIP_CHECK(hipMemsetAsync(b->get(), 0, sizeof(double) * b->size(), s_));
  gemm_f64(s_, m, np, m, 1., G.get(), ldm, 1, Va.get() + (size_t)ldm * n, ldm, 0, 0., PPV.get(), ldm);
  gemm_f64(s_, m, np, m, 1., F.Kinv_.get(), ldm, 0, KP.get(), ldm, 0, 0., Sig.get(), ldm);
  gemm_f64(s_, m, m, m, 1., F.Wi_.get(), ldm, 1, F.Wi_.get(), ldm, 0, 0., F.Winv_.get(), ldm, 0, 0, 1, 1);   // M^-1
  gemm_f64(s_, m, np, m, 1., F.Winv_.get(), ldm, 0, PPV.get(), ldm, 0, 0., S2.get(), ldm);
  gemm_f64(s_, m, np, m, 1., F.Winv_.get(), ldm, 0, Qt.get(), ldm, 0, 0., S3.get(), ldm);
  if (pvar != nullptr) {
    DevBuf<double> dv(np);
    hipLaunchKernelGGL(vif_pred_var_kernel, dim3((np + 3) / 4), dim3(kT), 0, s_, np, m, ldm, KP.get(), PPV.get(),
                       Qt.get(), Sig.get(), S2.get(), S3.get(), dv.get());
    HIP_CHECK(hipGetLastError());
    HIP_CHECK(hipMemcpyAsync(pvar, dv.get(), sizeof(double) * np, hipMemcpyDeviceToHost, s_));
    HIP_CHECK(hipStreamSynchronize(s_));
    for (int p = 0; p < np; ++p) {
      double dpart = hD[p];
      if (cond_all) {
        dpart = 0.;
        for (int q = 0; q <= p; ++q) dpart += Binv[(size_t)p * np + q] * Binv[(size_t)p * np + q] * hD[q];
      }
      pvar[p] += dpart;
    }
  }
  if (pcov != nullptr) {
    // cov = [Bp^-1] Dp [Bp^-T] + (KP - PPV + Q)^T Sig + (PPV - Q)^T S2 + Q^T S3 + Sig^T Q - S2^T Q (:1956-1964)
    DevBuf<double> C((size_t)np * np), T1((size_t)ldm * np);
    HIP_CHECK(hipMemcpyAsync(T1.get(), KP.get(), sizeof(double) * T1.size(), hipMemcpyDeviceToDevice, s_));
    launch_axpby(T1.size(), -1., PPV.get(), 1., T1.get(), T1.get(), s_);
    launch_axpby(T1.size(), 1., Qt.get(), 1., T1.get(), T1.get(), s_);
    gemm_f64(s_, np, np, m, 1., T1.get(), ldm, 1, Sig.get(), ldm, 0, 0., C.get(), np);
    HIP_CHECK(hipMemcpyAsync(T1.get(), PPV.get(), sizeof(double) * T1.size(), hipMemcpyDeviceToDevice, s_));
    launch_axpby(T1.size(), -1., Qt.get(), 1., T1.get(), T1.get(), s_);
    gemm_f64(s_, np, np, m, 1., T1.get(), ldm, 1, S2.get(), ldm, 0, 1., C.get(), np);
    gemm_f64(s_, np, np, m, 1., Qt.get(), ldm, 1, S3.get(), ldm, 0, 1., C.get(), np);
    gemm_f64(s_, np, np, m, 1., Sig.get(), ldm, 1, Qt.get(), ldm, 0, 1., C.get(), np);
    gemm_f64(s_, np, np, m, -1., S2.get(), ldm, 1, Qt.get(), ldm, 0, 1., C.get(), np);
    if (cond_all) {   // + Bp^-1 Dp Bp^-T: the row-major Bp^-1 read column-major is X = Bp^-T, C += (D X)^T X
      std::vector<double> XD(Binv);
      for (int p = 0; p < np; ++p)
        for (int k = 0; k < np; ++k) XD[(size_t)p * np + k] *= hD[k];
      DevBuf<double> dX((size_t)np * np), dXD((size_t)np * np);
      HIP_CHECK(hipMemcpyAsync(dX.get(), Binv.data(), sizeof(double) * Binv.size(), hipMemcpyHostToDevice, s_));
      HIP_CHECK(hipMemcpyAsync(dXD.get(), XD.data(), sizeof(double) * XD.size(), hipMemcpyHostToDevice, s_));
      gemm_f64(s_, np, np, np, 1., dXD.get(), np, 1, dX.get(), np, 0, 1., C.get(), np);
      HIP_CHECK(hipMemcpyAsync(pcov, C.get(), sizeof(double) * C.size(), hipMemcpyDeviceToHost, s_));
      HIP_CHECK(hipStreamSynchronize(s_));
    } else {
      HIP_CHECK(hipMemcpyAsync(pcov, C.get(), sizeof(double) * C.size(), hipMemcpyDeviceToHost, s_));
      HIP_CHECK(hipStreamSynchronize(s_));
      for (int p = 0; p < np; ++p) pcov[(size_t)p * np + p] += hD[p];
    }
  }
}

}  // namespace gpb_amd
