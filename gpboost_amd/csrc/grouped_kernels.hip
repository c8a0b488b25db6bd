// Device kernels of the grouped-random-effects engine (grouped.h).
//
// Blocks of t vectors are row-major M x t (one RE row = t contiguous doubles). Every product with
// a part of A = Sigma^-1 + Z^T Z (the matrix-vector product, the SSOR triangular solves, the probe
// transform) is a two-phase pass over precomputed entry chunks: phase 1 gives one workgroup to a
// chunk of one row's entries — tc lanes span the columns (a neighbour row's t values are one
// coalesced 8t-byte gather), 256 / tc lanes split the chunk's entries — and writes the chunk's
// partial sum (fixed-order LDS tree); phase 2 gives one thread to each (row, column), adds the
// row's chunk partials in chunk order and applies the operation's diagonal / solve formula. Rows of
// crossed effects have very different lengths (config 4: ~90 entries for a level of the 5000-level
// effect, ~900 for one of the 500-level effect); chunking makes the work per workgroup uniform
// and gives the chip tens of thousands of workgroups instead of one wave per (long) row. Results
// are deterministic (no atomics); they differ from the reference's sequential Eigen sums only by
// summation order.
#include <hip/hip_runtime.h>

#include "common.h"
#include "grouped_kernels.h"

namespace gpb_amd {
namespace {

constexpr int kEntriesPerLane = 8;

// Phase 1: P[q * t + c] = sum_{e in chunk q} coef_e X[col_e, c], coef_e = val_e (SCALE = false) or
// val_e sqrt(1/D_{col_e}) (SCALE = true: the L D^-1/2 factor of the SSOR preconditioner).
template <int TC, bool SCALE>
__global__ void __launch_bounds__(256) gre_chunk_kernel(const int* __restrict__ ce0, const int* __restrict__ ce1,
                                                        int chunk0, const int* __restrict__ col,
                                                        const double* __restrict__ val, const double* __restrict__ dis,
                                                        const double* __restrict__ X, int t, double* __restrict__ P) {
  constexpr int EG = 256 / TC;
  __shared__ double red[EG][TC];
  const int q = chunk0 + blockIdx.x;
  const int lc = threadIdx.x % TC;
  const int g = threadIdx.x / TC;
  const int c = blockIdx.y * TC + lc;
  double s = 0.;
  if (c < t) {
    const int e1 = ce1[q];
    for (int e = ce0[q] + g; e < e1; e += EG) {
      const int j = col[e];
      const double coef = SCALE ? val[e] * dis[j] : val[e];
      s += coef * X[(size_t)j * t + c];
    }
  }
  red[g][lc] = s;
  __syncthreads();
#pragma unroll
  for (int off = EG / 2; off > 0; off >>= 1) {
    if (g < off) red[g][lc] += red[g + off][lc];
    __syncthreads();
  }
  if (g == 0 && c < t) P[(size_t)q * t + c] = red[0][lc];
}

enum GreCombine : int {
  kCombApply = 0,   // Y = s + dg_r X_r
  kCombFwd,         // X_r = (R_r - s) / (D_r dis_r)            (lower solve)
  kCombBwd,         // Z_r = (X_r - dis_r s) / (D_r dis_r)      (upper solve of the transpose)
  kCombLds,         // Y = s + D_r dis_r R_r                    (probe transform)
  kCombUpper,       // Y = (1 / D_r) (D_r X_r + s)             (variance reduction)
};

// Phase 2 over rows [row0, row1): s = the row's chunk partials in chunk order, then the formula.
// In: the operation's own input (X for apply/upper, R for fwd/lds, X for bwd); Out: its output.
template <int OP>
__global__ void __launch_bounds__(256) gre_combine_kernel(int row0, int row1, int t, const int* __restrict__ ptr,
                                                          const double* __restrict__ P, const double* __restrict__ dg,
                                                          const double* __restrict__ dis,
                                                          const double* __restrict__ In, double* __restrict__ Out) {
  const size_t idx = (size_t)blockIdx.x * 256 + threadIdx.x;
  const size_t total = (size_t)(row1 - row0) * t;
  if (idx >= total) return;
  const int r = row0 + (int)(idx / t);
  const int c = (int)(idx % t);
  double s = 0.;
  for (int q = ptr[r]; q < ptr[r + 1]; ++q) s += P[(size_t)q * t + c];
  const size_t o = (size_t)r * t + c;
  if (OP == kCombApply) {
    Out[o] = s + dg[r] * In[o];
  } else if (OP == kCombFwd) {
    Out[o] = (In[o] - s) / (dg[r] * dis[r]);
  } else if (OP == kCombBwd) {
    Out[o] = (In[o] - dis[r] * s) / (dg[r] * dis[r]);
  } else if (OP == kCombLds) {
    Out[o] = s + (dg[r] * dis[r]) * In[o];
  } else {
    Out[o] = (1. / dg[r]) * (dg[r] * In[o] + s);
  }
}

// Z^T y: one wave per RE level, lanes stride its observations, fixed-order butterfly.
__global__ void __launch_bounds__(256) gre_zty_kernel(int M, const int* __restrict__ obs_ptr,
                                                      const int* __restrict__ obs, const double* __restrict__ y,
                                                      double* __restrict__ zty) {
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (r >= M) return;
  double s = 0.;
  for (int e = obs_ptr[r] + lane; e < obs_ptr[r + 1]; e += 64) s += y[obs[e]];
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
  if (lane == 0) zty[r] = s;
}

// Per effect k (one workgroup each): D_r = 1/tau_k + cnt_r, dis_r = sqrt(1/D_r) (the reference's
// P_SSOR_D_inv_.cwiseSqrt()), and the fixed-order sums out[k] = sum log D, out[K + k] = sum 1/D.
__global__ void __launch_bounds__(256) gre_diag_kernel(int K, const int* __restrict__ cum, const double* __restrict__ cnt,
                                                       const double* __restrict__ tau, double* __restrict__ D,
                                                       double* __restrict__ dis, double* __restrict__ out) {
  __shared__ double red[2][256];
  const int k = blockIdx.x;
  const double sinv = 1. / tau[k];
  double sl = 0., si = 0.;
  for (int r = cum[k] + threadIdx.x; r < cum[k + 1]; r += 256) {
    const double d = sinv + cnt[r];
    const double di = 1. / d;
    D[r] = d;
    dis[r] = sqrt(di);
    sl += log(d);
    si += di;
  }
  red[0][threadIdx.x] = sl;
  red[1][threadIdx.x] = si;
  __syncthreads();
  for (int off = 128; off > 0; off >>= 1) {
    if ((int)threadIdx.x < off) {
      red[0][threadIdx.x] += red[0][threadIdx.x + off];
      red[1][threadIdx.x] += red[1][threadIdx.x + off];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    out[k] = red[0][0];
    out[K + k] = red[1][0];
  }
}

// One grouping variable (A diagonal, re_model_template.h:8967-8969, 2279-2296): u = zty / D and the
// fixed-order sums out[0] = sum cnt (= n), out[1] = sum cnt^2 / D (= ||L^-1 Z^T Z||_F^2); one workgroup.
__global__ void __launch_bounds__(256) gre_single_kernel(int M, const double* __restrict__ zty,
                                                         const double* __restrict__ cnt, const double* __restrict__ D,
                                                         double* __restrict__ u, double* __restrict__ out) {
  __shared__ double red[2][256];
  double s0 = 0., s1 = 0.;
  for (int r = threadIdx.x; r < M; r += 256) {
    const double d = D[r], c = cnt[r];
    u[r] = zty[r] / d;
    s0 += c;
    s1 += c * c / d;
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
    out[0] = red[0][0];
    out[1] = red[1][0];
  }
}

// R = RHS - A U (warm-started PCG, CG_utils.cpp:1140-1143): V already holds A U
__global__ void __launch_bounds__(256) gre_residual_kernel(size_t count, const double* __restrict__ rhs,
                                                           const double* __restrict__ V, double* __restrict__ R) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i < count) R[i] = rhs[i] - V[i];
}

template <bool SCALE>
void chunk_pass(const GroupedOp& op, const GreChunks& ch, int q0, int q1, const double* dis, const double* X, int t,
                hipStream_t s) {
  if (q1 <= q0) return;
  const dim3 grid(q1 - q0, (t + op.tc - 1) / op.tc);
#define GRE_CHUNK_CASE(TCV)                                                                                         \
  case TCV:                                                                                                         \
    hipLaunchKernelGGL((gre_chunk_kernel<TCV, SCALE>), grid, dim3(256), 0, s, ch.e0, ch.e1, q0, op.col,              \
                       op.val, dis, X, t, op.P);                                                                    \
    break;
  switch (op.tc) {
    GRE_CHUNK_CASE(1)
    GRE_CHUNK_CASE(2)
    GRE_CHUNK_CASE(4)
    GRE_CHUNK_CASE(8)
    GRE_CHUNK_CASE(16)
    GRE_CHUNK_CASE(32)
    GRE_CHUNK_CASE(64)
    default: Fatal("grouped chunk pass: unsupported lane split %d", op.tc);
  }
#undef GRE_CHUNK_CASE
  HIP_CHECK(hipGetLastError());
}

template <int OP>
void combine_pass(const GreChunks& ch, const double* P, int row0, int row1, int t, const double* dg, const double* dis,
                  const double* In, double* Out, hipStream_t s) {
  const size_t total = (size_t)(row1 - row0) * t;
  if (total == 0) return;
  hipLaunchKernelGGL((gre_combine_kernel<OP>), dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, row0, row1, t,
                     ch.ptr, P, dg, dis, In, Out);
  HIP_CHECK(hipGetLastError());
}

}  // namespace

int gre_tc(int t) {
  int tc = 1;
  while (tc < t && tc < 64) tc <<= 1;
  return tc;
}

int gre_chunk_len(int tc) { return (256 / tc) * kEntriesPerLane; }

void launch_gre_zty(int M, const int* obs_ptr, const int* obs, const double* y, double* zty, hipStream_t s) {
  hipLaunchKernelGGL(gre_zty_kernel, dim3((M + 3) / 4), dim3(256), 0, s, M, obs_ptr, obs, y, zty);
  HIP_CHECK(hipGetLastError());
}

void launch_gre_diag(int K, const int* cum, const double* cnt, const double* tau, double* D, double* dis, double* out,
                     hipStream_t s) {
  hipLaunchKernelGGL(gre_diag_kernel, dim3(K), dim3(256), 0, s, K, cum, cnt, tau, D, dis, out);
  HIP_CHECK(hipGetLastError());
}

void launch_gre_apply(const GroupedOp& op, const double* dg, const double* X, double* Y, int t, hipStream_t s) {
  chunk_pass<false>(op, op.full, 0, op.full.n, nullptr, X, t, s);
  combine_pass<kCombApply>(op.full, op.P, 0, op.M, t, dg, nullptr, X, Y, s);
}

void launch_gre_lds_mult(const GroupedOp& op, const double* D, const double* dis, const double* R, double* Y, int t,
                         hipStream_t s) {
  chunk_pass<true>(op, op.lower, 0, op.lower.n, dis, R, t, s);
  combine_pass<kCombLds>(op.lower, op.P, 0, op.M, t, D, dis, R, Y, s);
}

void launch_gre_ssor(const GroupedOp& op, const std::vector<int>& cum, const std::vector<int>& lower_q,
                     const std::vector<int>& upper_q, const double* D, const double* dis, const double* R, double* X,
                     double* Z, int t, hipStream_t s) {
  const int K = (int)cum.size() - 1;
  for (int k = 0; k < K; ++k) {   // forward: effects ascending (their lower entries are solved)
    chunk_pass<true>(op, op.lower, lower_q[k], lower_q[k + 1], dis, X, t, s);
    combine_pass<kCombFwd>(op.lower, op.P, cum[k], cum[k + 1], t, D, dis, R, X, s);
  }
  for (int k = K - 1; k >= 0; --k) {   // backward on the transpose: effects descending
    chunk_pass<false>(op, op.upper, upper_q[k], upper_q[k + 1], nullptr, Z, t, s);
    combine_pass<kCombBwd>(op.upper, op.P, cum[k], cum[k + 1], t, D, dis, X, Z, s);
  }
}

void launch_gre_upper(const GroupedOp& op, const double* D, const double* X, double* Y, int t, hipStream_t s) {
  chunk_pass<false>(op, op.upper, 0, op.upper.n, nullptr, X, t, s);
  combine_pass<kCombUpper>(op.upper, op.P, 0, op.M, t, D, nullptr, X, Y, s);
}

void launch_gre_single(int M, const double* zty, const double* cnt, const double* D, double* u, double* out,
                       hipStream_t s) {
  hipLaunchKernelGGL(gre_single_kernel, dim3(1), dim3(256), 0, s, M, zty, cnt, D, u, out);
  HIP_CHECK(hipGetLastError());
}

namespace {
__global__ void __launch_bounds__(256) gre_dense_build_kernel(int M, int ld, const int* __restrict__ rowptr,
                                                              const int* __restrict__ col, const double* __restrict__ val,
                                                              const double* __restrict__ D, double* __restrict__ A) {
  const int r = blockIdx.x * 256 + threadIdx.x;
  if (r >= M) return;
  A[(size_t)r * ld + r] = D[r];
  for (int e = rowptr[r]; e < rowptr[r + 1]; ++e) A[(size_t)col[e] * ld + r] = val[e];
}

// one wave per column: sum of squares of the column's lower part (fixed lane order, then a shuffle tree)
__global__ void __launch_bounds__(256) gre_inv_diag_kernel(int M, int ld, const double* __restrict__ Li,
                                                           double* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (i >= M) return;
  const double* c = Li + (size_t)i * ld;
  double s = 0.;
  for (int r = i + lane; r < M; r += 64) s = fma(c[r], c[r], s);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  if (lane == 0) out[i] = s;
}
__global__ void __launch_bounds__(256) gre_pred_cols_kernel(int M, int ld, int K, int np, const int* __restrict__ idx,
                                                            const double* __restrict__ Li, double* __restrict__ E,
                                                            double* __restrict__ var) {
  const int lane = threadIdx.x & 63;
  const int p = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (p >= np) return;
  const int* ip = idx + (size_t)p * K;
  double s = 0.;
  for (int r = lane; r < M; r += 64) {
    double v = 0.;
    for (int k = 0; k < K; ++k) {
      const int a = ip[k];
      if (a >= 0 && r >= a) v += Li[(size_t)a * ld + r];
    }
    if (E) E[(size_t)p * ld + r] = v;
    s = fma(v, v, s);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  if (var && lane == 0) var[p] = s;
}
__global__ void __launch_bounds__(256) gre_fisher_cols_kernel(int M, int ld, int K, const int* __restrict__ cum,
                                                              const double* __restrict__ sc,
                                                              const double* __restrict__ Ainv, double* __restrict__ part,
                                                              double* __restrict__ diag) {
  const int lane = threadIdx.x & 63;
  const int c = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (c >= M) return;
  const double* col = Ainv + (size_t)c * ld;
  const double scc = sc[c];
  for (int k = 0; k < K; ++k) {
    double s = 0.;
    for (int r = cum[k] + lane; r < cum[k + 1]; r += 64) {
      const double b = col[r] * sc[r] * scc;
      s = fma(b, b, s);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    if (lane == 0) part[(size_t)c * K + k] = s;
  }
  if (lane == 0) diag[c] = col[c] * scc * scc;
}
}  // namespace

void launch_gre_fisher_cols(int M, int ld, int K, const int* cum, const double* sc, const double* Ainv, double* part,
                            double* diag, hipStream_t s) {
  hipLaunchKernelGGL(gre_fisher_cols_kernel, dim3((M + 3) / 4), dim3(256), 0, s, M, ld, K, cum, sc, Ainv, part, diag);
  HIP_CHECK(hipGetLastError());
}

void launch_gre_pred_cols(int M, int ld, int K, int np, const int* idx, const double* Li, double* E, double* var,
                          hipStream_t s) {
  hipLaunchKernelGGL(gre_pred_cols_kernel, dim3((np + 3) / 4), dim3(256), 0, s, M, ld, K, np, idx, Li, E, var);
  HIP_CHECK(hipGetLastError());
}

void launch_gre_dense_build(int M, int ld, const int* rowptr, const int* col, const double* val, const double* D,
                            double* A, hipStream_t s) {
  hipLaunchKernelGGL(gre_dense_build_kernel, dim3((M + 255) / 256), dim3(256), 0, s, M, ld, rowptr, col, val, D, A);
  HIP_CHECK(hipGetLastError());
}

void launch_gre_inv_diag(int M, int ld, const double* Li, double* out, hipStream_t s) {
  hipLaunchKernelGGL(gre_inv_diag_kernel, dim3((M + 3) / 4), dim3(256), 0, s, M, ld, Li, out);
  HIP_CHECK(hipGetLastError());
}

void launch_gre_residual(size_t count, const double* rhs, const double* V, double* R, hipStream_t s) {
  if (count == 0) return;
  hipLaunchKernelGGL(gre_residual_kernel, dim3((unsigned)((count + 255) / 256)), dim3(256), 0, s, count, rhs, V, R);
  HIP_CHECK(hipGetLastError());
}

}  // namespace gpb_amd
