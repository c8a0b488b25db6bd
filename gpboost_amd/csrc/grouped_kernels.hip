// Device kernels of the grouped-random-effects engine (grouped.h). Blocks of t vectors are row-major
// M x t (one RE row = t contiguous doubles); row kernels give one wave to a row, lane = column, so a
// neighbour row's t values are one coalesced gather. The SSOR solves mirror the reference's sparse
// triangular solves (Eigen, row-major P_SSOR_L_D_sqrt_inv_rm, CG_utils.cpp:1143-1148) operation for
// operation — same coefficients (L_ij sqrt(1/D_j), diagonal D_i sqrt(1/D_i)), same subtraction order,
// no FMA contraction — so the PCG iterates round like the reference's.
#include <hip/hip_runtime.h>

#include "common.h"
#include "grouped_kernels.h"

namespace gpb_amd {
namespace {

constexpr int kRowsPerBlock = 4;   // one wave per row, 256 threads

__device__ __forceinline__ int row_of_block() { return blockIdx.x * kRowsPerBlock + (threadIdx.x >> 6); }

// Z^T y, one thread per RE level summing its observations in ascending order (the order of the
// reference's col-major Zt_ * y_).
__global__ void __launch_bounds__(256) gre_zty_kernel(int M, const int* __restrict__ obs_ptr,
                                                      const int* __restrict__ obs, const double* __restrict__ y,
                                                      double* __restrict__ zty) {
  const int r = blockIdx.x * 256 + threadIdx.x;
  if (r >= M) return;
  double s = 0.;
  for (int e = obs_ptr[r]; e < obs_ptr[r + 1]; ++e) s += y[obs[e]];
  zty[r] = s;
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

// Y = A X with A = diag(dg) + offdiag(Z^T Z): per row, entries in ascending column order with the
// diagonal at its place (Eigen row-major sparse x dense). dg = D (with Sigma^-1) or cnt (Z^T Z only).
__global__ void __launch_bounds__(256) gre_apply_kernel(GroupedOp op, const double* __restrict__ dg,
                                                        const double* __restrict__ X, double* __restrict__ Y, int t) {
#pragma clang fp contract(off)
  const int r = row_of_block();
  if (r >= op.M) return;
  const int c = (threadIdx.x & 63) + blockIdx.y * 64;
  if (c >= t) return;
  const int e0 = op.rowptr[r], es = op.split[r], e1 = op.rowptr[r + 1];
  double s = 0.;
  for (int e = e0; e < es; ++e) s += op.val[e] * X[(size_t)op.col[e] * t + c];
  s += dg[r] * X[(size_t)r * t + c];
  for (int e = es; e < e1; ++e) s += op.val[e] * X[(size_t)op.col[e] * t + c];
  Y[(size_t)r * t + c] = s;
}

// probe_P = (L D^-1/2) R: row i sums (L_ij sqrt(1/D_j)) R_j over its lower entries, then the diagonal
// D_i sqrt(1/D_i) R_i (CG-probe draw from N(0, P), re_model_template.h:2808-2812).
__global__ void __launch_bounds__(256) gre_lds_mult_kernel(GroupedOp op, const double* __restrict__ D,
                                                           const double* __restrict__ dis, const double* __restrict__ R,
                                                           double* __restrict__ Y, int t) {
#pragma clang fp contract(off)
  const int r = row_of_block();
  if (r >= op.M) return;
  const int c = (threadIdx.x & 63) + blockIdx.y * 64;
  if (c >= t) return;
  double s = 0.;
  for (int e = op.rowptr[r]; e < op.split[r]; ++e) {
    const int j = op.col[e];
    s += (op.val[e] * dis[j]) * R[(size_t)j * t + c];
  }
  s += (D[r] * dis[r]) * R[(size_t)r * t + c];
  Y[(size_t)r * t + c] = s;
}

// Forward solve (L D^-1/2) X = R over the rows of one effect (lower effects already solved).
__global__ void __launch_bounds__(256) gre_ssor_fwd_kernel(GroupedOp op, int row0, int row1,
                                                           const double* __restrict__ D, const double* __restrict__ dis,
                                                           const double* __restrict__ R, double* __restrict__ X, int t) {
#pragma clang fp contract(off)
  const int r = row0 + row_of_block();
  if (r >= row1) return;
  const int c = (threadIdx.x & 63) + blockIdx.y * 64;
  if (c >= t) return;
  double tmp = R[(size_t)r * t + c];
  for (int e = op.rowptr[r]; e < op.split[r]; ++e) {
    const int j = op.col[e];
    tmp -= (op.val[e] * dis[j]) * X[(size_t)j * t + c];
  }
  X[(size_t)r * t + c] = tmp / (D[r] * dis[r]);
}

// Backward solve (L D^-1/2)^T Z = X over the rows of one effect (higher effects already solved).
// Eigen solves the transposed (column-major upper) system by scattering each solved z_j into the
// rows above it, j descending; gathered here in that same order.
__global__ void __launch_bounds__(256) gre_ssor_bwd_kernel(GroupedOp op, int row0, int row1,
                                                           const double* __restrict__ D, const double* __restrict__ dis,
                                                           const double* __restrict__ X, double* __restrict__ Z, int t) {
#pragma clang fp contract(off)
  const int r = row0 + row_of_block();
  if (r >= row1) return;
  const int c = (threadIdx.x & 63) + blockIdx.y * 64;
  if (c >= t) return;
  double tmp = X[(size_t)r * t + c];
  const double di = dis[r];
  for (int e = op.rowptr[r + 1] - 1; e >= op.split[r]; --e) tmp -= (op.val[e] * di) * Z[(size_t)op.col[e] * t + c];
  Z[(size_t)r * t + c] = tmp / (D[r] * di);
}

// DI = D^-1 (upper triangle of A incl. the diagonal) X (variance reduction, re_model_template.h:2327-2336)
__global__ void __launch_bounds__(256) gre_upper_kernel(GroupedOp op, const double* __restrict__ D,
                                                        const double* __restrict__ X, double* __restrict__ Y, int t) {
#pragma clang fp contract(off)
  const int r = row_of_block();
  if (r >= op.M) return;
  const int c = (threadIdx.x & 63) + blockIdx.y * 64;
  if (c >= t) return;
  double s = D[r] * X[(size_t)r * t + c];
  for (int e = op.split[r]; e < op.rowptr[r + 1]; ++e) s += op.val[e] * X[(size_t)op.col[e] * t + c];
  Y[(size_t)r * t + c] = (1. / D[r]) * s;
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

dim3 row_grid(int rows, int t) { return dim3((rows + kRowsPerBlock - 1) / kRowsPerBlock, (t + 63) / 64); }

}  // namespace

void launch_gre_zty(int M, const int* obs_ptr, const int* obs, const double* y, double* zty, hipStream_t s) {
  hipLaunchKernelGGL(gre_zty_kernel, dim3((M + 255) / 256), dim3(256), 0, s, M, obs_ptr, obs, y, zty);
  HIP_CHECK(hipGetLastError());
}

void launch_gre_diag(int K, const int* cum, const double* cnt, const double* tau, double* D, double* dis, double* out,
                     hipStream_t s) {
  hipLaunchKernelGGL(gre_diag_kernel, dim3(K), dim3(256), 0, s, K, cum, cnt, tau, D, dis, out);
  HIP_CHECK(hipGetLastError());
}

void launch_gre_apply(const GroupedOp& op, const double* dg, const double* X, double* Y, int t, hipStream_t s) {
  hipLaunchKernelGGL(gre_apply_kernel, row_grid(op.M, t), dim3(256), 0, s, op, dg, X, Y, t);
  HIP_CHECK(hipGetLastError());
}

void launch_gre_lds_mult(const GroupedOp& op, const double* D, const double* dis, const double* R, double* Y, int t,
                         hipStream_t s) {
  hipLaunchKernelGGL(gre_lds_mult_kernel, row_grid(op.M, t), dim3(256), 0, s, op, D, dis, R, Y, t);
  HIP_CHECK(hipGetLastError());
}

void launch_gre_ssor(const GroupedOp& op, const std::vector<int>& cum, const double* D, const double* dis,
                     const double* R, double* X, double* Z, int t, hipStream_t s) {
  const int K = (int)cum.size() - 1;
  for (int k = 0; k < K; ++k)
    hipLaunchKernelGGL(gre_ssor_fwd_kernel, row_grid(cum[k + 1] - cum[k], t), dim3(256), 0, s, op, cum[k], cum[k + 1],
                       D, dis, R, X, t);
  for (int k = K - 1; k >= 0; --k)
    hipLaunchKernelGGL(gre_ssor_bwd_kernel, row_grid(cum[k + 1] - cum[k], t), dim3(256), 0, s, op, cum[k], cum[k + 1],
                       D, dis, X, Z, t);
  HIP_CHECK(hipGetLastError());
}

void launch_gre_upper(const GroupedOp& op, const double* D, const double* X, double* Y, int t, hipStream_t s) {
  hipLaunchKernelGGL(gre_upper_kernel, row_grid(op.M, t), dim3(256), 0, s, op, D, X, Y, t);
  HIP_CHECK(hipGetLastError());
}

void launch_gre_single(int M, const double* zty, const double* cnt, const double* D, double* u, double* out,
                       hipStream_t s) {
  hipLaunchKernelGGL(gre_single_kernel, dim3(1), dim3(256), 0, s, M, zty, cnt, D, u, out);
  HIP_CHECK(hipGetLastError());
}

void launch_gre_residual(size_t count, const double* rhs, const double* V, double* R, hipStream_t s) {
  if (count == 0) return;
  hipLaunchKernelGGL(gre_residual_kernel, dim3((unsigned)((count + 255) / 256)), dim3(256), 0, s, count, rhs, V, R);
  HIP_CHECK(hipGetLastError());
}

}  // namespace gpb_amd
