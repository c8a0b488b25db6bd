// Kernels for linear regression covariates (generalised least squares) and for the training-data
// random-effect predictions of the exact Gaussian Vecchia approximation.
//
// Reference: UpdateCoefGLS / CalcXTPsiInvX (re_model_template.h:9125-9132) — beta = (X^T Psi^-1 X)^-1
// X^T Psi^-1 y with Psi^-1 = B^T D^-1 B for the Vecchia approximation — and
// PredictTrainingDataRandomEffects, Vecchia branch (re_model_template.h, mean y - Psi^-1 y,
// variance sigma^2 (1 - diag(B^T D^-1 B))).
//
// Layout: Z = [X | y] row-major n x c in Vecchia order (c <= kCovMaxCols); B values n x m
// (B(i, nbr[i m + r]) at i m + r, unit diagonal implicit), D^-1 n — the row kernel's factor mode
// output (VecchiaRowsArgs::B_out / Dinv_out). The Gram sums are fixed-order (bitwise repeatable).
#include <hip/hip_runtime.h>

#include "common.h"
#include "covariates.h"

namespace gpb_amd {

namespace {

constexpr int kGramRows = 64;       // rows per LDS tile
constexpr int kGramThreads = 256;
constexpr int kGramMaxBlocks = 256;
constexpr int kGramPairsPerThread = (kCovMaxCols * (kCovMaxCols + 1) / 2 + kGramThreads - 1) / kGramThreads;

// Block b sums rows of tiles b, b + gridDim.x, ...: w_i = Z_i + sum_r B[i, r] Z_nbr (all c columns),
// partial[b][pair(a <= b')] = sum_i D^-1_i w_ia w_ib'.
__global__ void __launch_bounds__(kGramThreads) vecchia_gram_kernel(int n, int m, int c, const int* __restrict__ nbr,
                                                                    const double* __restrict__ B,
                                                                    const double* __restrict__ Dinv,
                                                                    const double* __restrict__ Z,
                                                                    double* __restrict__ partial) {
  __shared__ double w[kGramRows][kCovMaxCols + 1];
  __shared__ double dv[kGramRows];
  const int npairs = c * (c + 1) / 2;
  double acc[kGramPairsPerThread];
  int pa[kGramPairsPerThread], pb[kGramPairsPerThread];
#pragma unroll
  for (int q = 0; q < kGramPairsPerThread; ++q) {
    acc[q] = 0.;
    const int pr = threadIdx.x + q * kGramThreads;
    int a = 0, rem = pr;
    while (a < c && rem >= c - a) { rem -= c - a; ++a; }   // pair index -> (a, a + rem)
    pa[q] = a;
    pb[q] = a + rem;
  }
  for (int t0 = blockIdx.x * kGramRows; t0 < n; t0 += gridDim.x * kGramRows) {
    const int rows = min(kGramRows, n - t0);
    // phase 1: (row, column) work items
    for (int it = threadIdx.x; it < rows * c; it += kGramThreads) {
      const int r = it / c, col = it - r * c;
      const int i = t0 + r;
      const int k = i < m ? i : m;
      double v = Z[(size_t)i * c + col];
      for (int e = 0; e < k; ++e) v = fma(B[(size_t)i * m + e], Z[(size_t)nbr[(size_t)i * m + e] * c + col], v);
      w[r][col] = v;
      if (col == 0) dv[r] = Dinv[i];
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < kGramPairsPerThread; ++q) {
      if (threadIdx.x + q * kGramThreads < npairs) {
        double s = 0.;
        for (int r = 0; r < rows; ++r) s = fma(dv[r] * w[r][pa[q]], w[r][pb[q]], s);
        acc[q] += s;
      }
    }
    __syncthreads();
  }
#pragma unroll
  for (int q = 0; q < kGramPairsPerThread; ++q) {
    const int pr = threadIdx.x + q * kGramThreads;
    if (pr < npairs) partial[(size_t)blockIdx.x * npairs + pr] = acc[q];
  }
}

// out[j] = sum_b partial[b][j], blocks in ascending order
__global__ void __launch_bounds__(256) colsum_kernel(const double* __restrict__ partial, int nblocks, int width,
                                                     double* __restrict__ out) {
  const int j = blockIdx.x * 256 + threadIdx.x;
  if (j >= width) return;
  double s = 0.;
  for (int b = 0; b < nblocks; ++b) s += partial[(size_t)b * width + j];
  out[j] = s;
}

// u_i = D^-1_i (B y)_i
__global__ void __launch_bounds__(256) vecchia_dinv_by_kernel(int n, int m, const int* __restrict__ nbr,
                                                              const double* __restrict__ B,
                                                              const double* __restrict__ Dinv,
                                                              const double* __restrict__ y, double* __restrict__ u) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const int k = i < m ? i : m;
  double v = y[i];
  for (int e = 0; e < k; ++e) v = fma(B[(size_t)i * m + e], y[nbr[(size_t)i * m + e]], v);
  u[i] = Dinv[i] * v;
}

// Through the transposed lists (column j -> entries [tptr[j], tptr[j+1]) of rows trow, value slot
// tslot, rows ascending): yaux_j = u_j + sum_e B[slot_e] u[row_e] (= (B^T u)_j) and
// diag_j = D^-1_j + sum_e B[slot_e]^2 D^-1[row_e] (= diag(B^T D^-1 B)_j).
__global__ void __launch_bounds__(256) vecchia_bt_diag_kernel(int n, const int* __restrict__ tptr,
                                                              const int* __restrict__ trow,
                                                              const int* __restrict__ tslot,
                                                              const double* __restrict__ B,
                                                              const double* __restrict__ Dinv,
                                                              const double* __restrict__ u, double* __restrict__ yaux,
                                                              double* __restrict__ diag) {
  const int j = blockIdx.x * 256 + threadIdx.x;
  if (j >= n) return;
  double a = u[j], dg = Dinv[j];
  for (int e = tptr[j]; e < tptr[j + 1]; ++e) {
    const double b = B[tslot[e]];
    const int r = trow[e];
    a = fma(b, u[r], a);
    dg = fma(b * b, Dinv[r], dg);
  }
  yaux[j] = a;
  diag[j] = dg;
}

}  // namespace

int vecchia_gram_blocks(int n) {
  const int tiles = (n + kGramRows - 1) / kGramRows;
  return tiles < kGramMaxBlocks ? (tiles > 0 ? tiles : 1) : kGramMaxBlocks;
}

void launch_vecchia_gram(int n, int m, int c, const int* nbr, const double* B, const double* Dinv, const double* Z,
                         double* partial, double* out, hipStream_t s) {
  if (c < 1 || c > kCovMaxCols) Fatal("number of covariates + 1 = %d outside [1, %d]", c, kCovMaxCols);
  const int nb = vecchia_gram_blocks(n);
  const int npairs = c * (c + 1) / 2;
  hipLaunchKernelGGL(vecchia_gram_kernel, dim3(nb), dim3(kGramThreads), 0, s, n, m, c, nbr, B, Dinv, Z, partial);
  HIP_CHECK(hipGetLastError());
  hipLaunchKernelGGL(colsum_kernel, dim3((npairs + 255) / 256), dim3(256), 0, s, partial, nb, npairs, out);
  HIP_CHECK(hipGetLastError());
}

void launch_vecchia_psi_inv_diag(int n, int m, const int* nbr, const int* tptr, const int* trow, const int* tslot,
                                 const double* B, const double* Dinv, const double* y, double* u, double* yaux,
                                 double* diag, hipStream_t s) {
  const int g = (n + 255) / 256;
  hipLaunchKernelGGL(vecchia_dinv_by_kernel, dim3(g), dim3(256), 0, s, n, m, nbr, B, Dinv, y, u);
  HIP_CHECK(hipGetLastError());
  hipLaunchKernelGGL(vecchia_bt_diag_kernel, dim3(g), dim3(256), 0, s, n, tptr, trow, tslot, B, Dinv, u, yaux, diag);
  HIP_CHECK(hipGetLastError());
}

}  // namespace gpb_amd
