// Microbenchmark: one-wave 64 x 64 Cholesky + inverse of the diagonal block (dense POTRF's
// potrf_diag_wave_kernel) and variants, on an SPD block; average device time per launch.
//   V0: the production form (dense_kernels.hip)
//   V1: factorization only (no inverse)
//   V2: production factorization, inverse with 4 independent partial sums per row
//   V3: V2 + reciprocal-multiply instead of a divide per step
//   V6, V7: see below (code size; the production kernel's fully unrolled form is ~19k instructions)
// hipcc --offload-arch=gfx950 -O3 -o diag_bench diag_bench.hip && ./diag_bench
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { std::printf("HIP error %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

template <int V>
__global__ void __launch_bounds__(64) diag_kernel(double* A, int lda, int ib, double* Winv, int ldw, int* info) {
  __shared__ double colb[2][64];
  __shared__ double Ls[64][65];
  const int r = threadIdx.x;
  double row[64];
#pragma unroll
  for (int c = 0; c < 64; ++c) row[c] = (r < ib && c < ib && c <= r) ? A[(size_t)r + (size_t)c * lda] : 0.;
#pragma unroll
  for (int j = 0; j < 64; ++j) {
    if (j < ib) {
      const double p = __shfl(row[j], j, 64);
      double d;
      if (!(p > 0.)) {
        if (r == 0) atomicAdd(info, 1);
        d = 1.;
      } else {
        d = sqrt(p);
      }
      double l;
      if constexpr (V == 3) {
        const double rd = 1. / d;
        l = (r > j) ? row[j] * rd : (r == j ? d : 0.);
      } else {
        l = (r > j) ? row[j] / d : (r == j ? d : 0.);
      }
      if (r >= j) row[j] = l;
      colb[j & 1][r] = l;
      __syncthreads();
#pragma unroll
      for (int c = j + 1; c < 64; ++c) row[c] = fma(-l, colb[j & 1][c], row[c]);
    }
  }
#pragma unroll
  for (int c = 0; c < 64; ++c) {
    Ls[r][c] = row[c];
    if (r < ib && c < ib && c <= r) A[(size_t)r + (size_t)c * lda] = row[c];
  }
  if constexpr (V == 1) return;
  __syncthreads();
  double x[64];
  if constexpr (V == 0) {
#pragma unroll
    for (int i = 0; i < 64; ++i) {
      double s = (i == r) ? 1. : 0.;
#pragma unroll
      for (int p = 0; p < i; ++p) s -= Ls[i][p] * x[p];
      x[i] = (i >= r && i < ib) ? s / Ls[i][i] : 0.;
    }
  } else {
#pragma unroll
    for (int i = 0; i < 64; ++i) {
      double s0 = (i == r) ? 1. : 0., s1 = 0., s2 = 0., s3 = 0.;
#pragma unroll
      for (int p = 0; p + 3 < i; p += 4) {
        s0 -= Ls[i][p] * x[p];
        s1 -= Ls[i][p + 1] * x[p + 1];
        s2 -= Ls[i][p + 2] * x[p + 2];
        s3 -= Ls[i][p + 3] * x[p + 3];
      }
#pragma unroll
      for (int p = (i / 4) * 4; p < i; ++p) s0 -= Ls[i][p] * x[p];
      const double s = (s0 + s1) + (s2 + s3);
      x[i] = (i >= r && i < ib) ? s / Ls[i][i] : 0.;
    }
  }
#pragma unroll
  for (int i = 0; i < 64; ++i)
    if (i < ib && r < ib) Winv[(size_t)i + (size_t)r * ldw] = (r <= i) ? x[i] : 0.;
}

// V4: full 64 block without per-step branches, reciprocal multiply, column j+1 updated first (the
//     next pivot's sqrt / reciprocal can overlap the rest of the step's FMAs); inverse with the
//     diagonal reciprocals from the factorization and 4 partial sums
template <int V>
__global__ void __launch_bounds__(64) diag_kernel_la(double* A, int lda, double* Winv, int ldw, int* info) {
  __shared__ double colb[2][64];
  __shared__ double Ls[64][65];
  __shared__ double rdg[64];
  const int r = threadIdx.x;
  double row[64];
#pragma unroll
  for (int c = 0; c < 64; ++c) row[c] = (c <= r) ? A[(size_t)r + (size_t)c * lda] : 0.;
#pragma unroll
  for (int j = 0; j < 64; ++j) {
    const double p = __shfl(row[j], j, 64);
    const double d = p > 0. ? sqrt(p) : 1.;
    if (!(p > 0.) && r == 0) atomicAdd(info, 1);
    const double rd = 1. / d;
    const double l = (r > j) ? row[j] * rd : (r == j ? d : 0.);
    if (r >= j) row[j] = l;
    if (r == j) rdg[j] = rd;
    colb[j & 1][r] = l;
    __syncthreads();
    if (j + 1 < 64) row[j + 1] = fma(-l, colb[j & 1][j + 1], row[j + 1]);
#pragma unroll
    for (int c = j + 2; c < 64; ++c) row[c] = fma(-l, colb[j & 1][c], row[c]);
#pragma unroll
    for (int c = j + 1; c < 64; ++c) asm volatile("" : "+v"(row[c]));   // keep the step's updates in place
  }
#pragma unroll
  for (int c = 0; c < 64; ++c) {
    Ls[r][c] = row[c];
    if (c <= r) A[(size_t)r + (size_t)c * lda] = row[c];
  }
  if constexpr (V == 1) return;
  __syncthreads();
  // column r of L^-1 in LDS (X[i][r]), terms p < r are zero: start at p = r
  __shared__ double X[64][65];
  for (int i = 0; i < 64; ++i) {
    double s0 = (i == r) ? 1. : 0., s1 = 0.;
    int p = r;
    for (; p + 1 < i; p += 2) {
      s0 -= Ls[i][p] * X[p][r];
      s1 -= Ls[i][p + 1] * X[p + 1][r];
    }
    if (p < i) s0 -= Ls[i][p] * X[p][r];
    X[i][r] = (i >= r) ? (s0 + s1) * rdg[i] : 0.;
  }
  for (int i = 0; i < 64; ++i) Winv[(size_t)i + (size_t)r * ldw] = (r <= i) ? X[i][r] : 0.;
}


__device__ __forceinline__ double readlane_f64(double v, int l) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), l);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), l);
  return __hiloint2double(hi, lo);
}

// V6: one wave, full 64 block always (a partial block padded with the identity), pivot by v_readlane,
// reciprocal multiply, no per-step guards, column broadcast by one LDS write + 16-byte reads; inverse
// with the diagonal reciprocals from the factorization (fewer instructions: the I-cache holds more of it)
__global__ void __launch_bounds__(64) diag_v6(double* A, int lda, int ib, double* Winv, int ldw, int* info) {
  typedef double v2d __attribute__((ext_vector_type(2)));
  __shared__ __attribute__((aligned(16))) double colb[64];
  __shared__ __attribute__((aligned(16))) double Ls[64][66];
  __shared__ double rdg[64];
  const int r = threadIdx.x;
  const int rr = min(r, ib - 1);
  double row[64];
#pragma unroll
  for (int c = 0; c < 64; ++c) {
    const double v = A[(size_t)rr + (size_t)min(c, ib - 1) * lda];
    row[c] = (r < ib && c < ib) ? (c <= r ? v : 0.) : (r == c ? 1. : 0.);
  }
  bool bad = false;
#pragma unroll
  for (int j = 0; j < 64; ++j) {
    const double p = readlane_f64(row[j], j);
    bad = bad || !(p > 0.);
    const double d = p > 0. ? sqrt(p) : 1.;
    const double rd = 1. / d;
    const double l = r > j ? row[j] * rd : (r == j ? d : 0.);
    if (r >= j) row[j] = l;
    colb[r] = l;
    rdg[j] = rd;
    const v2d* cb = reinterpret_cast<const v2d*>(colb);
#pragma unroll
    for (int c = j + 1; c < 64; ++c) {
      const double lc = (c & 1) ? cb[c >> 1].y : cb[c >> 1].x;
      row[c] = fma(-l, lc, row[c]);
    }
  }
  if (bad && r == 0) atomicAdd(info, 1);
#pragma unroll
  for (int c = 0; c < 64; c += 2) *reinterpret_cast<v2d*>(&Ls[r][c]) = v2d{row[c], row[c + 1]};
#pragma unroll
  for (int c = 0; c < 64; ++c)
    if (c <= r && r < ib && c < ib) A[(size_t)r + (size_t)c * lda] = row[c];
  double x[64];
#pragma unroll
  for (int i = 0; i < 64; ++i) {
    double s = (i == r) ? 1. : 0.;
    const v2d* li = reinterpret_cast<const v2d*>(&Ls[i][0]);
#pragma unroll
    for (int p = 0; p + 1 < i; p += 2) {
      const v2d q = li[p >> 1];
      s = fma(-q.x, x[p], s);
      s = fma(-q.y, x[p + 1], s);
    }
    if (i & 1) s = fma(-Ls[i][i - 1], x[i - 1], s);
    x[i] = (i >= r) ? s * rdg[i] : 0.;
  }
#pragma unroll
  for (int i = 0; i < 64; ++i)
    if (i < ib && r < ib) Winv[(size_t)i + (size_t)r * ldw] = (r <= i) ? x[i] : 0.;
}

// V7: 256 threads, the block in LDS, runtime loop over the 64 pivots (compact code); trailing update
// thread (row r = t & 63, phase q = t >> 6) over columns j + 1 + q, +4, ...; inverse column c = t & 63
// by forward substitution with the k-sum split over the 4 waves (LDS partials, fixed order)
__global__ void __launch_bounds__(256) diag_v7(double* A, int lda, int ib, double* Winv, int ldw, int* info) {
  __shared__ double Ls[64][65];
  __shared__ double Wx[64][65];
  __shared__ double part[4][64];
  __shared__ double rdg[64];
  const int t = threadIdx.x;
  const int r = t & 63, q = t >> 6;
  for (int e = t; e < 64 * 64; e += 256) {
    const int i = e & 63, c = e >> 6;
    Ls[i][c] = (i < ib && c < ib) ? (c <= i ? A[(size_t)i + (size_t)c * lda] : 0.) : (i == c ? 1. : 0.);
  }
  __syncthreads();
  for (int j = 0; j < 64; ++j) {
    const double p = Ls[j][j];
    const double d = p > 0. ? sqrt(p) : 1.;
    const double rd = 1. / d;
    __syncthreads();
    if (q == 0) {
      if (r > j) Ls[r][j] *= rd;
      else if (r == j) Ls[j][j] = d;
      if (r == j) rdg[j] = rd;
      if (r == 0 && !(p > 0.)) atomicAdd(info, 1);
    }
    __syncthreads();
    if (r > j) {
      const double lr = Ls[r][j];
      for (int c = j + 1 + q; c <= r; c += 4) Ls[r][c] = fma(-lr, Ls[c][j], Ls[r][c]);
    }
    __syncthreads();
  }
  for (int e = t; e < 64 * 64; e += 256) {
    const int i = e & 63, c = e >> 6;
    if (i < ib && c < ib && c <= i) A[(size_t)i + (size_t)c * lda] = Ls[i][c];
  }
  // inverse: column c = r; x_i = (delta_ic - sum_{c <= k < i} L_ik x_k) * rdg_i; wave q sums k = c + q, +4, ...
  for (int i = 0; i < 64; ++i) {
    double s = 0.;
    if (i > r)
      for (int k = r + q; k < i; k += 4) s = fma(Ls[i][k], Wx[k][r], s);
    part[q][r] = s;
    __syncthreads();
    if (q == 0) {
      const double tot = (part[0][r] + part[1][r]) + (part[2][r] + part[3][r]);
      Wx[i][r] = i < r ? 0. : (((i == r) ? 1. : 0.) - tot) * rdg[i];
    }
    __syncthreads();
  }
  for (int e = t; e < 64 * 64; e += 256) {
    const int i = e & 63, c = e >> 6;
    if (i < ib && c < ib) Winv[(size_t)i + (size_t)c * ldw] = (c <= i) ? Wx[i][c] : 0.;
  }
}


// V8: four waves; wave w holds the columns c = 4k + w (k < 16) of all 64 rows (lane r = row r) in
// registers. Pivot j: its owner wave (j & 3) takes the pivot by v_readlane, scales its column and
// publishes L[:, j] (zero for rows <= j) to LDS; after ONE barrier every wave updates its columns
// c > j with it (registers whose columns are all <= j are skipped at compile time; the published zeros
// make the rest branch-free). The inverse the same way by rows: wave (i & 3) owns row i of X = L^-1
// (lane r = column r); each wave sums its rows' share of L[i][k] x_k into an LDS partial, one barrier,
// the owner finishes x_i = (delta_ir - sum) / L_ii.
__global__ void __launch_bounds__(256) diag_v8(double* A, int lda, int ib, double* Winv, int ldw, int* info) {
  __shared__ double colb[2][64];
  __shared__ double Ls[64][65];
  __shared__ double part[2][4][64];
  __shared__ double rdg[64];
  const int r = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int rr = min(r, ib - 1);
  double col[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int c = 4 * k + w;
    const double v = A[(size_t)rr + (size_t)min(c, ib - 1) * lda];
    col[k] = (r < ib && c < ib) ? (c <= r ? v : 0.) : (r == c ? 1. : 0.);
  }
  bool bad = false;
#pragma unroll
  for (int j = 0; j < 64; ++j) {
    if (w == (j & 3)) {
      const double p = readlane_f64(col[j >> 2], j);
      bad = bad || !(p > 0.);
      const double d = p > 0. ? sqrt(p) : 1.;
      const double rd = 1. / d;
      const double l = r > j ? col[j >> 2] * rd : (r == j ? d : col[j >> 2]);
      col[j >> 2] = l;
      colb[j & 1][r] = r > j ? l : 0.;
      if (r == j) rdg[j] = rd;
    }
    __syncthreads();
    const double lr = colb[j & 1][r];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      if (4 * k + 3 <= j) continue;   // every column of register k is <= j
      col[k] = fma(-lr, colb[j & 1][4 * k + w], col[k]);
    }
  }
  if (bad && r == 0 && w == 0) atomicAdd(info, 1);
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int c = 4 * k + w;
    Ls[r][c] = col[k];
    if (c <= r && r < ib && c < ib) A[(size_t)r + (size_t)c * lda] = col[k];
  }
  __syncthreads();
  // X = L^-1, lane r = column r; wave w owns rows i = 4m + w of X (x[m])
  double x[16];
#pragma unroll
  for (int i = 0; i < 64; ++i) {
    double s = 0.;
#pragma unroll
    for (int m = 0; m < 16; ++m) {
      if (4 * m >= i) continue;      // rows k = 4m + w < i only
      const int k = 4 * m + w;
      s = (k < i) ? fma(Ls[i][k], x[m], s) : s;
    }
    part[i & 1][w][r] = s;
    __syncthreads();
    if (w == (i & 3)) {
      const double tot = (part[i & 1][0][r] + part[i & 1][1][r]) + (part[i & 1][2][r] + part[i & 1][3][r]);
      x[i >> 2] = (i < r) ? 0. : (((i == r) ? 1. : 0.) - tot) * rdg[i];
    }
  }
#pragma unroll
  for (int m = 0; m < 16; ++m) {
    const int i = 4 * m + w;
    if (i < ib && r < ib) Winv[(size_t)i + (size_t)r * ldw] = (r <= i) ? x[m] : 0.;
  }
}

template <int V>
int run_la(const std::vector<double>& h, double* dA, double* dW, int* dinfo, const char* name) {
  const int reps = 200;
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  float tot = 0.f;
  for (int r = 0; r <= reps; ++r) {
    CK(hipMemcpy(dA, h.data(), sizeof(double) * 64 * 64, hipMemcpyHostToDevice));
    CK(hipEventRecord(a, 0));
    hipLaunchKernelGGL(diag_kernel_la<V>, dim3(1), dim3(64), 0, 0, dA, 64, dW, 64, dinfo);
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms = 0.f;
    CK(hipEventElapsedTime(&ms, a, b));
    if (r > 0) tot += ms;
  }
  std::vector<double> W(64 * 64);
  CK(hipMemcpy(W.data(), dW, sizeof(double) * 64 * 64, hipMemcpyDeviceToHost));
  double chk = 0.;
  for (double v : W) chk += v;
  std::printf("%s: %.2f us per launch (checksum %.12g)\n", name, 1e3 * tot / reps, chk);
  return 0;
}

template <int V>
int run(const std::vector<double>& h, double* dA, double* dW, int* dinfo, const char* name) {
  const int reps = 200;
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  // warm-up
  CK(hipMemcpy(dA, h.data(), sizeof(double) * 64 * 64, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(diag_kernel<V>, dim3(1), dim3(64), 0, 0, dA, 64, 64, dW, 64, dinfo);
  CK(hipDeviceSynchronize());
  float tot = 0.f;
  for (int r = 0; r < reps; ++r) {
    CK(hipMemcpy(dA, h.data(), sizeof(double) * 64 * 64, hipMemcpyHostToDevice));
    CK(hipEventRecord(a, 0));
    hipLaunchKernelGGL(diag_kernel<V>, dim3(1), dim3(64), 0, 0, dA, 64, 64, dW, 64, dinfo);
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms = 0.f;
    CK(hipEventElapsedTime(&ms, a, b));
    tot += ms;
  }
  std::vector<double> W(64 * 64);
  CK(hipMemcpy(W.data(), dW, sizeof(double) * 64 * 64, hipMemcpyDeviceToHost));
  double chk = 0.;
  for (double v : W) chk += v;
  std::printf("%s: %.2f us per launch (checksum %.12g)\n", name, 1e3 * tot / reps, chk);
  return 0;
}


template <int KV>
int run_new(const std::vector<double>& h, double* dA, double* dW, int* dinfo, const char* name) {
  const int reps = 200;
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  float tot = 0.f;
  for (int r = 0; r <= reps; ++r) {
    CK(hipMemcpy(dA, h.data(), sizeof(double) * 64 * 64, hipMemcpyHostToDevice));
    CK(hipEventRecord(a, 0));
    if (KV == 6) hipLaunchKernelGGL(diag_v6, dim3(1), dim3(64), 0, 0, dA, 64, 64, dW, 64, dinfo);
    else if (KV == 8) hipLaunchKernelGGL(diag_v8, dim3(1), dim3(256), 0, 0, dA, 64, 64, dW, 64, dinfo);
    else hipLaunchKernelGGL(diag_v7, dim3(1), dim3(256), 0, 0, dA, 64, 64, dW, 64, dinfo);
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms = 0.f;
    CK(hipEventElapsedTime(&ms, a, b));
    if (r > 0) tot += ms;
  }
  std::vector<double> W(64 * 64), L(64 * 64);
  CK(hipMemcpy(W.data(), dW, sizeof(double) * 64 * 64, hipMemcpyDeviceToHost));
  CK(hipMemcpy(L.data(), dA, sizeof(double) * 64 * 64, hipMemcpyDeviceToHost));
  double chk = 0., chl = 0.;
  for (double v : W) chk += v;
  for (int i = 0; i < 64; ++i)
    for (int c = 0; c <= i; ++c) chl += L[i + 64 * c];
  // back-to-back (warm clocks): 500 launches refactoring the block in place
  CK(hipMemcpy(dA, h.data(), sizeof(double) * 64 * 64, hipMemcpyHostToDevice));
  CK(hipEventRecord(a, 0));
  for (int r = 0; r < 500; ++r) {
    if (KV == 6) hipLaunchKernelGGL(diag_v6, dim3(1), dim3(64), 0, 0, dA, 64, 64, dW, 64, dinfo);
    else if (KV == 8) hipLaunchKernelGGL(diag_v8, dim3(1), dim3(256), 0, 0, dA, 64, 64, dW, 64, dinfo);
    else hipLaunchKernelGGL(diag_v7, dim3(1), dim3(256), 0, 0, dA, 64, 64, dW, 64, dinfo);
  }
  CK(hipEventRecord(b, 0));
  CK(hipEventSynchronize(b));
  float ms = 0.f;
  CK(hipEventElapsedTime(&ms, a, b));
  std::printf("%s: %.2f us per launch, back-to-back %.2f us (checksums W %.12g L %.12g)\n", name, 1e3 * tot / reps,
              1e3 * ms / 500, chk, chl);
  return 0;
}

int main() {
  std::vector<double> h(64 * 64);
  for (int i = 0; i < 64; ++i)
    for (int j = 0; j < 64; ++j) h[i + 64 * j] = std::exp(-std::fabs(i - j) * 0.3) + (i == j ? 0.5 : 0.);
  double *dA, *dW;
  int* dinfo;
  CK(hipMalloc(&dA, sizeof(double) * 64 * 64));
  CK(hipMalloc(&dW, sizeof(double) * 64 * 64));
  CK(hipMalloc(&dinfo, sizeof(int)));
  CK(hipMemset(dinfo, 0, sizeof(int)));
  CK(hipMemset(dW, 0, sizeof(double) * 64 * 64));
  if (run<0>(h, dA, dW, dinfo, "V0 production")) return 1;
  if (run<1>(h, dA, dW, dinfo, "V1 factor only")) return 1;
  if (run<2>(h, dA, dW, dinfo, "V2 inverse, 4 partial sums")) return 1;
  if (run<3>(h, dA, dW, dinfo, "V3 V2 + reciprocal multiply")) return 1;
  if (run_la<1>(h, dA, dW, dinfo, "V4 lookahead factor only")) return 1;
  if (run_la<0>(h, dA, dW, dinfo, "V5 lookahead factor + inverse")) return 1;
  if (run_new<6>(h, dA, dW, dinfo, "V6 compact registers, readlane pivot, rcp-multiply")) return 1;
  if (run_new<7>(h, dA, dW, dinfo, "V7 LDS, 256 threads, runtime pivot loop")) return 1;
  if (run_new<8>(h, dA, dW, dinfo, "V8 four waves, column-owner registers, one barrier per pivot")) return 1;
  // back-to-back launches (no host copy in between: clocks stay up); the block is refactored in place
  {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int v = 0; v < 2; ++v) {
      CK(hipMemcpy(dA, h.data(), sizeof(double) * 64 * 64, hipMemcpyHostToDevice));
      CK(hipEventRecord(a, 0));
      for (int r = 0; r < 500; ++r) {
        if (v == 0) hipLaunchKernelGGL(diag_kernel<0>, dim3(1), dim3(64), 0, 0, dA, 64, 64, dW, 64, dinfo);
        else hipLaunchKernelGGL(diag_kernel_la<0>, dim3(1), dim3(64), 0, 0, dA, 64, dW, 64, dinfo);
      }
      CK(hipEventRecord(b, 0));
      CK(hipEventSynchronize(b));
      float ms = 0.f;
      CK(hipEventElapsedTime(&ms, a, b));
      std::printf("back-to-back %s: %.2f us per launch\n", v ? "V5" : "V0", 1e3 * ms / 500);
    }
  }
  return 0;
}
