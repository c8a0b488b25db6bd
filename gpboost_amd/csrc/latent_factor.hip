// Latent Vecchia factor kernel for gfx950: B = I - A, D^-1 and their range derivatives
// for the latent GP of non-Gaussian likelihoods / gp_approx = "vecchia_latent".
//
// Reference replaced: CalcCovFactorGradientVecchia (Vecchia_utils.cpp:1307-1632) with
// gauss_likelihood = false: no nugget, D_ii starts at 0 (:1354-1356) and receives the
// marginal variance (:1507), the between-neighbour diagonal is multiplied by
// JITTER_MULT_VECCHIA (:1547), the marginal-variance derivative is not formed
// (exclude_marg_var_grad: its SigmaI derivative is -Sigma^-1, likelihoods.h:5036-5038).
//
// Same lane-group mapping as the exact-Gaussian row kernel (vecchia_kernels.hip): K lanes
// own one row, the k x k between-neighbour covariance C and dC/dlog(phi) live in packed
// LDS triangles, one LDS broadcast per elimination step. The solves use a Cholesky factor
// (not the Gauss-Jordan sweep of the nugget-regularised exact-Gaussian kernel): without a
// nugget, C has only a 1e-10 jitter and can be very ill-conditioned (e.g. Gaussian kernel),
// where only triangular solves stay as accurate as the reference's LLT. L overwrites the
// packed C in LDS; the second right-hand side (dA = C^-1 (dc - dC a) needs a first)
// reuses it. The kernel runs once per likelihood evaluation.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "common.h"
#include "cov.h"
#include "latent_kernels.h"

namespace gpb_amd {
namespace {

constexpr int kDMax = 3;
constexpr int kMaxBlocks = 4096;

__device__ __forceinline__ void wave_lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
__device__ __forceinline__ void compiler_fence() { asm volatile("" ::: "memory"); }

template <int K>
__device__ __forceinline__ double group_sum(double v) {
#pragma unroll
  for (int off = K / 2; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

template <int K>
constexpr int block_threads() { return K == 64 ? 64 : 128; }

template <int K>
constexpr int group_lds_doubles() { return K * (K + 1) + kDMax * K + 2 * K; }

__device__ __forceinline__ int packed(int r, int c) { return r * (r + 1) / 2 + c; }

__device__ __forceinline__ double rcp_nr(double x) {   // 1/x: hardware reciprocal + 2 Newton steps
  double r = __builtin_amdgcn_rcp(x);
  r = fma(r, fma(-x, r, 1.), r);
  return fma(r, fma(-x, r, 1.), r);
}

// Right-looking Cholesky C = L L^T of the packed lower triangle, lane r owning row r,
// with the forward solve L y = rhs fused in (one LDS broadcast of column j per step).
// On return row[p] = L(r, p) for p <= r, *inv_diag = 1 / L(r, r), result = y_r.
// Rows >= k are identity padding. (Cholesky rather than Gauss-Jordan: without a nugget the
// between-neighbour covariance can be very ill-conditioned, and only the triangular
// solves keep the error at the level of the reference's LLT, Vecchia_utils.cpp:1556.)
template <int K>
__device__ __forceinline__ double chol_fwd(const double* Cp, int r, double* slot_c, double* slot_a, double rhs,
                                           double (&row)[K], double* inv_diag) {
#pragma unroll
  for (int c = 0; c < K; ++c) row[c] = (c <= r) ? Cp[packed(r, c)] : 0.;
  double aug = rhs;
  double invd = 1.;
#pragma unroll
  for (int j = 0; j < K; ++j) {
    compiler_fence();
    slot_c[r] = row[j];
    slot_a[r] = aug;
    wave_lds_sync();
    const double piv = slot_c[j];
    const double ljj = sqrt(piv);
    const double inv = rcp_nr(ljj);
    const double yj = slot_a[j] * inv;
    const double lr = row[j] * inv;            // L(r, j) for r > j
    const double f = (r > j) ? lr * inv : 0.;  // L(r, j) / L(j, j)
#pragma unroll
    for (int c = j + 1; c < K; ++c) row[c] = fma(-f, slot_c[c], row[c]);
    if (r == j) { row[j] = ljj; aug = yj; invd = inv; }
    if (r > j) { row[j] = lr; aug = fma(-lr, yj, aug); }
#pragma unroll
    for (int c = j; c < K; ++c) asm volatile("" : "+v"(row[c]));
    asm volatile("" : "+v"(aug));
  }
  *inv_diag = invd;
  compiler_fence();
  return aug;
}

// Forward solve L y = rhs with L in registers (row[p] = L(r, p)).
template <int K>
__device__ __forceinline__ double fwd_solve(const double (&row)[K], double inv_diag, int r, double* slot_a,
                                            double rhs) {
  double v = rhs;
#pragma unroll
  for (int j = 0; j < K; ++j) {
    compiler_fence();
    if (r == j) slot_a[j] = v * inv_diag;
    wave_lds_sync();
    const double yj = slot_a[j];
    if (r > j) v = fma(-row[j], yj, v);
    if (r == j) v = yj;
  }
  compiler_fence();
  return v;
}

// Back solve L^T x = y with L packed in LDS (Lp); lane r owns y_r / x_r.
template <int K>
__device__ __forceinline__ double back_solve(const double* Lp, double inv_diag, int r, double* slot_a, double y) {
  double v = y;
#pragma unroll
  for (int j = K - 1; j >= 0; --j) {
    compiler_fence();
    if (r == j) slot_a[j] = v * inv_diag;
    wave_lds_sync();
    const double xj = slot_a[j];
    if (r < j) v = fma(-Lp[packed(j, r)], xj, v);
    if (r == j) v = xj;
  }
  compiler_fence();
  return v;
}

template <int K, int COV>
__global__ void __launch_bounds__(block_threads<K>()) latent_factor_kernel(LatentFactorArgs a) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  constexpr int BT = block_threads<K>();
  constexpr int G = 64 / K;
  constexpr int rows_per_block = (BT / 64) * G;
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int g = lane / K;
  const int r = lane - g * K;
  const int group_id = wave * G + g;
  const int d = a.d;
  const double var = a.var, phi = a.phi;
  const double cdiag = var * a.jitter + a.nugget;
  const bool want_grad = a.dBv != nullptr;

  double* Cp = smem + group_id * group_lds_doubles<K>();
  double* dCp = Cp + K * (K + 1) / 2;
  double* nbx = dCp + K * (K + 1) / 2;
  double* slot_c = nbx + K * kDMax;
  double* slot_a = slot_c + K;

  for (int base = blockIdx.x * rows_per_block; base < a.n; base += gridDim.x * rows_per_block) {
    const int i = base + group_id;
    const bool active = i < a.n;
    const int k = active ? min(i, a.m) : 0;
    const bool rv = r < k;
    const int irow = active ? i : 0;

    const int nb = rv ? a.nbr[(size_t)i * a.m + r] : 0;
    double xi[kDMax], xr[kDMax];
#pragma unroll
    for (int q = 0; q < kDMax; ++q) {
      xi[q] = (q < d) ? a.X[(size_t)irow * d + q] : 0.;
      xr[q] = (q < d && rv) ? a.X[(size_t)nb * d + q] : 0.;
    }
    compiler_fence();
#pragma unroll
    for (int q = 0; q < kDMax; ++q) nbx[r * kDMax + q] = xr[q];

    double cvec = 0., dcvec = 0.;
    {
      double s = 0.;
#pragma unroll
      for (int q = 0; q < kDMax; ++q) { const double t = xi[q] - xr[q]; s += t * t; }
      double cv, dcv;
      cov_dcov<COV>(sqrt(s), var, phi, cv, dcv);
      cvec = rv ? cv : 0.;
      dcvec = rv ? dcv : 0.;
    }
    Cp[packed(r, r)] = rv ? cdiag : 1.;
    dCp[packed(r, r)] = 0.;
    wave_lds_sync();
    {
      const int h = r & (K / 2 - 1);
      const int qlo = (r >= K / 2) ? K / 2 : 0;
      for (int q = qlo; q < qlo + K / 2 && q < K - 1; ++q) {
        int rr, cc;
        if (q < h) { rr = h; cc = q; } else { rr = K - 1 - h; cc = q - h; }
        double cv = 0., dcv = 0.;
        if (rr < k) {
          double s = 0.;
#pragma unroll
          for (int qq = 0; qq < kDMax; ++qq) {
            const double t = nbx[rr * kDMax + qq] - nbx[cc * kDMax + qq];
            s += t * t;
          }
          cov_dcov<COV>(sqrt(s), var, phi, cv, dcv);
        }
        Cp[packed(rr, cc)] = cv;
        dCp[packed(rr, cc)] = dcv;
      }
    }
    wave_lds_sync();

    // a = C^-1 c: Cholesky with fused forward solve, L to LDS (over C), back solve
    double row[K];
    double invd;
    const double y1 = chol_fwd<K>(Cp, r, slot_c, slot_a, cvec, row, &invd);
#pragma unroll
    for (int c = 0; c < K; ++c)
      if (c <= r) Cp[packed(r, c)] = row[c];
    wave_lds_sync();
    const double av_r = back_solve<K>(Cp, invd, r, slot_a, y1);
    const double ac = group_sum<K>(av_r * cvec);
    if (active && r < a.m) a.Bv[(size_t)i * a.m + r] = rv ? -av_r : 0.;
    if (active && r == 0) a.Dinv[i] = 1. / (var + a.nugget - ac);   // Vecchia_utils.cpp:1507, 1562, 1615

    if (a.dBv_var != nullptr) {
      // dc = c, dC = C - nugget I: dA^T = C^-1 (c - (C - I) a) = C^-1 a, dD = var - (dA.c + a.c) = var - a.a - a.c
      const double aa = group_sum<K>(av_r * av_r);
      const double yv = fwd_solve<K>(row, invd, r, slot_a, av_r);
      const double wv = back_solve<K>(Cp, invd, r, slot_a, yv);
      if (active && r < a.m) a.dBv_var[(size_t)i * a.m + r] = rv ? -wv : 0.;
      if (active && r == 0) a.dD_var[i] = var - ac - aa;
    }
    if (want_grad) {
      // t = dC a (dC diagonal is 0), then w = C^-1 (dc - t) = dA^T (:1573-1574)
      compiler_fence();
      slot_c[r] = av_r;
      wave_lds_sync();
      double t = 0.;
      for (int c = 0; c < k; ++c) {
        const double dcrc = (c < r) ? dCp[packed(r, c)] : dCp[packed(c, r)];
        t = fma(dcrc, slot_c[c], t);
      }
      t = rv ? t : 0.;
      const double dca = group_sum<K>(dcvec * av_r);
      const double ta = group_sum<K>(t * av_r);
      const double y2 = fwd_solve<K>(row, invd, r, slot_a, dcvec - t);
      const double w_r = back_solve<K>(Cp, invd, r, slot_a, y2);
      if (active && r < a.m) a.dBv[(size_t)i * a.m + r] = rv ? -w_r : 0.;
      if (active && r == 0) a.dD[i] = -(2. * dca - ta);               // :1583 (range: overwrite)
    }
    compiler_fence();
  }
}

// Rows with more than 64 neighbours (e.g. num_neighbors = n - 1, the R tests' exact Vecchia): one 256-thread
// workgroup per row, the packed between-neighbour covariance in LDS, right-looking Cholesky with the workgroup
// (two barriers per column), the triangular solves on one thread. dC is recomputed from the coordinates when
// the gradient needs t = dC a. Correct for any k <= kWideMax; far slower per row than the lane-group kernel.
constexpr int kWideMax = 180;
template <int COV>
__global__ void __launch_bounds__(256) latent_factor_wide_kernel(LatentFactorArgs a) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int K = a.m;
  double* Cp = smem;                        // K (K + 1) / 2
  double* nbx = Cp + K * (K + 1) / 2;       // K x kDMax
  double* cv = nbx + K * kDMax;             // c
  double* dcv = cv + K;                     // dc / dlog(phi)
  double* av = dcv + K;                     // a = C^-1 c
  double* wv = av + K;                      // work
  const int tid = threadIdx.x, d = a.d;
  const double var = a.var, phi = a.phi;
  const double cdiag = var * a.jitter + a.nugget;
  for (int i = blockIdx.x; i < a.n; i += gridDim.x) {
    const int k = min(i, a.m);
    __syncthreads();
    for (int r = tid; r < k; r += 256) {
      const int nb = a.nbr[(size_t)i * a.m + r];
      double s = 0.;
      for (int q = 0; q < kDMax; ++q) {
        const double x = q < d ? a.X[(size_t)nb * d + q] : 0.;
        nbx[r * kDMax + q] = x;
        const double t = (q < d ? a.X[(size_t)i * d + q] : 0.) - x;
        s += t * t;
      }
      double c, dc;
      cov_dcov<COV>(sqrt(s), var, phi, c, dc);
      cv[r] = c;
      dcv[r] = dc;
    }
    __syncthreads();
    for (int e = tid; e < k * (k + 1) / 2; e += 256) {
      int r = (int)((sqrt(8. * e + 1.) - 1.) / 2.);
      while (r * (r + 1) / 2 > e) --r;
      while ((r + 1) * (r + 2) / 2 <= e) ++r;
      const int c = e - r * (r + 1) / 2;
      double v = cdiag;
      if (c != r) {
        double s = 0.;
        for (int q = 0; q < kDMax; ++q) { const double t = nbx[r * kDMax + q] - nbx[c * kDMax + q]; s += t * t; }
        double dv;
        cov_dcov<COV>(sqrt(s), var, phi, v, dv);
      }
      Cp[e] = v;
    }
    __syncthreads();
    for (int j = 0; j < k; ++j) {   // right-looking LLT of the packed lower triangle
      if (tid == 0) Cp[packed(j, j)] = sqrt(Cp[packed(j, j)]);
      __syncthreads();
      const double ljj = Cp[packed(j, j)];
      for (int r = j + 1 + tid; r < k; r += 256) Cp[packed(r, j)] /= ljj;
      __syncthreads();
      const int w = k - j - 1;
      for (int e = tid; e < w * (w + 1) / 2; e += 256) {
        int rr = (int)((sqrt(8. * e + 1.) - 1.) / 2.);
        while (rr * (rr + 1) / 2 > e) --rr;
        while ((rr + 1) * (rr + 2) / 2 <= e) ++rr;
        const int r = j + 1 + rr, c = j + 1 + (e - rr * (rr + 1) / 2);
        Cp[packed(r, c)] -= Cp[packed(r, j)] * Cp[packed(c, j)];
      }
      __syncthreads();
    }
    auto solve = [&](const double* rhs, double* x) {   // x = C^-1 rhs (thread 0)
      for (int r = 0; r < k; ++r) {
        double s = rhs[r];
        for (int c = 0; c < r; ++c) s -= Cp[packed(r, c)] * x[c];
        x[r] = s / Cp[packed(r, r)];
      }
      for (int r = k - 1; r >= 0; --r) {
        double s = x[r];
        for (int c = r + 1; c < k; ++c) s -= Cp[packed(c, r)] * x[c];
        x[r] = s / Cp[packed(r, r)];
      }
    };
    if (tid == 0) {
      solve(cv, av);
      double ac = 0.;
      for (int r = 0; r < k; ++r) ac += av[r] * cv[r];
      a.Dinv[i] = 1. / (var + a.nugget - ac);
      if (a.dBv != nullptr) {
        // t = dC a (zero diagonal), w = C^-1 (dc - t) = dA^T, dD = -(2 dc.a - t.a) (Vecchia_utils.cpp:1573-1583)
        double dca = 0., ta = 0.;
        for (int r = 0; r < k; ++r) {
          double t = 0.;
          for (int c = 0; c < k; ++c) {
            if (c == r) continue;
            double s = 0.;
            for (int q = 0; q < kDMax; ++q) { const double u = nbx[r * kDMax + q] - nbx[c * kDMax + q]; s += u * u; }
            double cvv, dvv;
            cov_dcov<COV>(sqrt(s), var, phi, cvv, dvv);
            t += dvv * av[c];
          }
          dca += dcv[r] * av[r];
          ta += t * av[r];
          wv[r] = dcv[r] - t;
        }
        a.dD[i] = -(2. * dca - ta);
      }
    }
    __syncthreads();
    for (int r = tid; r < a.m; r += 256) a.Bv[(size_t)i * a.m + r] = r < k ? -av[r] : 0.;
    if (a.dBv != nullptr) {
      __syncthreads();
      if (tid == 0) {
        double* x = av;   // a no longer needed
        solve(wv, x);
      }
      __syncthreads();
      for (int r = tid; r < a.m; r += 256) a.dBv[(size_t)i * a.m + r] = r < k ? -av[r] : 0.;
    }
  }
}

template <int COV>
void launch_wide(const LatentFactorArgs& a, hipStream_t s) {
  const size_t lds = sizeof(double) * ((size_t)a.m * (a.m + 1) / 2 + (size_t)a.m * kDMax + 4 * (size_t)a.m);
  hipLaunchKernelGGL((latent_factor_wide_kernel<COV>), dim3(std::min(a.n, kMaxBlocks)), dim3(256), lds, s, a);
  HIP_CHECK(hipGetLastError());
}

int lanes_for_m(int m) {
  if (m <= 16) return 16;
  if (m <= 32) return 32;
  if (m <= 64) return 64;
  return 0;
}

template <int K, int COV>
void launch_k(const LatentFactorArgs& a, hipStream_t s) {
  constexpr int rpb = (block_threads<K>() / 64) * (64 / K);
  int blocks = (a.n + rpb - 1) / rpb;
  if (blocks > kMaxBlocks) blocks = kMaxBlocks;
  const size_t lds = (size_t)rpb * group_lds_doubles<K>() * sizeof(double);
  hipLaunchKernelGGL((latent_factor_kernel<K, COV>), dim3(blocks), dim3(block_threads<K>()), lds, s, a);
  HIP_CHECK(hipGetLastError());
}

template <int K>
void launch_cov(int cov, const LatentFactorArgs& a, hipStream_t s) {
  switch (cov) {
    case kMatern05: launch_k<K, kMatern05>(a, s); break;
    case kMatern15: launch_k<K, kMatern15>(a, s); break;
    case kMatern25: launch_k<K, kMatern25>(a, s); break;
    case kGaussian: launch_k<K, kGaussian>(a, s); break;
    default: Fatal("unsupported covariance type %d", cov);
  }
}

}  // namespace

void launch_latent_factor(int cov_type, const LatentFactorArgs& a, hipStream_t s) {
  if (a.d < 1 || a.d > kDMax) Fatal("GPU Vecchia kernel supports 1 <= dim_gp_coords <= %d, got %d", kDMax, a.d);
  if (a.n <= 0) return;
  switch (lanes_for_m(a.m)) {
    case 16: launch_cov<16>(cov_type, a, s); break;
    case 32: launch_cov<32>(cov_type, a, s); break;
    case 64: launch_cov<64>(cov_type, a, s); break;
    default:
      if (a.m > kWideMax) Fatal("num_neighbors = %d > %d is not supported by the GPU latent Vecchia kernel", a.m, kWideMax);
      if (a.dBv_var != nullptr) Fatal("num_neighbors = %d > 64 is not supported for the Vecchia Fisher information", a.m);
      switch (cov_type) {
        case kMatern05: launch_wide<kMatern05>(a, s); break;
        case kMatern15: launch_wide<kMatern15>(a, s); break;
        case kMatern25: launch_wide<kMatern25>(a, s); break;
        case kGaussian: launch_wide<kGaussian>(a, s); break;
        default: Fatal("unsupported covariance type %d", cov_type);
      }
  }
}

}  // namespace gpb_amd
