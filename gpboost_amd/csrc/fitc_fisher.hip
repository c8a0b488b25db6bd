// Fisher information of the covariance parameters of the Gaussian FITC model (gp_approx = "fitc"), for
// their standard deviations: FitcSolver::Fisher (fitc.h).
//
// Reference path replaced: CalcStdDevCovPar (re_model_template.h:9775-9789) -> CalcFisherInformation_FITC_FSA
// (:9363-9548, gp_approx = "fitc", cholesky), Hutchinson estimates over t probes z (GenRandVecNormalParallel):
//   x0 = Psi^-1 z,  S_k = Psi^-1 G_k z,  R_k = G_k Psi^-1 z,
//   FI = 1/2 mean_c [x0 . x0, x0 . S_k, R_k . S_l (k <= l)] / sigma^4
// with Psi on the transformed scale (Woodbury: Psi^-1 = D^-1 - D^-1 K_nm M^-1 K_mn D^-1, M = K_mm,s + K_mn
// D^-1 K_nm) and G_k the derivative of the ORIGINAL covariance (GetZSigmaZtGrad(k, false, sigma^2)):
//   G_k X = dd_k .* X + A^T (dK_k^T X - dK_mm,k A X) + dK_k (A X),   A = K_mm,s^-1 K_mn,
//   dd_k = base_k - (2 A_i . dK_k,i - A_i . (dK_mm,k A)_i)          (:9481-9496)
// computed here in transformed-scale units (dK_var = K_mn, dK_mm,var = K_mm un-jittered, base v; range:
// the dlog(phi) derivatives, base 0) and rescaled on the host (d / dsigma1^2 = 1 / v, d / drho =
// sigma^2 dlog(phi) / drho). Every product is an MFMA GEMM over the n x t probe block (column-major, ld n)
// and the m x n matrices of the factor; the M^-1 solves use the clean triangular inverse factor WiT
// (fitc_lower_t) twice, the K_mm,s^-1 product LiT — no explicit inverse. HBM traffic per probe column:
// ~10 passes over the m x n matrices (8 m n bytes each), shared by the t columns of one GEMM.
#include <hip/hip_runtime.h>

#include <cmath>
#include <vector>

#include "cov.h"
#include "dense.h"
#include "fitc.h"
#include "kernels.h"
#include "slq_host.h"

namespace gpb_amd {
namespace {

template <int COV>
__global__ void __launch_bounds__(256) ff_dkmn_kernel(const double* __restrict__ X, const double* __restrict__ Z, int n,
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

// dd_i = base - (2 A_i . dK_i - A_i . M_i) over the columns of the m x n matrices; one wave per column
__global__ void __launch_bounds__(256) ff_diag_grad_kernel(const double* __restrict__ A, const double* __restrict__ dK,
                                                           const double* __restrict__ M, int n, int m, int ldm,
                                                           double base, double* __restrict__ dd) {
  const int lane = threadIdx.x & 63;
  const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (i >= n) return;
  double s1 = 0., s2 = 0.;
  for (int j = lane; j < m; j += 64) {
    const double a = A[(size_t)j + (size_t)i * ldm];
    s1 = fma(a, dK[(size_t)j + (size_t)i * ldm], s1);
    s2 = fma(a, M[(size_t)j + (size_t)i * ldm], s2);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    s1 += __shfl_xor(s1, o, 64);
    s2 += __shfl_xor(s2, o, 64);
  }
  if (lane == 0) dd[i] = base - (2. * s1 - s2);
}

__global__ void __launch_bounds__(256) ff_recip_kernel(int n, const double* __restrict__ x, double* __restrict__ y) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < n) y[i] = 1. / x[i];
}

// Y = alpha s .* X (+ Yin), row i of the column-major n x t blocks scaled by s[i]; Y may alias Yin
__global__ void __launch_bounds__(256) ff_rowscale_kernel(int n, int t, const double* __restrict__ s,
                                                          const double* __restrict__ X, double alpha,
                                                          const double* Yin, double* Y) {
  const size_t total = (size_t)n * t;
  for (size_t e = (size_t)blockIdx.x * 256 + threadIdx.x; e < total; e += (size_t)gridDim.x * 256) {
    const double v = alpha * s[e % (size_t)n] * X[e];
    Y[e] = Yin ? Yin[e] + v : v;
  }
}

// block partials of sum_e a_e b_e (fixed order: per-thread strided sums, then a wave / block tree)
constexpr int kDotBlocks = 512;
__global__ void __launch_bounds__(256) ff_dot_kernel(size_t count, const double* __restrict__ a,
                                                     const double* __restrict__ b, double* __restrict__ part) {
  __shared__ double red[4];
  double s = 0.;
  for (size_t e = (size_t)blockIdx.x * 256 + threadIdx.x; e < count; e += (size_t)gridDim.x * 256)
    s = fma(a[e], b[e], s);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}

}  // namespace

void FitcSolver::Fisher(int cov_type, const double* orig, const double* trafo, int t, int seed, uint64_t run_id,
                        double* FI) {
  const int n = n_, m = m_, ldm = ldm_, d = d_;
  if (t < 1) Fatal("num_rand_vec_trace must be > 0");
  if (!(orig[0] > 0. && orig[1] > 0. && orig[2] > 0.)) Fatal("covariance parameters must be > 0");
  const double var = trafo[1], phi = trafo[2];
  const size_t nt = (size_t)n * t, mt = (size_t)ldm * t;
  DevBuf<double> blk(9 * nt), mblk(4 * mt), nv(4 * (size_t)n), part(kDotBlocks), dots(8);
  double* Zc = blk.get();
  double* X0 = Zc + nt;
  double* Y = X0 + nt;
  double* S[2] = {Y + nt, Y + 2 * nt};
  double* Rk[2] = {Y + 3 * nt, Y + 4 * nt};
  double* T = Y + 5 * nt;
  double* X1 = Y + 6 * nt;
  double* U = mblk.get();
  double* U1 = U + mt;
  double* AX = U1 + mt;
  double* Q = AX + mt;
  double* zero_y = nv.get();
  double* dinv = zero_y + n;
  double* dd[2] = {dinv + n, dinv + 2 * n};
  HIP_CHECK(hipMemsetAsync(zero_y, 0, sizeof(double) * n, stream_));

  // factor on the transformed scale (the response does not enter the Fisher information)
  double* red = red_.get();
  Factor(cov_type, var, phi, zero_y, red);
  int info = 0;
  HIP_CHECK(hipMemcpyAsync(&info, info_.get(), sizeof(int), hipMemcpyDeviceToHost, stream_));
  HIP_CHECK(hipStreamSynchronize(stream_));
  if (info != 0) Fatal("the FITC factor is not positive definite at these covariance parameters");
  const int nb4 = (n + 3) / 4;
  // A = K_mm,s^-1 K_mn = L^-T V (LiT: the clean upper triangle of L^-T); dK_mn / dlog(phi) into Kd_
  gemm_f64(stream_, m, n, m, 1., LiT_.get(), ldm, 0, V_.get(), ldm, 0, 0., A_.get(), ldm, 0, 0, 1, 0);
  switch (cov_type) {
#define GPB_FF_DKMN(C)                                                                                             \
  case C:                                                                                                          \
    hipLaunchKernelGGL((ff_dkmn_kernel<C>), dim3((m + 63) / 64, (n + 3) / 4), dim3(256), 0, stream_, d_X_, dZ_.get(), \
                       n, m, d, ldm, var, phi, Kd_.get());                                                         \
    break;
    GPB_FF_DKMN(kMatern05)
    GPB_FF_DKMN(kMatern15)
    GPB_FF_DKMN(kMatern25)
    GPB_FF_DKMN(kGaussian)
#undef GPB_FF_DKMN
    default: Fatal("unsupported covariance type %d", cov_type);
  }
  hipLaunchKernelGGL(ff_recip_kernel, dim3((n + 255) / 256), dim3(256), 0, stream_, n, vec_.get(), dinv);
  const double* dK[2] = {Kmn_.get(), Kd_.get()};
  const double* dKmm[2] = {Kmm_.get(), dKmm_.get()};
  const double base[2] = {var, 0.};
  for (int k = 0; k < 2; ++k) {   // dK_mm,k A into V_ (free after A), then the diagonal derivative
    gemm_f64(stream_, m, n, m, 1., dKmm[k], ldm, 0, A_.get(), ldm, 0, 0., V_.get(), ldm);
    hipLaunchKernelGGL(ff_diag_grad_kernel, dim3(nb4), dim3(256), 0, stream_, A_.get(), dK[k], V_.get(), n, m, ldm,
                       base[k], dd[k]);
  }
  HIP_CHECK(hipGetLastError());
  const int eb = (int)std::min<size_t>((nt + 255) / 256, 4096);
  auto rowscale = [&](const double* s, const double* X, double alpha, const double* Yin, double* Yo) {
    hipLaunchKernelGGL(ff_rowscale_kernel, dim3(eb), dim3(256), 0, stream_, n, t, s, X, alpha, Yin, Yo);
  };
  // Y = Psi^-1 X
  auto psi_inv = [&](const double* X, double* Yo) {
    rowscale(dinv, X, 1., nullptr, X1);
    gemm_f64(stream_, m, t, n, 1., Kmn_.get(), ldm, 0, X1, n, 0, 0., U, ldm);
    gemm_f64(stream_, m, t, m, 1., WiT_.get(), ldm, 1, U, ldm, 0, 0., U1, ldm, 0, 1, 0, 0);   // Lw^-1 U
    gemm_f64(stream_, m, t, m, 1., WiT_.get(), ldm, 0, U1, ldm, 0, 0., U, ldm, 0, 0, 1, 0);   // Lw^-T (.)
    gemm_f64(stream_, n, t, m, 1., Kmn_.get(), ldm, 1, U, ldm, 0, 0., T, n);
    rowscale(dinv, T, -1., X1, Yo);
  };
  // Y = G_k X (transformed-scale units)
  auto gmul = [&](int k, const double* X, double* Yo) {
    gemm_f64(stream_, m, t, n, 1., A_.get(), ldm, 0, X, n, 0, 0., AX, ldm);
    gemm_f64(stream_, m, t, n, 1., dK[k], ldm, 0, X, n, 0, 0., Q, ldm);
    gemm_f64(stream_, m, t, m, -1., dKmm[k], ldm, 0, AX, ldm, 0, 1., Q, ldm);
    gemm_f64(stream_, n, t, m, 1., A_.get(), ldm, 1, Q, ldm, 0, 0., Yo, n);
    gemm_f64(stream_, n, t, m, 1., dK[k], ldm, 1, AX, ldm, 0, 1., Yo, n);
    rowscale(dd[k], X, 1., Yo, Yo);
  };
  // probes: row-major n x t from the reference's generator, to the column-major block
  {
    std::vector<double> Zr(nt), Zh(nt);
    gen_probes_normal(n, t, seed, run_id, Zr.data());
    for (int i = 0; i < n; ++i)
      for (int c = 0; c < t; ++c) Zh[(size_t)c * n + i] = Zr[(size_t)i * t + c];
    HIP_CHECK(hipMemcpyAsync(Zc, Zh.data(), sizeof(double) * nt, hipMemcpyHostToDevice, stream_));
  }
  psi_inv(Zc, X0);
  for (int k = 0; k < 2; ++k) {
    gmul(k, Zc, Y);
    psi_inv(Y, S[k]);
    gmul(k, X0, Rk[k]);
  }
  const double* da[6] = {X0, X0, X0, Rk[0], Rk[0], Rk[1]};
  const double* db[6] = {X0, S[0], S[1], S[0], S[1], S[1]};
  for (int q = 0; q < 6; ++q) {
    hipLaunchKernelGGL(ff_dot_kernel, dim3(kDotBlocks), dim3(256), 0, stream_, nt, da[q], db[q], part.get());
    launch_sum_blocks(part.get(), kDotBlocks, 1, dots.get() + q, stream_);
  }
  HIP_CHECK(hipGetLastError());
  double h[6];
  HIP_CHECK(hipMemcpyAsync(h, dots.get(), sizeof(h), hipMemcpyDeviceToHost, stream_));
  HIP_CHECK(hipStreamSynchronize(stream_));
  const double s2 = orig[0];
  const double c[3] = {1., 1. / var, s2 * (cov_type == kGaussian ? -2. : -1.) / orig[2]};
  const int kl[6][2] = {{0, 0}, {0, 1}, {0, 2}, {1, 1}, {1, 2}, {2, 2}};
  for (int q = 0; q < 6; ++q) {
    const int k = kl[q][0], l = kl[q][1];
    const double v = 0.5 * h[q] / t * c[k] * c[l] / (s2 * s2);
    FI[k * 3 + l] = v;
    FI[l * 3 + k] = v;
  }
}

}  // namespace gpb_amd
