// Latent-model Vecchia predictions: the device parts of the predictive-variance simulation of
// PredictLaplaceApproxVecchia (likelihoods.h:6628-6746, iterative branch):
//   z ~ N(0, (Sigma^-1 + W)^-1) from (Sigma^-1 + W) z = B^T D^-1/2 e1 + W^1/2 e2, e1, e2 ~ N(0, I),
//   pred_var = Dp + mean over draws of (Bpo z)^2.
// The draws come from a counter-based generator (statistically equivalent to the reference's
// thread-seeded mt19937 streams, whose values depend on its OpenMP thread count).
#include <hip/hip_runtime.h>

#include "common.h"
#include "latent_kernels.h"

namespace gpb_amd {
namespace {

__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

// out[i * t + c] ~ N(0, 1), one Box-Muller pair per (row, column, stream): the value is a function of
// (seed, stream, global column c0 + c, row i) only.
__global__ void __launch_bounds__(256) gen_normal_kernel(int n, int t, uint64_t seed, int stream, long c0,
                                                         double* __restrict__ out) {
  const long k = (long)blockIdx.x * 256 + threadIdx.x;
  if (k >= (long)n * t) return;
  const long i = k / t, c = k - i * t;
  const uint64_t key = splitmix64(seed ^ splitmix64((uint64_t)stream * 0x100000001B3ull + (uint64_t)(c0 + c)));
  const uint64_t h = splitmix64(key + (uint64_t)i);
  const double u1 = ((h >> 11) + 0.5) * 0x1.0p-53;                      // (0, 1)
  const double u2 = (splitmix64(h) >> 11) * 0x1.0p-53;                  // [0, 1)
  out[k] = sqrt(-2. * log(u1)) * cospi(2. * u2);
}

__global__ void __launch_bounds__(256) sqrt_vec_kernel(int n, const double* __restrict__ x, double* __restrict__ y) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < n) y[i] = sqrt(x[i]);
}

// One wave per prediction point, lane = column: s_c = sum_r B[p, r] Z[nbr[p, r], c] (Bpo z_c, the
// minus sign of Bpo squared away), acc[p] += sum_c s_c^2 (fixed-order wave reduction).
__global__ void __launch_bounds__(256) pred_sq_acc_kernel(int n_pred, int mp, int t, const int* __restrict__ nbr,
                                                          const double* __restrict__ B, const double* __restrict__ Z,
                                                          double* __restrict__ acc) {
  const int p = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int c = threadIdx.x & 63;
  if (p >= n_pred) return;
  double s = 0.;
  if (c < t) {
    for (int r = 0; r < mp; ++r) {
      const double b = B[(size_t)p * mp + r];
      if (b != 0.) s = fma(b, Z[(size_t)nbr[(size_t)p * mp + r] * t + c], s);
    }
  }
  double q = s * s;
  for (int off = 32; off > 0; off >>= 1) q += __shfl_xor(q, off, 64);
  if (c == 0) acc[p] += q;
}

// The draws themselves (predictive covariance / cond_all): V[p + (col0 + c) * ldv] = sum_r B[p, r]
// Z[nbr[p, r], c] for the tc valid columns of the block; one thread per (point, column).
__global__ void __launch_bounds__(256) pred_samples_kernel(int n_pred, int mp, int t, int tc, const int* __restrict__ nbr,
                                                           const double* __restrict__ B, const double* __restrict__ Z,
                                                           double* __restrict__ V, int ldv, int col0) {
  const int p = blockIdx.x * 256 + threadIdx.x, c = blockIdx.y;
  if (p >= n_pred || c >= tc) return;
  double s = 0.;
  for (int r = 0; r < mp; ++r) {
    const double b = B[(size_t)p * mp + r];
    if (b != 0.) s = fma(b, Z[(size_t)nbr[(size_t)p * mp + r] * t + c], s);
  }
  V[(size_t)p + (size_t)(col0 + c) * ldv] = s;
}

__device__ __forceinline__ double sigmoid_stable(double x) {   // DF_utils.h:37-46
  if (x >= 0.) return 1. / (1. + exp(-x));
  const double t = exp(x);
  return t / (1. + t);
}

// Response mean of bernoulli_logit at latent N(mean, var) by the reference's adaptive
// Gauss-Hermite quadrature (RespMeanAdaptiveGHQuadrature, likelihoods.h:7857-7889): Newton for the
// mode of sigmoid(x) N(x; mu, var) from 0 (relative-update stop delta, <= 100 steps), then the
// order-point rule around it; var_out (nullable) = p (1 - p) (PredictResponse :7550-7555).
__global__ void __launch_bounds__(256) resp_logit_kernel(int n, const double* __restrict__ mean,
                                                         const double* __restrict__ var, const double* __restrict__ nodes,
                                                         const double* __restrict__ aw, int order, double delta,
                                                         double* __restrict__ out_mean, double* __restrict__ out_var) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const double mu = mean[i];
  const double s2inv = 1. / var[i];
  const double ss_inv = sqrt(s2inv);
  double mode = 0.;
  for (int it = 0; it < 100; ++it) {
    const double last = mode;
    const double p = sigmoid_stable(mode);
    const double upd = (sigmoid_stable(-mode) - s2inv * (mode - mu)) / (-p * (1. - p) - s2inv);
    mode -= upd;
    if (fabs(upd) / fabs(last) < delta) break;
  }
  const double p = sigmoid_stable(mode);
  const double sh = 1.4142135623730951 / sqrt(p * (1. - p) + s2inv);   // M_SQRT2 / sqrt(-f'' + 1/var)
  double r = 0.;
  for (int j = 0; j < order; ++j) {
    const double x = sh * nodes[j] + mode;
    const double z = ss_inv * (x - mu);
    r += aw[j] * sigmoid_stable(x) * (exp(-z * z / 2.) / 2.5066282746310002);   // normalPDF, DF_utils.h:62
  }
  r *= sh * ss_inv;
  out_mean[i] = r;
  if (out_var != nullptr) out_var[i] = r * (1. - r);
}

}  // namespace

void launch_resp_logit(int n, const double* mean, const double* var, const double* nodes, const double* aw, int order,
                       double delta, double* out_mean, double* out_var, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(resp_logit_kernel, dim3((n + 255) / 256), dim3(256), 0, s, n, mean, var, nodes, aw, order, delta,
                     out_mean, out_var);
  HIP_CHECK(hipGetLastError());
}

void launch_gen_normal(int n, int t, uint64_t seed, int stream, long c0, double* out, hipStream_t s) {
  const long cnt = (long)n * t;
  if (cnt <= 0) return;
  hipLaunchKernelGGL(gen_normal_kernel, dim3((unsigned)((cnt + 255) / 256)), dim3(256), 0, s, n, t, seed, stream, c0, out);
  HIP_CHECK(hipGetLastError());
}

void launch_sqrt_vec(int n, const double* x, double* y, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(sqrt_vec_kernel, dim3((n + 255) / 256), dim3(256), 0, s, n, x, y);
  HIP_CHECK(hipGetLastError());
}

void launch_pred_samples(int n_pred, int mp, int t, int tc, const int* nbr, const double* B, const double* Z, double* V,
                         int ldv, int col0, hipStream_t s) {
  if (n_pred <= 0 || tc <= 0) return;
  hipLaunchKernelGGL(pred_samples_kernel, dim3((n_pred + 255) / 256, tc), dim3(256), 0, s, n_pred, mp, t, tc, nbr, B, Z,
                     V, ldv, col0);
  HIP_CHECK(hipGetLastError());
}

void launch_pred_sq_acc(int n_pred, int mp, int t, const int* nbr, const double* B, const double* Z, double* acc,
                        hipStream_t s) {
  if (n_pred <= 0) return;
  if (t > 64) Fatal("pred_sq_acc: t = %d > 64", t);
  hipLaunchKernelGGL(pred_sq_acc_kernel, dim3((n_pred + 3) / 4), dim3(256), 0, s, n_pred, mp, t, nbr, B, Z, acc);
  HIP_CHECK(hipGetLastError());
}

}  // namespace gpb_amd
