// Laplace approximation on the dense covariance (dense_laplace.h gives the model and the reference lines).
// Per Newton step (n observations, Sigma full n x n column-major, ld a multiple of 64):
//   d1, W, W^1/2, rhs = W mode + d1                     one thread per observation
//   B = I + W^1/2 Sigma W^1/2, B = L L^T, L^-1             POTRF + TRTRI (MFMA trailing updates)
//   a_upd = rhs - W^1/2 L^-T L^-1 (W^1/2 Sigma rhs)        four one-column GEMMs, mode_upd = Sigma a_upd
//   Armijo line search on -1/2 a^T mode + sum log p(y | mode + F)
// and for the gradient Q = L^-1 W^1/2, R = Q^T Q = (W^-1 + Sigma)^-1, C = Q Sigma (two MFMA GEMMs), one fused
// pass over the columns of Sigma / R with the range derivative of Sigma recomputed from the coordinates.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>

#include "cov.h"
#include "dense.h"
#include "dense_laplace.h"
#include "kernels.h"
#include "lik_device.h"

namespace gpb_amd {
namespace {

constexpr int kT = 256;

__device__ __forceinline__ double wsum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ double block_sum(double v, double* red) {
  red[threadIdx.x] = v;
  __syncthreads();
  for (int off = kT / 2; off > 0; off >>= 1) {
    if ((int)threadIdx.x < off) red[threadIdx.x] += red[threadIdx.x + off];
    __syncthreads();
  }
  const double s = red[0];
  __syncthreads();
  return s;
}

__device__ __forceinline__ double sqdist(const double* X, const double* Y, int i, int j, int d) {
  double s = 0.;
  for (int q = 0; q < d; ++q) {
    const double t = X[(size_t)i * d + q] - Y[(size_t)j * d + q];
    s += t * t;
  }
  return s;
}

// Sigma (full, both triangles) = var corr(phi) (CalculateCovMat cov_fcts.h:564-679; diagonal var)
template <int COV>
__global__ void __launch_bounds__(kT) dl_build_sigma_kernel(const double* __restrict__ X, int n, int d, int ld,
                                                           double var, double phi, double* __restrict__ S) {
  const int i = blockIdx.x * 64 + (threadIdx.x & 63);
  const int j0 = blockIdx.y * 64;
  if (i >= n) return;
  for (int jj = threadIdx.x >> 6; jj < 64; jj += 4) {
    const int j = j0 + jj;
    if (j >= n) break;
    double c = var, dc;
    if (i != j) cov_dcov<COV>(sqrt(sqdist(X, X, i, j, d)), var, phi, c, dc);
    S[(size_t)i + (size_t)j * ld] = c;
  }
}

// C[i + p ld] = cov(x_i, xp_p) (n x np)
template <int COV>
__global__ void __launch_bounds__(kT) dl_cross_kernel(const double* __restrict__ X, const double* __restrict__ Xp, int n,
                                                     int np, int d, int ld, double var, double phi, double* __restrict__ C) {
  const int i = blockIdx.x * 64 + (threadIdx.x & 63);
  const int p = blockIdx.y * 4 + (threadIdx.x >> 6);
  if (i >= n || p >= np) return;
  const double s = sqdist(X, Xp, i, p, d);
  double c = var, dc;
  if (s != 0.) cov_dcov<COV>(sqrt(s), var, phi, c, dc);
  C[(size_t)i + (size_t)p * ld] = c;
}

// B = I + W^1/2 Sigma W^1/2, lower triangle (likelihoods.h:1890-1891)
__global__ void __launch_bounds__(kT) dl_build_b_kernel(const double* __restrict__ S, const double* __restrict__ ws, int n,
                                                       int ld, double* __restrict__ B) {
  const int i = blockIdx.x * 64 + (threadIdx.x & 63);
  const int j0 = blockIdx.y * 64;
  if (i >= n || j0 > i) return;
  const double wi = ws[i];
  for (int jj = threadIdx.x >> 6; jj < 64; jj += 4) {
    const int j = j0 + jj;
    if (j > i) break;
    const double v = (wi * S[(size_t)i + (size_t)j * ld]) * ws[j];
    B[(size_t)i + (size_t)j * ld] = i == j ? 1. + v : v;
  }
}

// Newton step quantities (likelihoods.h:1881-1895): d1, W, W^1/2, rhs = W mode + d1
__global__ void __launch_bounds__(kT) dl_prep_kernel(int n, int lik, double aux, const double* __restrict__ y,
                                                    const double* __restrict__ off, const double* __restrict__ mode,
                                                    double* __restrict__ d1, double* __restrict__ w,
                                                    double* __restrict__ ws, double* __restrict__ rhs) {
  const int i = blockIdx.x * kT + threadIdx.x;
  if (i >= n) return;
  const double mi = mode[i];
  const double l = off ? mi + off[i] : mi;
  const double g = lik_d1(lik, aux, y[i], l);
  const double wi = lik_info(lik, aux, y[i], l);
  d1[i] = g;
  w[i] = wi;
  ws[i] = sqrt(wi);
  if (rhs) rhs[i] = wi * mi + g;
}

__global__ void __launch_bounds__(kT) dl_mul_kernel(int n, const double* __restrict__ a, const double* __restrict__ b,
                                                   double* __restrict__ out) {
  const int i = blockIdx.x * kT + threadIdx.x;
  if (i < n) out[i] = a[i] * b[i];
}

// SigmaI_mode_update = rhs - W^1/2 B^-1 rhs2 (likelihoods.h:1900-1902)
__global__ void __launch_bounds__(kT) dl_aupd_kernel(int n, const double* __restrict__ rhs, const double* __restrict__ ws,
                                                    const double* __restrict__ t, double* __restrict__ aupd) {
  const int i = blockIdx.x * kT + threadIdx.x;
  if (i >= n) return;
  aupd[i] = (-t[i]) * ws[i] + rhs[i];
}

// Armijo slope: sum_i dir_i (aupd_i - a_i + W_i dir_i), dir = mupd - mode (likelihoods.h:1906-1909)
__global__ void __launch_bounds__(kT) dl_gdd_kernel(int n, const double* __restrict__ mode, const double* __restrict__ a,
                                                   const double* __restrict__ mupd, const double* __restrict__ aupd,
                                                   const double* __restrict__ w, double* __restrict__ part) {
  __shared__ double red[kT];
  double acc = 0.;
  for (int i = blockIdx.x * kT + threadIdx.x; i < n; i += gridDim.x * kT) {
    const double dir = mupd[i] - mode[i];
    acc += dir * (aupd[i] - a[i] + w[i] * dir);
  }
  const double s = block_sum(acc, red);
  if (threadIdx.x == 0) part[blockIdx.x] = s;
}

// one line-search trial (likelihoods.h:1910-1928) at learning rate lam; partials of [a^T mode, sum log p]
__global__ void __launch_bounds__(kT) dl_trial_kernel(int n, int lik, double aux, double lam, const double* __restrict__ mode,
                                                     const double* __restrict__ a, const double* __restrict__ mupd,
                                                     const double* __restrict__ aupd, const double* __restrict__ y,
                                                     const double* __restrict__ off, double* __restrict__ mnew,
                                                     double* __restrict__ anew, double* __restrict__ part) {
  __shared__ double red[kT];
  double sq = 0., sl = 0.;
  for (int i = blockIdx.x * kT + threadIdx.x; i < n; i += gridDim.x * kT) {
    double mi, ai;
    if (lam == 1.) {
      mi = mupd[i];
      ai = aupd[i];
    } else {
      ai = (1. - lam) * a[i] + lam * aupd[i];
      mi = (1. - lam) * mode[i] + lam * mupd[i];
    }
    mnew[i] = mi;
    anew[i] = ai;
    sq += ai * mi;
    sl += lik_loglik(lik, aux, y[i], off ? mi + off[i] : mi);
  }
  const double s0 = block_sum(sq, red);
  const double s1 = block_sum(sl, red);
  if (threadIdx.x == 0) {
    part[2 * blockIdx.x] = s0;
    part[2 * blockIdx.x + 1] = s1;
  }
}

// Q = L^-1 diag(W^1/2) in place (L_inv_Wsqrt, likelihoods.h:3298-3301): lower triangle, column scaling
__global__ void __launch_bounds__(kT) dl_colscale_lower_kernel(double* __restrict__ Q, const double* __restrict__ ws, int n,
                                                              int ld) {
  const int i = blockIdx.x * 64 + (threadIdx.x & 63);
  const int j0 = blockIdx.y * 64;
  if (i >= n || j0 > i) return;
  for (int jj = threadIdx.x >> 6; jj < 64; jj += 4) {
    const int j = j0 + jj;
    if (j > i) break;
    Q[(size_t)i + (size_t)j * ld] *= ws[j];
  }
}

// diag((Sigma^-1 + W)^-1) = diag(Sigma) - colsums(C o C), C = Q Sigma (likelihoods.h:3305-3311); then
// d_mll_d_mode = 1/2 diag o dW/dmode (:3315); one wave per column
__global__ void __launch_bounds__(kT) dl_dmll_kernel(const double* __restrict__ C, const double* __restrict__ S, int n, int ld,
                                                    int lik, double aux, const double* __restrict__ y,
                                                    const double* __restrict__ off, const double* __restrict__ mode,
                                                    double* __restrict__ dmll, double* __restrict__ dgo) {
  const int lane = threadIdx.x & 63;
  const int j = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (j >= n) return;
  double s = 0.;
  for (int k = lane; k < n; k += 64) {
    const double c = C[(size_t)k + (size_t)j * ld];
    s += c * c;
  }
  s = wsum(s);
  if (lane == 0) {
    const double dg = S[(size_t)j + (size_t)j * ld] - s;
    const double l = off ? mode[j] + off[j] : mode[j];
    dmll[j] = 0.5 * dg * lik_dinfo(lik, aux, y[j], l);
    if (dgo) dgo[j] = dg;
  }
}

// One wave per column j of the symmetric Sigma / R: cols[k ld + j] for
//   k = 0: (Sigma a)_j, 1: (dSigma_r a)_j, 2: (Sigma d1)_j, 3: (dSigma_r d1)_j, 4: sum_i R_ij Sigma_ij,
//   5: sum_i R_ij dSigma_r,ij       (dSigma_r = dSigma / dlog phi from the coordinates, 0 on the diagonal)
template <int COV>
__global__ void __launch_bounds__(kT) dl_grad_cols_kernel(const double* __restrict__ X, int n, int d, int ld, double var,
                                                         double phi, const double* __restrict__ S,
                                                         const double* __restrict__ R, const double* __restrict__ a,
                                                         const double* __restrict__ d1, double* __restrict__ cols) {
  const int lane = threadIdx.x & 63;
  const int j = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (j >= n) return;
  double s0 = 0., s1 = 0., s2 = 0., s3 = 0., s4 = 0., s5 = 0.;
  for (int i = lane; i < n; i += 64) {
    const double c = S[(size_t)i + (size_t)j * ld];
    double dc = 0., cc;
    if (i != j) cov_dcov<COV>(sqrt(sqdist(X, X, i, j, d)), var, phi, cc, dc);
    const double r = R[(size_t)i + (size_t)j * ld];
    const double ai = a[i], gi = d1[i];
    s0 += c * ai;
    s1 += dc * ai;
    s2 += c * gi;
    s3 += dc * gi;
    s4 += r * c;
    s5 += r * dc;
  }
  s0 = wsum(s0);
  s1 = wsum(s1);
  s2 = wsum(s2);
  s3 = wsum(s3);
  s4 = wsum(s4);
  s5 = wsum(s5);
  if (lane == 0) {
    cols[j] = s0;
    cols[(size_t)ld + j] = s1;
    cols[2 * (size_t)ld + j] = s2;
    cols[3 * (size_t)ld + j] = s3;
    cols[4 * (size_t)ld + j] = s4;
    cols[5 * (size_t)ld + j] = s5;
  }
}

// per-observation records of the gradient sums:
//   [a (Sigma a), a (dSigma_r a), R o Sigma, R o dSigma_r, dmll (dmode_var), dmll (dmode_range)],
//   dmode_k = u_k - Sigma R u_k (likelihoods.h:3343-3346), u = (Sigma d1, dSigma_r d1)
__global__ void __launch_bounds__(kT) dl_grad_rec_kernel(int n, int ld, const double* __restrict__ a,
                                                        const double* __restrict__ cols, const double* __restrict__ dmll,
                                                        const double* __restrict__ yv, const double* __restrict__ yr,
                                                        double* __restrict__ rec) {
  const int i = blockIdx.x * kT + threadIdx.x;
  if (i >= n) return;
  double* r = rec + (size_t)i * 6;
  r[0] = a[i] * cols[i];
  r[1] = a[i] * cols[(size_t)ld + i];
  r[2] = cols[4 * (size_t)ld + i];
  r[3] = cols[5 * (size_t)ld + i];
  r[4] = dmll[i] * (cols[2 * (size_t)ld + i] - yv[i]);
  r[5] = dmll[i] * (cols[3 * (size_t)ld + i] - yr[i]);
}

// gamma shape gradient records [l + y e^-l, W diag, d1 v] (likelihoods.h:3379-3411, 10514-10524, 10862-10868)
__global__ void __launch_bounds__(kT) dl_aux_rec_kernel(int n, const double* __restrict__ y, const double* __restrict__ off,
                                                       const double* __restrict__ mode, const double* __restrict__ w,
                                                       const double* __restrict__ dg, const double* __restrict__ d1,
                                                       const double* __restrict__ t, const double* __restrict__ v,
                                                       double* __restrict__ rec) {
  const int i = blockIdx.x * kT + threadIdx.x;
  if (i >= n) return;
  const double l = off ? mode[i] + off[i] : mode[i];
  rec[3 * (size_t)i] = l + y[i] * exp(-l);
  rec[3 * (size_t)i + 1] = w[i] * dg[i];
  rec[3 * (size_t)i + 2] = d1[i] * (t[i] - v[i]);
}

// fixed_effect_grad = -d1 + dmll - W o (Sigma dmll - C^T C dmll) (likelihoods.h:3354-3376)
__global__ void __launch_bounds__(kT) dl_gradf_kernel(int n, const double* __restrict__ d1, const double* __restrict__ dmll,
                                                     const double* __restrict__ w, const double* __restrict__ t,
                                                     const double* __restrict__ v, double* __restrict__ out) {
  const int i = blockIdx.x * kT + threadIdx.x;
  if (i >= n) return;
  out[i] = -d1[i] + (dmll[i] - (t[i] - v[i]) * w[i]);
}

// variances: var - column norms^2 of M (n x np)
__global__ void __launch_bounds__(kT) dl_predvar_kernel(const double* __restrict__ M, int n, int np, int ld, double var,
                                                       double* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int p = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (p >= np) return;
  double s = 0.;
  for (int i = lane; i < n; i += 64) {
    const double x = M[(size_t)i + (size_t)p * ld];
    s += x * x;
  }
  s = wsum(s);
  if (lane == 0) out[p] = var - s;
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

inline int nb_thread(int n) { return std::max(1, (n + kT - 1) / kT); }
inline int nb_red(int n) { return std::min(1024, nb_thread(n)); }

}  // namespace

DenseLaplace::DenseLaplace(int n, int d, const double* d_X, hipStream_t stream)
    : n_(n), d_(d), ld_(((n + 63) / 64) * 64), d_X_(d_X), s_(stream) {
  const size_t nn = (size_t)ld_ * ld_;
  for (DevBuf<double>* b : {&Sig_, &B_, &Li_, &R_, &C_}) {
    b->alloc(nn);
    HIP_CHECK(hipMemsetAsync(b->get(), 0, nn * sizeof(double), s_));
  }
  X_.alloc((size_t)ld_ * (ld_ / 2 + 64));
  for (DevBuf<double>* b : {&y_, &off_, &mode_, &a_, &mode_prev_, &a_prev_, &mode_upd_, &a_upd_, &d1_, &w_, &ws_, &rhs_,
                            &t1_, &t2_, &t3_, &t4_, &dmll_, &dg_, &uv_, &ur_}) {
    b->alloc(ld_);
    HIP_CHECK(hipMemsetAsync(b->get(), 0, sizeof(double) * ld_, s_));
  }
  rec_.alloc(std::max<size_t>((size_t)6 * ld_, (size_t)2 * nb_red(n)));
  cols_.alloc((size_t)6 * ld_);
  red_.alloc(32);
  info_.alloc(1);
  HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&h_red_), 32 * sizeof(double), hipHostMallocDefault));
  for (auto& e : ev_) HIP_CHECK(hipEventCreate(&e));
  HIP_CHECK(hipStreamSynchronize(s_));
}

DenseLaplace::~DenseLaplace() {
  if (h_red_) (void)hipHostFree(h_red_);
  for (auto& e : ev_)
    if (e) (void)hipEventDestroy(e);
}

void DenseLaplace::SetY(const double* y) {
  sum_log_y_ = 0.;   // aux_log_normalizing_constant_ of likelihood 'gamma' (likelihoods.h:8181-8191)
  for (int i = 0; i < n_; ++i) sum_log_y_ += y[i] > 0. ? std::log(y[i]) : 0.;
  HIP_CHECK(hipMemcpyAsync(y_.get(), y, sizeof(double) * n_, hipMemcpyHostToDevice, s_));
  HIP_CHECK(hipStreamSynchronize(s_));
  y_set_ = true;
}

void DenseLaplace::SetOffset(const double* off) {
  has_off_ = off != nullptr;
  if (has_off_) {
    HIP_CHECK(hipMemcpyAsync(off_.get(), off, sizeof(double) * n_, hipMemcpyHostToDevice, s_));
    HIP_CHECK(hipStreamSynchronize(s_));
  }
}

void DenseLaplace::GetMode(double* mode) {
  HIP_CHECK(hipMemcpyAsync(mode, mode_.get(), sizeof(double) * n_, hipMemcpyDeviceToHost, s_));
  HIP_CHECK(hipStreamSynchronize(s_));
}

void DenseLaplace::ResetModeToPrevious() {
  if (!prev_valid_) return;
  HIP_CHECK(hipMemcpyAsync(mode_.get(), mode_prev_.get(), sizeof(double) * n_, hipMemcpyDeviceToDevice, s_));
  HIP_CHECK(hipMemcpyAsync(a_.get(), a_prev_.get(), sizeof(double) * n_, hipMemcpyDeviceToDevice, s_));
  HIP_CHECK(hipStreamSynchronize(s_));
}

void DenseLaplace::BuildSigma(int cov_type, double var, double phi) {
  const int nt = (n_ + 63) / 64;
  dispatch_cov(cov_type, [&](auto c) {
    hipLaunchKernelGGL((dl_build_sigma_kernel<decltype(c)::value>), dim3(nt, nt), dim3(kT), 0, s_, d_X_, n_, d_, ld_, var,
                       phi, Sig_.get());
  });
  HIP_CHECK(hipGetLastError());
}

void DenseLaplace::FactorB(double* logdet_dev, bool with_inverse) {
  const int nt = (n_ + 63) / 64;
  hipLaunchKernelGGL(dl_build_b_kernel, dim3(nt, nt), dim3(kT), 0, s_, Sig_.get(), ws_.get(), n_, ld_, B_.get());
  HIP_CHECK(hipGetLastError());
  HIP_CHECK(hipMemsetAsync(info_.get(), 0, sizeof(int), s_));
  chol_lower(s_, B_.get(), Li_.get(), n_, ld_, info_.get());
  launch_logdet_chol(s_, B_.get(), ld_, n_, logdet_dev);
  if (with_inverse) trtri_lower(s_, B_.get(), Li_.get(), X_.get(), 0, n_, ld_);
}

void DenseLaplace::Gemv(const double* M, bool lower, bool trans, const double* x, double* y) {
  gemm_f64(s_, n_, 1, n_, 1., M, ld_, trans ? 1 : 0, x, ld_, 0, 0., y, ld_, 0, lower && !trans ? 1 : 0,
           lower && trans ? 1 : 0, 0);
}

bool DenseLaplace::InfoFailed() {
  int info = 0;
  HIP_CHECK(hipMemcpyAsync(&info, info_.get(), sizeof(int), hipMemcpyDeviceToHost, s_));
  HIP_CHECK(hipStreamSynchronize(s_));
  return info != 0;
}

LatentResult DenseLaplace::Eval(int cov_type, int lik, const double* trafo, double aux, const IterativeConfig& cfg,
                                bool want_grad, bool want_aux_grad, double* grad_f, ModeStart start) {
  if (!y_set_) Fatal("response variable y has not been set");
  aux_ = lik == kLikGamma ? aux : 1.;
  want_aux_grad = want_aux_grad && want_grad && lik == kLikGamma;
  if (lik == kLikGaussian) Fatal("DenseLaplace: the Gaussian likelihood uses the exact dense path");
  const int n = n_, ld = ld_;
  const double var = trafo[0], phi = trafo[1];
  cov_type_ = cov_type;
  var_ = var;
  phi_ = phi;
  const double* off = has_off_ ? off_.get() : nullptr;
  double* red = red_.get();
  HIP_CHECK(hipEventRecord(ev_[0], s_));
  BuildSigma(cov_type, var, phi);
  const int nbr = nb_red(n);
  auto objective = [&](double lam, const double* mu, const double* au, double* mnew, double* anew) {
    hipLaunchKernelGGL(dl_trial_kernel, dim3(nbr), dim3(kT), 0, s_, n, lik, aux_, lam, mode_.get(), a_.get(), mu, au, y_.get(),
                       off, mnew, anew, rec_.get());
    HIP_CHECK(hipGetLastError());
    launch_sum_blocks(rec_.get(), nbr, 2, red + 4, s_);
    HIP_CHECK(hipMemcpyAsync(h_red_ + 4, red + 4, 2 * sizeof(double), hipMemcpyDeviceToHost, s_));
    HIP_CHECK(hipStreamSynchronize(s_));
    return -0.5 * h_red_[4] + (h_red_[5] + loglik_const_);
  };
  LatentResult res;
  // mode start (likelihoods.h:1851-1865): zero, or mode = Sigma a of the previous a
  if (start == ModeStart::kZero || !evaluated_) {
    HIP_CHECK(hipMemsetAsync(mode_.get(), 0, sizeof(double) * n, s_));
    HIP_CHECK(hipMemsetAsync(a_.get(), 0, sizeof(double) * n, s_));
    prev_valid_ = false;
  } else if (start == ModeStart::kWarm) {
    HIP_CHECK(hipMemcpyAsync(mode_prev_.get(), mode_.get(), sizeof(double) * n, hipMemcpyDeviceToDevice, s_));
    HIP_CHECK(hipMemcpyAsync(a_prev_.get(), a_.get(), sizeof(double) * n, hipMemcpyDeviceToDevice, s_));
    prev_valid_ = true;
    Gemv(Sig_.get(), false, false, a_.get(), mode_.get());
  }
  double* logdet_B = red + 1;
  int it = 0;
  if (start != ModeStart::kKeep || !evaluated_) {
    double obj = objective(1., mode_.get(), a_.get(), mode_upd_.get(), a_upd_.get());
    const int maxit = 1000;                              // maxit_mode_newton_ (likelihoods.h:12721)
    const double delta = cfg.delta_conv_mode_finding;    // :12723
    bool terminate = false, has_nan = false;
    for (it = 0; it < maxit; ++it) {
      // the information changes in every step for the supported likelihoods (information_changes_during_mode_finding_)
      hipLaunchKernelGGL(dl_prep_kernel, dim3(nb_thread(n)), dim3(kT), 0, s_, n, lik, aux_, y_.get(), off, mode_.get(),
                         d1_.get(), w_.get(), ws_.get(), rhs_.get());
      HIP_CHECK(hipGetLastError());
      FactorB(logdet_B, true);
      // rhs2 = W^1/2 Sigma rhs; a_upd = rhs - W^1/2 L^-T L^-1 rhs2; mode_upd = Sigma a_upd (:1897-1903)
      Gemv(Sig_.get(), false, false, rhs_.get(), t1_.get());
      hipLaunchKernelGGL(dl_mul_kernel, dim3(nb_thread(n)), dim3(kT), 0, s_, n, ws_.get(), t1_.get(), t2_.get());
      Gemv(Li_.get(), true, false, t2_.get(), t3_.get());
      Gemv(Li_.get(), true, true, t3_.get(), t4_.get());
      hipLaunchKernelGGL(dl_aupd_kernel, dim3(nb_thread(n)), dim3(kT), 0, s_, n, rhs_.get(), ws_.get(), t4_.get(),
                         a_upd_.get());
      HIP_CHECK(hipGetLastError());
      Gemv(Sig_.get(), false, false, a_upd_.get(), mode_upd_.get());
      if (InfoFailed()) {
        has_nan = true;
        break;
      }
      hipLaunchKernelGGL(dl_gdd_kernel, dim3(nbr), dim3(kT), 0, s_, n, mode_.get(), a_.get(), mode_upd_.get(),
                         a_upd_.get(), w_.get(), rec_.get());
      launch_sum_blocks(rec_.get(), nbr, 1, red + 6, s_);
      HIP_CHECK(hipMemcpyAsync(h_red_ + 6, red + 6, sizeof(double), hipMemcpyDeviceToHost, s_));
      HIP_CHECK(hipStreamSynchronize(s_));
      const double gdd = h_red_[6];
      // backtracking (:1910-1928); the last trial is kept when none is accepted
      double lam = 1., obj_new = obj;
      for (int ih = 0; ih < 20; ++ih) {   // max_number_lr_shrinkage_steps_newton_ (:12725)
        obj_new = objective(lam, mode_upd_.get(), a_upd_.get(), t1_.get(), t2_.get());
        if (obj_new < obj + 1e-4 * lam * gdd || std::isnan(obj_new) || std::isinf(obj_new)) lam *= 0.5;   // c_armijo_
        else break;
      }
      std::swap(mode_, t1_);   // mode_ = mode_new, SigmaI_mode_ = SigmaI_mode_new
      std::swap(a_, t2_);
      // CheckConvergenceModeFinding (:11820-11870)
      if (std::isnan(obj_new) || std::isinf(obj_new)) {
        has_nan = true;
        obj = obj_new;
        break;
      }
      if (it == 0) terminate = std::abs(obj_new - obj) < delta * std::abs(obj);
      else terminate = (obj_new - obj) < delta * std::abs(obj);
      obj = obj_new;
      if (terminate) {
        ++it;
        break;
      }
    }
    if (has_nan) throw LatentNan("NaN or Inf occurred in the dense mode finding");
    res.newton_its = it;
    cached_obj_ = obj;
  }
  evaluated_ = true;
  // at the mode (:1941-1953): d1, W, B = I + W^1/2 Sigma W^1/2 = L L^T; mll = obj - sum log L_ii
  const bool need_inv = want_grad || want_aux_grad || grad_f != nullptr;
  hipLaunchKernelGGL(dl_prep_kernel, dim3(nb_thread(n)), dim3(kT), 0, s_, n, lik, aux_, y_.get(), off, mode_.get(), d1_.get(),
                     w_.get(), ws_.get(), nullptr);
  HIP_CHECK(hipGetLastError());
  FactorB(logdet_B, need_inv);
  HIP_CHECK(hipMemcpyAsync(h_red_, red, 2 * sizeof(double), hipMemcpyDeviceToHost, s_));
  if (InfoFailed()) throw LatentNan("I + W^1/2 Sigma W^1/2 is not positive definite (Cholesky failed)");
  const double mll = cached_obj_ - 0.5 * h_red_[1];
  res.nll = -mll;
  res.logdet = 0.5 * h_red_[1];
  if (!std::isfinite(res.nll)) throw LatentNan("NaN or Inf in the dense approximate marginal likelihood");
  if (need_inv) {
    const int nt = (n + 63) / 64;
    double* Q = Li_.get();
    hipLaunchKernelGGL(dl_colscale_lower_kernel, dim3(nt, nt), dim3(kT), 0, s_, Q, ws_.get(), n, ld);
    HIP_CHECK(hipGetLastError());
    // C = Q Sigma (Q lower), R = Q^T Q
    gemm_f64(s_, n, n, n, 1., Q, ld, 0, Sig_.get(), ld, 0, 0., C_.get(), ld, 0, 1, 0, 0);
    gemm_f64(s_, n, n, n, 1., Q, ld, 1, Q, ld, 0, 0., R_.get(), ld, 0, 0, 1, 1);
    hipLaunchKernelGGL(dl_dmll_kernel, dim3((n + 3) / 4), dim3(kT), 0, s_, C_.get(), Sig_.get(), n, ld, lik, aux_, y_.get(),
                       off, mode_.get(), dmll_.get(), dg_.get());
    HIP_CHECK(hipGetLastError());
    if (want_grad) {
      double* recs = rec_.get();   // n records of 6
      dispatch_cov(cov_type, [&](auto c) {
        hipLaunchKernelGGL((dl_grad_cols_kernel<decltype(c)::value>), dim3((n + 3) / 4), dim3(kT), 0, s_, d_X_, n, d_, ld,
                           var, phi, Sig_.get(), R_.get(), a_.get(), d1_.get(), cols_.get());
      });
      HIP_CHECK(hipGetLastError());
      const double* cb = cols_.get();
      // implicit terms: y_k = Sigma (R u_k)
      Gemv(R_.get(), false, false, cb + 2 * (size_t)ld, t1_.get());
      Gemv(Sig_.get(), false, false, t1_.get(), uv_.get());
      Gemv(R_.get(), false, false, cb + 3 * (size_t)ld, t1_.get());
      Gemv(Sig_.get(), false, false, t1_.get(), ur_.get());
      hipLaunchKernelGGL(dl_grad_rec_kernel, dim3(nb_thread(n)), dim3(kT), 0, s_, n, ld, a_.get(), cb, dmll_.get(),
                         uv_.get(), ur_.get(), recs);
      HIP_CHECK(hipGetLastError());
      launch_sum_blocks(recs, n, 6, red + 8, s_);
      HIP_CHECK(hipMemcpyAsync(h_red_ + 8, red + 8, 6 * sizeof(double), hipMemcpyDeviceToHost, s_));
      HIP_CHECK(hipStreamSynchronize(s_));
      const double* g = h_red_ + 8;
      // cov_grad = -1/2 a^T dSigma a + 1/2 tr((W^-1 + Sigma)^-1 dSigma) + d_mll_d_mode^T d_mode (:3338-3346)
      res.grad = {-0.5 * g[0] + 0.5 * g[2] + g[4], -0.5 * g[1] + 0.5 * g[3] + g[5]};
    }
    if (grad_f != nullptr || want_aux_grad) {   // SigmaI_plus_W_inv_d_mll_d_mode = Sigma dmll - C^T C dmll (:3354-3358)
      Gemv(Sig_.get(), false, false, dmll_.get(), t1_.get());
      Gemv(C_.get(), false, false, dmll_.get(), t2_.get());
      Gemv(C_.get(), false, true, t2_.get(), t3_.get());
    }
    if (want_aux_grad) {
      // gamma shape on the log scale: a [sum (l + y e^-l) - n (log a + 1 - digamma(a)) - sum log y]
      // + 1/2 sum W_i diag_i + sum d1_i (Sigma dmll - C^T C dmll)_i  (dW/dlog a = W, d2 ll / dl dlog a = d1)
      hipLaunchKernelGGL(dl_aux_rec_kernel, dim3(nb_thread(n)), dim3(kT), 0, s_, n, y_.get(), off, mode_.get(), w_.get(),
                         dg_.get(), d1_.get(), t1_.get(), t3_.get(), rec_.get());
      HIP_CHECK(hipGetLastError());
      launch_sum_blocks(rec_.get(), n, 3, red + 16, s_);
      HIP_CHECK(hipMemcpyAsync(h_red_ + 16, red + 16, 3 * sizeof(double), hipMemcpyDeviceToHost, s_));
      HIP_CHECK(hipStreamSynchronize(s_));
      const double a = aux_;
      double neg = h_red_[16] - n * (std::log(a) + 1. - digamma_asa103(a)) - sum_log_y_;
      neg *= a;
      if (res.grad.empty()) res.grad = {0., 0.};
      res.grad.push_back(neg + 0.5 * h_red_[17] + h_red_[18]);
    }
    if (grad_f != nullptr) {
      hipLaunchKernelGGL(dl_gradf_kernel, dim3(nb_thread(n)), dim3(kT), 0, s_, n, d1_.get(), dmll_.get(), w_.get(),
                         t1_.get(), t3_.get(), t4_.get());
      HIP_CHECK(hipGetLastError());
      HIP_CHECK(hipMemcpyAsync(grad_f, t4_.get(), sizeof(double) * n, hipMemcpyDeviceToHost, s_));
    }
  }
  HIP_CHECK(hipEventRecord(ev_[1], s_));
  HIP_CHECK(hipEventSynchronize(ev_[1]));
  float ms = 0.f;
  HIP_CHECK(hipEventElapsedTime(&ms, ev_[0], ev_[1]));
  res.ms_total = ms;
  return res;
}

void DenseLaplace::Predict(int cov_type, double var, double phi, const double* Xp, int np, bool want_var, bool want_cov,
                           double* mean, double* pvar, double* pcov) {
  if (!evaluated_) Fatal("DenseLaplace::Predict: no mode has been found");
  const int n = n_, ld = ld_, d = d_;
  DevBuf<double> dXp((size_t)np * d), Cp((size_t)ld * np), m(np);
  HIP_CHECK(hipMemcpyAsync(dXp.get(), Xp, sizeof(double) * np * d, hipMemcpyHostToDevice, s_));
  dispatch_cov(cov_type, [&](auto c) {
    hipLaunchKernelGGL((dl_cross_kernel<decltype(c)::value>), dim3((n + 63) / 64, (np + 3) / 4), dim3(kT), 0, s_, d_X_,
                       dXp.get(), n, np, d, ld, var, phi, Cp.get());
  });
  HIP_CHECK(hipGetLastError());
  // pred_mean = Cross_Cov d1 (likelihoods.h:5629-5631)
  gemm_f64(s_, np, 1, n, 1., Cp.get(), ld, 1, d1_.get(), ld, 0, 0., m.get(), np);
  HIP_CHECK(hipMemcpyAsync(mean, m.get(), sizeof(double) * np, hipMemcpyDeviceToHost, s_));
  if (want_var || want_cov) {
    // M = L^-1 W^1/2 Sigma_op (:5663-5664) with L = chol(I + W^1/2 Sigma W^1/2) at the mode
    double* red = red_.get();
    FactorB(red + 1, true);
    const int nt = (n + 63) / 64;
    hipLaunchKernelGGL(dl_colscale_lower_kernel, dim3(nt, nt), dim3(kT), 0, s_, Li_.get(), ws_.get(), n, ld);
    HIP_CHECK(hipGetLastError());
    DevBuf<double> M((size_t)ld * np);
    gemm_f64(s_, n, np, n, 1., Li_.get(), ld, 0, Cp.get(), ld, 0, 0., M.get(), ld, 0, 1, 0, 0);
    if (want_cov) {
      DevBuf<double> Spp((size_t)np * np);
      dispatch_cov(cov_type, [&](auto c) {
        hipLaunchKernelGGL((dl_cross_kernel<decltype(c)::value>), dim3((np + 63) / 64, (np + 3) / 4), dim3(kT), 0, s_,
                           dXp.get(), dXp.get(), np, np, d, np, var, phi, Spp.get());
      });
      HIP_CHECK(hipGetLastError());
      gemm_f64(s_, np, np, n, -1., M.get(), ld, 1, M.get(), ld, 0, 1., Spp.get(), np);
      HIP_CHECK(hipMemcpyAsync(pcov, Spp.get(), sizeof(double) * np * np, hipMemcpyDeviceToHost, s_));
    }
    if (want_var) {
      DevBuf<double> v(np);
      hipLaunchKernelGGL(dl_predvar_kernel, dim3((np + 3) / 4), dim3(kT), 0, s_, M.get(), n, np, ld, var, v.get());
      HIP_CHECK(hipGetLastError());
      HIP_CHECK(hipMemcpyAsync(pvar, v.get(), sizeof(double) * np, hipMemcpyDeviceToHost, s_));
    }
    if (InfoFailed()) Fatal("I + W^1/2 Sigma W^1/2 is not positive definite (Cholesky failed)");
  }
  HIP_CHECK(hipStreamSynchronize(s_));
}

}  // namespace gpb_amd
