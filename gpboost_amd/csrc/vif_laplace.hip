// VifLaplace (vif_laplace.h): the full-scale Vecchia Laplace approximation with the sparse Cholesky of
// A = B^T D^-1 B + W (sparse_chol.h) and the m x m Woodbury matrices of the low-rank part.
//
// Device layout: n x m column sets are kept point-major (m x n, leading dimension ldm: point i's m values
// contiguous), as in VifSolver; the sparse solves take them column-major (n x m, ld n) through a tiled
// transpose. Per Newton step: one numeric factorization of A, one forward solve with the m columns of
// C = R K (M2 = M - (L^-1 C)^T (L^-1 C) by the split-K MFMA Gram), two vector solves. Gradient: the selected
// inverse of A (traces tr(S' A^-1), diag A^-1), one solve with m columns (A^-1 C), three m x n GEMMs with
// M2^-1, the sparse products R X / S' X over m-columns, and Frobenius products for the m x m traces.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <limits>
#include <string>
#include <utility>
#include <vector>

#include "dense.h"
#include "fitc.h"
#include "kernels.h"
#include "latent_kernels.h"
#include "lik_device.h"
#include "vif_laplace.h"

namespace gpb_amd {
namespace {

constexpr int kT = 256;
constexpr int kNvl = 14;                              // n-vector scratch slots
constexpr int kMvl = 16;                              // m-vector scratch slots
constexpr double kMaxChangeMode = 4.605170185988091;  // MAX_CHANGE_MODE_NEWTON_ = log(100) (likelihoods.h:12733)
constexpr double kCArmijo = 1e-4;                     // c_armijo_ (likelihoods.h:12737)

inline int nblk(int n) { return std::max(1, std::min(1024, (n + kT - 1) / kT)); }

__device__ __forceinline__ double wsum64(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// fixed-order block sum of per-thread values (4 waves)
__device__ __forceinline__ double block_sum(double v, double* red) {
  v = wsum64(v);
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (lane == 0) red[w] = v;
  __syncthreads();
  const double s = (red[0] + red[1]) + (red[2] + red[3]);
  __syncthreads();
  return s;
}

__global__ void __launch_bounds__(kT) vl_recip_kernel(int n, const double* __restrict__ D, double* __restrict__ out) {
  const int i = blockIdx.x * kT + threadIdx.x;
  if (i < n) out[i] = 1. / D[i];
}

// d1, W (information), dW (its derivative) at loc = mode + F; rhs = W mode + d1 (likelihoods.h:2585)
__global__ void __launch_bounds__(kT) vl_prep_kernel(int n, int lik, double aux, const double* __restrict__ y,
                                                     const double* __restrict__ off, const double* __restrict__ mode,
                                                     double* __restrict__ d1, double* __restrict__ W,
                                                     double* __restrict__ dW, double* __restrict__ rhs,
                                                     double* __restrict__ part) {
  __shared__ double red[4];
  double zeros = 0.;
  for (int i = blockIdx.x * kT + threadIdx.x; i < n; i += gridDim.x * kT) {
    const double loc = off ? mode[i] + off[i] : mode[i];
    const double a = lik_d1(lik, aux, y[i], loc), w = lik_info(lik, aux, y[i], loc);
    d1[i] = a;
    W[i] = w;
    if (dW) dW[i] = lik_dinfo(lik, aux, y[i], loc);
    if (rhs) rhs[i] = w * mode[i] + a;
    zeros += w == 0. ? 1. : 0.;
  }
  const double s = block_sum(zeros, red);
  if (part && threadIdx.x == 0) part[blockIdx.x] = s;
}

// trial mode (first: the update itself, else (1 - lam) mode + lam upd), capped for poisson / gamma
// (CapChangeModeUpdateNewton :11800-11810), and the block partials of log p(y | trial + F)
__global__ void __launch_bounds__(kT) vl_trial_kernel(int n, int lik, double aux, const double* __restrict__ y,
                                                      const double* __restrict__ off, const double* __restrict__ mode,
                                                      const double* __restrict__ upd, double lam, int first, int cap,
                                                      double* __restrict__ trial, double* __restrict__ part) {
  __shared__ double red[4];
  double ll = 0.;
  for (int i = blockIdx.x * kT + threadIdx.x; i < n; i += gridDim.x * kT) {
    double t = first ? upd[i] : (1. - lam) * mode[i] + lam * upd[i];
    if (cap) {
      const double c = fabs(t - mode[i]);
      if (c > kMaxChangeMode) t = mode[i] + (t - mode[i]) / c * kMaxChangeMode;
    }
    trial[i] = t;
    ll += lik_loglik(lik, aux, y[i], off ? t + off[i] : t);
  }
  const double s = block_sum(ll, red);
  if (threadIdx.x == 0) part[blockIdx.x] = s;
}

// block partials of sum a_i b_i c_i (b, c nullable = 1)
__global__ void __launch_bounds__(kT) vl_dot_kernel(int n, const double* __restrict__ a, const double* __restrict__ b,
                                                    const double* __restrict__ c, double* __restrict__ part) {
  __shared__ double red[4];
  double acc = 0.;
  for (int i = blockIdx.x * kT + threadIdx.x; i < n; i += gridDim.x * kT) {
    double v = a[i];
    if (b) v *= b[i];
    if (c) v *= c[i];
    acc += v;
  }
  const double s = block_sum(acc, red);
  if (threadIdx.x == 0) part[blockIdx.x] = s;
}

// out = a . b over m entries (one block, fixed order)
__global__ void __launch_bounds__(kT) vl_mdot_kernel(int m, const double* __restrict__ a, const double* __restrict__ b,
                                                     double* __restrict__ out) {
  __shared__ double red[4];
  double acc = 0.;
  for (int j = threadIdx.x; j < m; j += kT) acc += a[j] * b[j];
  const double s = block_sum(acc, red);
  if (threadIdx.x == 0) *out = s;
}

__global__ void __launch_bounds__(kT) vl_mul_kernel(int n, const double* __restrict__ a, const double* __restrict__ b,
                                                    double* __restrict__ out) {
  const int i = blockIdx.x * kT + threadIdx.x;
  if (i < n) out[i] = a[i] * b[i];
}

// out = (e - dD o u) o dinv
__global__ void __launch_bounds__(kT) vl_zvec_kernel(int n, const double* __restrict__ e, const double* __restrict__ dD,
                                                     const double* __restrict__ u, const double* __restrict__ dinv,
                                                     double* __restrict__ out) {
  const int i = blockIdx.x * kT + threadIdx.x;
  if (i < n) out[i] = (e[i] - dD[i] * u[i]) * dinv[i];
}

// point-major m x n sets: E_i = (E_i - dD_i U_i) / D_i
__global__ void __launch_bounds__(kT) vl_zmat_kernel(int n, int m, int ldm, double* __restrict__ E,
                                                     const double* __restrict__ U, const double* __restrict__ dD,
                                                     const double* __restrict__ D) {
  const int lane = threadIdx.x & 63;
  const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (i >= n) return;
  const double dd = dD[i], inv = 1. / D[i];
  for (int q = lane; q < m; q += 64) {
    const size_t e = (size_t)i * ldm + q;
    E[e] = (E[e] - dd * U[e]) * inv;
  }
}

// M2 = M - sum of the split-K Gram chunks
__global__ void __launch_bounds__(kT) vl_m2_kernel(const double* __restrict__ P, int chunks, long stride, int m, int ldm,
                                                   const double* __restrict__ M, double* __restrict__ M2) {
  const int j = blockIdx.x * 64 + (threadIdx.x & 63);
  const int k = blockIdx.y * 4 + (threadIdx.x >> 6);
  if (j >= m || k >= m) return;
  const size_t e = (size_t)j + (size_t)k * ldm;
  double s = P[e];
  for (int z = 1; z < chunks; ++z) s += P[(size_t)z * stride + e];
  M2[e] = M[e] - s;
}

// point-major m x n (ld ldm) <-> column-major n x m (ld n), 64 x 64 tiles through LDS
__global__ void __launch_bounds__(kT) vl_to_nm_kernel(const double* __restrict__ mn, int n, int m, int ldm,
                                                      double* __restrict__ nm) {
  __shared__ double tile[64][65];
  const int i0 = blockIdx.x * 64, q0 = blockIdx.y * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  for (int r = ty; r < 64; r += 4) {
    const int i = i0 + r, q = q0 + tx;
    tile[r][tx] = (i < n && q < m) ? mn[(size_t)i * ldm + q] : 0.;
  }
  __syncthreads();
  for (int r = ty; r < 64; r += 4) {
    const int q = q0 + r, i = i0 + tx;
    if (i < n && q < m) nm[(size_t)q * n + i] = tile[tx][r];
  }
}

__global__ void __launch_bounds__(kT) vl_to_mn_kernel(const double* __restrict__ nm, int n, int m, int ldm,
                                                      double* __restrict__ mn) {
  __shared__ double tile[64][65];
  const int i0 = blockIdx.x * 64, q0 = blockIdx.y * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  for (int r = ty; r < 64; r += 4) {
    const int q = q0 + r, i = i0 + tx;
    tile[r][tx] = (i < n && q < m) ? nm[(size_t)q * n + i] : 0.;
  }
  __syncthreads();
  for (int r = ty; r < 64; r += 4) {
    const int i = i0 + r, q = q0 + tx;
    if (i < n && q < ldm) mn[(size_t)i * ldm + q] = q < m ? tile[tx][r] : 0.;
  }
}

// d_mll_d_mode = 1/2 (diag A^-1 + cd) o dW (likelihoods.h:4760-4763)
__global__ void __launch_bounds__(kT) vl_dmll_kernel(int n, const double* __restrict__ diagS, const double* __restrict__ cd,
                                                     const double* __restrict__ dW, double* __restrict__ full,
                                                     double* __restrict__ dmll) {
  const int i = blockIdx.x * kT + threadIdx.x;
  if (i >= n) return;
  const double f = diagS[i] + cd[i];
  full[i] = f;
  dmll[i] = 0.5 * f * dW[i];
}

// gradient wrt F: -d1 + d_mll - W o v (likelihoods.h:4890-4893)
__global__ void __launch_bounds__(kT) vl_gradf_kernel(int n, const double* __restrict__ d1, const double* __restrict__ dmll,
                                                      const double* __restrict__ W, const double* __restrict__ v,
                                                      double* __restrict__ out) {
  const int i = blockIdx.x * kT + threadIdx.x;
  if (i < n) out[i] = -d1[i] + dmll[i] - W[i] * v[i];
}

// gamma shape: block partials of [sum (loc + y e^-loc), sum W (diag_full + diag A^-1), sum d1 v]
__global__ void __launch_bounds__(kT) vl_gamma_kernel(int n, const double* __restrict__ y, const double* __restrict__ off,
                                                      const double* __restrict__ mode, const double* __restrict__ W,
                                                      const double* __restrict__ full, const double* __restrict__ diagS,
                                                      const double* __restrict__ d1, const double* __restrict__ v,
                                                      double* __restrict__ part) {
  __shared__ double red[4];
  double a0 = 0., a1 = 0., a2 = 0.;
  for (int i = blockIdx.x * kT + threadIdx.x; i < n; i += gridDim.x * kT) {
    const double loc = off ? mode[i] + off[i] : mode[i];
    a0 += loc + y[i] * exp(-loc);
    a1 += W[i] * (full[i] + diagS[i]);
    a2 += d1[i] * v[i];
  }
  const double s0 = block_sum(a0, red), s1 = block_sum(a1, red), s2 = block_sum(a2, red);
  if (threadIdx.x == 0) {
    part[(size_t)blockIdx.x * 3] = s0;
    part[(size_t)blockIdx.x * 3 + 1] = s1;
    part[(size_t)blockIdx.x * 3 + 2] = s2;
  }
}

// point-major m x n: out_i = K_i * s_i
__global__ void __launch_bounds__(kT) vl_colscale_kernel(int n, int m, int ldm, const double* __restrict__ K,
                                                         const double* __restrict__ sc, double* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (i >= n) return;
  const double f = sc[i];
  for (int q = lane; q < m; q += 64) out[(size_t)i * ldm + q] = K[(size_t)i * ldm + q] * f;
}

// out = add (nullable) + sum of the split-K chunks
__global__ void __launch_bounds__(kT) vl_psum_kernel(const double* __restrict__ P, int chunks, long stride, int m, int ldm,
                                                     const double* __restrict__ add, double* __restrict__ out) {
  const int j = blockIdx.x * 64 + (threadIdx.x & 63);
  const int k = blockIdx.y * 4 + (threadIdx.x >> 6);
  if (j >= m || k >= m) return;
  const size_t e = (size_t)j + (size_t)k * ldm;
  double s = P[e];
  for (int z = 1; z < chunks; ++z) s += P[(size_t)z * stride + e];
  out[e] = add ? add[e] + s : s;
}

// out[p] = sum_k M(k, p)^2 over the n rows of column p (column-major n x np), one block per column
__global__ void __launch_bounds__(kT) vl_colsq_kernel(int n, const double* __restrict__ M, double* __restrict__ out) {
  __shared__ double red[4];
  const double* c = M + (size_t)blockIdx.x * n;
  double acc = 0.;
  for (int k = threadIdx.x; k < n; k += kT) acc += c[k] * c[k];
  const double s = block_sum(acc, red);
  if (threadIdx.x == 0) out[blockIdx.x] = s;
}

// the low-rank terms of the predictive variance (likelihoods.h:6539-6543), columns p of m x np sets:
// |Vp|^2 - Sig . X1 + X2 . X1 + 2 Sig . X3 - 2 X2 . X3 + X4 . X3
__global__ void __launch_bounds__(kT) vl_pvar_kernel(int np, int m, int ldm, const double* __restrict__ Vp,
                                                     const double* __restrict__ Sig, const double* __restrict__ X1,
                                                     const double* __restrict__ X2, const double* __restrict__ X3,
                                                     const double* __restrict__ X4, double* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int p = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (p >= np) return;
  const size_t o = (size_t)p * ldm;
  double s = 0.;
  for (int q = lane; q < m; q += 64) {
    const double v = Vp[o + q], sg = Sig[o + q], x1 = X1[o + q], x2 = X2[o + q], x3 = X3[o + q], x4 = X4[o + q];
    s += v * v - sg * x1 + x2 * x1 + 2. * sg * x3 - 2. * x2 * x3 + x4 * x3;
  }
  s = wsum64(s);
  if (lane == 0) out[p] = s;
}

}  // namespace

VifLaplace::VifLaplace(VifSolver* vif, const std::vector<int>& nbr, const std::vector<double>& X, hipStream_t stream)
    : V_(vif), s_(stream), n_(vif->n_), m_(vif->m_), ldm_(vif->ldm_) {
  V_->latent_ = true;
  chol_.reset(new SparseChol(n_, V_->nn_, nbr.data(), V_->d_, X.data(), stream));
  const int n = n_;
  for (DevBuf<double>* b : {&y_, &off_, &mode_, &mode_prev_, &upd_, &trial_, &d1_, &w_, &dw_, &rhs_, &dinv_, &diagS_,
                            &dmll_, &vS_})
    b->alloc(n);
  HIP_CHECK(hipMemsetAsync(mode_.get(), 0, sizeof(double) * n, s_));
  vec_.alloc((size_t)kNvl * n);
  mv_.alloc((size_t)kMvl * ldm_);
  HIP_CHECK(hipMemsetAsync(mv_.get(), 0, sizeof(double) * mv_.size(), s_));
  const size_t mm = (size_t)ldm_ * ldm_;
  for (DevBuf<double>* b : {&M_, &M2_, &M2i_, &M2iT_, &M2inv_}) {
    b->alloc(mm);
    HIP_CHECK(hipMemsetAsync(b->get(), 0, sizeof(double) * mm, s_));
  }
  const size_t mn = (size_t)ldm_ * n;
  for (DevBuf<double>* b : {&C_, &Cnm_, &CL_}) {
    b->alloc(mn);
    HIP_CHECK(hipMemsetAsync(b->get(), 0, sizeof(double) * mn, s_));
  }
  part_.alloc((size_t)1024 * 8);
  red_.alloc(64);
  info_.alloc(1);
  HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&h_red_), 64 * sizeof(double), hipHostMallocDefault));
  for (auto& e : ev_) HIP_CHECK(hipEventCreate(&e));
  HIP_CHECK(hipStreamSynchronize(s_));
}

VifLaplace::~VifLaplace() {
  V_->latent_ = false;   // the solver serves the Gaussian likelihood again (SetLikelihood)
  if (h_red_) (void)hipHostFree(h_red_);
  for (auto& e : ev_) if (e) (void)hipEventDestroy(e);
}

void VifLaplace::SetY(const double* y) {
  HIP_CHECK(hipMemcpyAsync(y_.get(), y, sizeof(double) * n_, hipMemcpyHostToDevice, s_));
  HIP_CHECK(hipStreamSynchronize(s_));
  sum_log_y_ = 0.;   // aux_log_normalizing_constant_ of likelihood 'gamma' (likelihoods.h:8181-8191)
  for (int i = 0; i < n_; ++i) sum_log_y_ += y[i] > 0. ? std::log(y[i]) : 0.;
  y_set_ = true;
}

void VifLaplace::SetOffset(const double* off) {
  has_off_ = off != nullptr;
  if (has_off_) {
    HIP_CHECK(hipMemcpyAsync(off_.get(), off, sizeof(double) * n_, hipMemcpyHostToDevice, s_));
    HIP_CHECK(hipStreamSynchronize(s_));
  }
}

void VifLaplace::SetGradOffset(const double* off) {
  has_goff_ = off != nullptr;
  if (has_goff_) {
    for (DevBuf<double>* b : {&goff_, &gd1_, &gw_})
      if (b->size() < (size_t)n_) b->alloc(n_);
    HIP_CHECK(hipMemcpyAsync(goff_.get(), off, sizeof(double) * n_, hipMemcpyHostToDevice, s_));
    HIP_CHECK(hipStreamSynchronize(s_));
  }
}

void VifLaplace::GetMode(double* mode) {
  HIP_CHECK(hipMemcpyAsync(mode, mode_.get(), sizeof(double) * n_, hipMemcpyDeviceToHost, s_));
  HIP_CHECK(hipStreamSynchronize(s_));
}

void VifLaplace::ResetModeToPrevious() {
  if (prev_valid_) launch_copy(n_, mode_prev_.get(), mode_.get(), s_);
}

void VifLaplace::ToNM(const double* mn, double* nm) {
  hipLaunchKernelGGL(vl_to_nm_kernel, dim3((n_ + 63) / 64, (m_ + 63) / 64), dim3(kT), 0, s_, mn, n_, m_, ldm_, nm);
  HIP_CHECK(hipGetLastError());
}

void VifLaplace::ToMN(const double* nm, double* mn) {
  hipLaunchKernelGGL(vl_to_mn_kernel, dim3((n_ + 63) / 64, (ldm_ + 63) / 64), dim3(kT), 0, s_, nm, n_, m_, ldm_, mn);
  HIP_CHECK(hipGetLastError());
}

void VifLaplace::RVec(const double* x, double* out, double* t) {
  V_->BVec(x, V_->Bv_.get(), 1., t);
  hipLaunchKernelGGL(vl_mul_kernel, dim3((n_ + kT - 1) / kT), dim3(kT), 0, s_, n_, t, dinv_.get(), t);
  HIP_CHECK(hipGetLastError());
  V_->BtVec(t, V_->BvT_.get(), 1., out);
}

void VifLaplace::SpVec(const double* x, double* out, double* t, double* t2) {
  // S'_1 x = dB^T u + B^T D^-1 (dB x - dD o u), u = D^-1 B x (SigmaI_deriv, likelihoods.h:4758-4762)
  V_->BVec(x, V_->Bv_.get(), 1., t);
  hipLaunchKernelGGL(vl_mul_kernel, dim3((n_ + kT - 1) / kT), dim3(kT), 0, s_, n_, t, dinv_.get(), t);
  V_->BVec(x, V_->dBv1_.get(), 0., t2);
  hipLaunchKernelGGL(vl_zvec_kernel, dim3((n_ + kT - 1) / kT), dim3(kT), 0, s_, n_, t2, V_->dD1_.get(), t,
                     dinv_.get(), t2);
  HIP_CHECK(hipGetLastError());
  V_->BtVec(t2, V_->BvT_.get(), 1., out);
  V_->BtVec(t, V_->dBvT1_.get(), 0., t2);
  launch_axpby(n_, 1., out, 1., t2, out, s_);
}

void VifLaplace::RMat(const double* X, double* out, double* t) {
  V_->BRow(X, V_->Bv_.get(), 1., true, t);
  V_->BCol(t, V_->BvT_.get(), 1., out);
}

void VifLaplace::SpMat(const double* X, double* out, double* t, double* t2) {
  V_->BRow(X, V_->Bv_.get(), 1., true, t);      // U = D^-1 B X
  V_->BRow(X, V_->dBv1_.get(), 0., false, t2);  // dB X
  hipLaunchKernelGGL(vl_zmat_kernel, dim3((n_ + 3) / 4), dim3(kT), 0, s_, n_, m_, ldm_, t2, t, V_->dD1_.get(),
                     V_->D_.get());
  HIP_CHECK(hipGetLastError());
  V_->BCol(t2, V_->BvT_.get(), 1., out);
  V_->BCol(t, V_->dBvT1_.get(), 0., t2);
  launch_axpby((size_t)ldm_ * n_, 1., out, 1., t2, out, s_);
}

double VifLaplace::Objective(int lik, const double* mode, const double* upd, double lam, bool first, bool cap,
                             double* trial) {
  FitcSolver& F = *V_->F_;
  const int n = n_, m = m_, ldm = ldm_, nb = nblk(n);
  double* red = red_.get();
  double* t = vec_.get();
  double* mt = mv_.get();
  double* mu = mv_.get() + ldm;
  double* mtmp = mv_.get() + 2 * (size_t)ldm;
  hipLaunchKernelGGL(vl_trial_kernel, dim3(nb), dim3(kT), 0, s_, n, lik, aux_, y_.get(), has_off_ ? off_.get() : nullptr,
                     mode, upd, lam, first ? 1 : 0, cap ? 1 : 0, trial, part_.get());
  launch_sum_blocks(part_.get(), nb, 1, red + 0, s_);
  // m^T R m = |D^-1/2 B m|^2; (C^T m)^T M^-1 (C^T m)
  V_->BVec(trial, V_->Bv_.get(), 1., t);
  hipLaunchKernelGGL(vl_dot_kernel, dim3(nb), dim3(kT), 0, s_, n, t, t, dinv_.get(), part_.get() + 1024);
  launch_sum_blocks(part_.get() + 1024, nb, 1, red + 1, s_);
  V_->Gemv(C_.get(), trial, mt);
  fitc_chol_solve(s_, F.Wi_.get(), F.WiT_.get(), mt, m, ldm, mtmp, mu);
  hipLaunchKernelGGL(vl_mdot_kernel, dim3(1), dim3(kT), 0, s_, m, mt, mu, red + 2);
  HIP_CHECK(hipGetLastError());
  HIP_CHECK(hipMemcpyAsync(h_red_, red, 3 * sizeof(double), hipMemcpyDeviceToHost, s_));
  HIP_CHECK(hipStreamSynchronize(s_));
  return h_red_[0] + loglik_const_ - 0.5 * (h_red_[1] - h_red_[2]);
}

void VifLaplace::Woodbury2(double* logdet_dev) {
  FitcSolver& F = *V_->F_;
  const int n = n_, m = m_, ldm = ldm_;
  const long mm = (long)ldm * ldm;
  // CL = L^-1 P C (n x m), then point-major for the Gram CL^T CL (the split-K GEMM of VifSolver::Prepare)
  chol_->ForwardCols(Cnm_.get(), CL_.get(), m);
  double* CLmn = V_->P0_.get();   // P_0 is free after the residual rows
  ToMN(CL_.get(), CLmn);
  const int chunks = gemm_f64_splitk(s_, m, m, n, CLmn, ldm, 0, CLmn, ldm, 1, F.part_.get(), ldm, mm, 2048,
                                     F.max_chunks_);
  hipLaunchKernelGGL(vl_m2_kernel, dim3((m + 63) / 64, (m + 3) / 4), dim3(kT), 0, s_, F.part_.get(), chunks, mm, m, ldm,
                     M_.get(), M2_.get());
  HIP_CHECK(hipGetLastError());
  HIP_CHECK(hipMemsetAsync(info_.get(), 0, sizeof(int), s_));
  chol_lower(s_, M2_.get(), M2i_.get(), m, ldm, info_.get());
  launch_logdet_chol(s_, M2_.get(), ldm, m, logdet_dev);
  trtri_lower(s_, M2_.get(), M2i_.get(), F.T_.get(), 0, m, ldm);
  fitc_lower_t(s_, M2i_.get(), m, ldm, M2iT_.get());
}

// out = (A - C M^-1 C^T)^-1 r = A^-1 r + A^-1 C M2^-1 C^T A^-1 r (likelihoods.h:2586-2601: two full solves; the
// algebraically equal one-forward-one-backward form y = L^-1 P r, out = P^T L^-T (y + CL M2^-1 CL^T y) halves the
// sweeps but moved the smooth-kernel fixtures' nll by ~3e-9 relative, past the parity bound). x: A^-1 r.
void VifLaplace::SolveSW(const double* r, double* out, double* x) {
  const int m = m_, ldm = ldm_;
  double* t = mv_.get() + 3 * (size_t)ldm;
  double* u = mv_.get() + 4 * (size_t)ldm;
  double* mtmp = mv_.get() + 5 * (size_t)ldm;
  chol_->Solve(r, x);
  V_->Gemv(C_.get(), x, t);
  fitc_chol_solve(s_, M2i_.get(), M2iT_.get(), t, m, ldm, mtmp, u);
  V_->ColDot(C_.get(), u, nullptr, out);
  chol_->Solve(out, out);
  launch_axpby(n_, 1., x, 1., out, out, s_);
}

double VifLaplace::MDot(const double* a, const double* b) {
  hipLaunchKernelGGL(vl_mdot_kernel, dim3(1), dim3(kT), 0, s_, m_, a, b, red_.get() + 63);
  HIP_CHECK(hipGetLastError());
  HIP_CHECK(hipMemcpyAsync(h_red_ + 63, red_.get() + 63, sizeof(double), hipMemcpyDeviceToHost, s_));
  HIP_CHECK(hipStreamSynchronize(s_));
  return h_red_[63];
}

LatentResult VifLaplace::Eval(int cov_type, int lik, const double* trafo, double aux, const IterativeConfig& cfg,
                              bool want_grad, bool want_aux_grad, double* grad_f, ModeStart start) {
  if (!y_set_) Fatal("response variable y has not been set");
  if (lik == kLikGaussian) Fatal("VifLaplace: the Gaussian likelihood uses the exact full-scale Vecchia path");
  aux_ = lik == kLikGamma ? aux : 1.;
  lik_ = lik;
  const bool want_aux = want_aux_grad && want_grad && lik == kLikGamma;
  const bool grad_any = want_grad || grad_f != nullptr;
  FitcSolver& F = *V_->F_;
  const int n = n_, m = m_, ldm = ldm_, nb = nblk(n);
  const double var = trafo[0], phi = trafo[1];
  const double* off = has_off_ ? off_.get() : nullptr;
  const bool cap = lik == kLikPoisson || lik == kLikGamma;   // cap_change_mode_newton_ (likelihoods.h:481-490)
  double* red = red_.get();
  HIP_CHECK(hipEventRecord(ev_[0], s_));
  // phase timing (GPBOOST_AMD_TIMING): events after each phase, summed per label at the end
  static const bool timing = std::getenv("GPBOOST_AMD_TIMING") != nullptr;
  std::vector<std::pair<const char*, hipEvent_t>> marks;
  auto mark = [&](const char* label) {
    if (!timing) return;
    hipEvent_t e;
    HIP_CHECK(hipEventCreate(&e));
    HIP_CHECK(hipEventRecord(e, s_));
    marks.emplace_back(label, e);
  };
  // prior: K, K_mm,s, V, residual factor (+ derivatives), M = K_mm,s + (BK)^T D^-1 (BK) (red[0] log det K_mm,s,
  // red[1] log det M), C = B^T D^-1 B K (the reference's Bt_D_inv_B_cross_cov, re_model_template.h:8839-8855)
  HIP_CHECK(hipMemsetAsync(F.info_.get(), 0, sizeof(int), s_));
  V_->Prepare(cov_type, var, phi, grad_any, red + 48, M_.get());   // red[48] log det K_mm,s, red[49] log det M
  hipLaunchKernelGGL(vl_recip_kernel, dim3((n + kT - 1) / kT), dim3(kT), 0, s_, n, V_->D_.get(), dinv_.get());
  HIP_CHECK(hipGetLastError());
  V_->BCol(F.Kd_.get(), V_->BvT_.get(), 1., C_.get());
  ToNM(C_.get(), Cnm_.get());
  chol_->SetB(V_->Bv_.get(), dinv_.get(), grad_any ? V_->dBv1_.get() : nullptr, grad_any ? V_->dD1_.get() : nullptr);
  mark("prepare");
  auto info_failed = [&](const int* info) {
    int h = 0;
    HIP_CHECK(hipMemcpyAsync(&h, info, sizeof(int), hipMemcpyDeviceToHost, s_));
    HIP_CHECK(hipStreamSynchronize(s_));
    return h != 0;
  };
  if (info_failed(F.info_.get()))
    throw LatentNan("the full-scale Vecchia Woodbury matrix is not positive definite (Cholesky failed)");
  auto factor = [&]() {
    chol_->Factor(w_.get());
    if (chol_->Info() > 0)
      throw LatentNan("NaN or Inf occurred in the mode finding algorithm for the Laplace approximation "
                      "(Sigma^-1 + W not positive definite)");
  };
  LatentResult res;
  // mode start (likelihoods.h:2347-2353)
  if (start == ModeStart::kZero || !evaluated_) {
    HIP_CHECK(hipMemsetAsync(mode_.get(), 0, sizeof(double) * n, s_));
    prev_valid_ = false;
  } else if (start == ModeStart::kWarm) {
    launch_copy(n, mode_.get(), mode_prev_.get(), s_);
    prev_valid_ = true;
  }
  double* x = vec_.get() + (size_t)n;
  double* dir = vec_.get() + 2 * (size_t)n;
  double* t = vec_.get() + 3 * (size_t)n;
  double* logdet_M2 = red + 4;
  double obj = 0.;
  if (start != ModeStart::kKeep || !evaluated_) {
    obj = Objective(lik, mode_.get(), mode_.get(), 1., true, false, trial_.get());
    const int maxit = 1000;                           // maxit_mode_newton_ (likelihoods.h:12721)
    const double delta = cfg.delta_conv_mode_finding;  // :12723
    bool terminate = false, has_nan = false;
    int it = 0;
    for (it = 0; it < maxit; ++it) {
      // W, d1 at the mode; rhs = W mode + d1; A = R + W; M2 (:2561-2601)
      hipLaunchKernelGGL(vl_prep_kernel, dim3(nb), dim3(kT), 0, s_, n, lik, aux_, y_.get(), off, mode_.get(), d1_.get(),
                         w_.get(), static_cast<double*>(nullptr), rhs_.get(), static_cast<double*>(nullptr));
      HIP_CHECK(hipGetLastError());
      mark("newton other");
      factor();
      mark("factor");
      Woodbury2(logdet_M2);
      mark("woodbury (L^-1 P C, m columns)");
      if (info_failed(info_.get())) {
        has_nan = true;
        break;
      }
      SolveSW(rhs_.get(), upd_.get(), x);
      mark("newton solves");
      // Armijo slope (:2603-2611): dir^T (Sigma^-1 + W) dir with Sigma^-1 by the Woodbury form
      launch_axpby(n, 1., upd_.get(), -1., mode_.get(), dir, s_);
      {
        double* mt = mv_.get();
        double* mu = mv_.get() + ldm;
        double* mtmp = mv_.get() + 2 * (size_t)ldm;
        V_->BVec(dir, V_->Bv_.get(), 1., t);
        hipLaunchKernelGGL(vl_dot_kernel, dim3(nb), dim3(kT), 0, s_, n, t, t, dinv_.get(), part_.get());
        launch_sum_blocks(part_.get(), nb, 1, red + 8, s_);
        hipLaunchKernelGGL(vl_dot_kernel, dim3(nb), dim3(kT), 0, s_, n, dir, dir, w_.get(), part_.get() + 1024);
        launch_sum_blocks(part_.get() + 1024, nb, 1, red + 9, s_);
        V_->Gemv(C_.get(), dir, mt);
        fitc_chol_solve(s_, F.Wi_.get(), F.WiT_.get(), mt, m, ldm, mtmp, mu);
        hipLaunchKernelGGL(vl_mdot_kernel, dim3(1), dim3(kT), 0, s_, m, mt, mu, red + 10);
        HIP_CHECK(hipGetLastError());
        HIP_CHECK(hipMemcpyAsync(h_red_ + 8, red + 8, 3 * sizeof(double), hipMemcpyDeviceToHost, s_));
        HIP_CHECK(hipStreamSynchronize(s_));
      }
      const double gdd = h_red_[8] - h_red_[10] + h_red_[9];
      double lam = 1., obj_new = obj;
      for (int ih = 0; ih < 20; ++ih) {   // max_number_lr_shrinkage_steps_newton_ (:12725)
        obj_new = Objective(lik, mode_.get(), upd_.get(), lam, ih == 0, cap, trial_.get());
        if (obj_new < obj + kCArmijo * lam * gdd || std::isnan(obj_new) || std::isinf(obj_new)) lam *= 0.5;
        else break;
      }
      std::swap(mode_, trial_);
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
    if (has_nan) throw LatentNan("NaN or Inf occurred in the mode finding algorithm for the Laplace approximation");
    res.newton_its = it;
    cached_obj_ = obj;
  } else {
    obj = cached_obj_;
  }
  evaluated_ = true;
  // at the mode (:2661-2736): d1, W, dW; A refactored; M2; the log-determinants
  hipLaunchKernelGGL(vl_prep_kernel, dim3(nb), dim3(kT), 0, s_, n, lik, aux_, y_.get(), off, mode_.get(), d1_.get(),
                     w_.get(), dw_.get(), static_cast<double*>(nullptr), part_.get());
  HIP_CHECK(hipGetLastError());
  launch_sum_blocks(part_.get(), nb, 1, red + 6, s_);
  mark("newton other");
  factor();
  mark("factor");
  Woodbury2(logdet_M2);
  mark("woodbury (L^-1 P C, m columns)");
  if (info_failed(info_.get())) throw LatentNan("the full-scale Vecchia Woodbury matrix M2 is not positive definite");
  const double ldA = chol_->LogDet();
  HIP_CHECK(hipMemcpyAsync(h_red_, red, 50 * sizeof(double), hipMemcpyDeviceToHost, s_));
  HIP_CHECK(hipStreamSynchronize(s_));
  const double ld_Ks = h_red_[48], ld_M2 = h_red_[4];
  // sum log D^-1 = -sum log D; D > 0 (CalcCovFactorGradientVecchia :1619-1630, Fatal for non-Gaussian likelihoods)
  double sum_log_dinv = 0.;
  {
    std::vector<double> hD(n);
    HIP_CHECK(hipMemcpyAsync(hD.data(), V_->D_.get(), sizeof(double) * n, hipMemcpyDeviceToHost, s_));
    HIP_CHECK(hipStreamSynchronize(s_));
    if (std::getenv("GPBOOST_AMD_VIFL_DEBUG") != nullptr)
      std::fprintf(stderr, "[vif laplace] D[0..4] %.12g %.12g %.12g %.12g %.12g\n", hD[0], hD[1], hD[2], hD[3], hD[4]);
    for (int i = 0; i < n; ++i) {
      if (!(hD[i] > 0.))
        Fatal("The matrix D in the Vecchia approximation contains negative or zero values. This likely results from "
              "numerical instabilities ");
      sum_log_dinv -= std::log(hD[i]);
    }
  }
  const double logdet = ldA - sum_log_dinv - ld_Ks + ld_M2;   // log |Sigma W + I|
  if (std::getenv("GPBOOST_AMD_VIFL_DEBUG") != nullptr)
    std::fprintf(stderr, "[vif laplace] its %d obj %.12g logdet A %.12g sum log Dinv %.12g logdet Ks %.12g logdet M %.12g "
                 "logdet M2 %.12g\n", res.newton_its, obj, ldA, sum_log_dinv, ld_Ks, h_red_[49], ld_M2);
  res.logdet = logdet;
  res.nll = -(obj - 0.5 * logdet);
  if (!std::isfinite(res.nll)) throw LatentNan("NaN or Inf in the full-scale Vecchia approximate marginal likelihood");
  if (grad_any) {
    if (h_red_[6] > 0.)
      Fatal("CalcGradNegMargLikelihoodLaplaceApproxFSVA: 0's found in the (diagonal) Hessian (or Fisher information) of "
            "the negative log-likelihood. This is not permitted when using the VIF approximation and gradient-based "
            "optimization ");
    const size_t mn = (size_t)ldm * n;
    for (DevBuf<double>* b : {&AiC_, &Y_, &G_, &T1_, &T2_, &T3_})
      if (b->size() < mn) {
        b->alloc(mn);
        HIP_CHECK(hipMemsetAsync(b->get(), 0, sizeof(double) * mn, s_));
      }
    // selected inverse of A: tr(S R), tr(S S'_1), diag(A^-1) (CalcLtLGivenSparsityPattern, :4737-4739)
    double tr_R = 0., tr_Sp1 = 0.;
    mark("gradient other");
    chol_->SelectedInverse(&tr_R, &tr_Sp1, diagS_.get());
    mark("selected inverse");
    // A^-1 C (m columns), M2^-1 (full), Y = M2^-1 (A^-1 C), G = M2^-1 K, CM = M2^-1 C (point-major)
    chol_->SolveMulti(Cnm_.get(), CL_.get(), m);
    mark("A^-1 C (m columns)");
    ToMN(CL_.get(), AiC_.get());
    gemm_f64(s_, m, m, m, 1., M2i_.get(), ldm, 1, M2i_.get(), ldm, 0, 0., M2inv_.get(), ldm, 0, 0, 1, 1);
    double* CM = CL_.get();   // n x m free again: M2^-1 C (point-major)
    gemm_f64(s_, m, n, m, 1., M2inv_.get(), ldm, 0, AiC_.get(), ldm, 0, 0., Y_.get(), ldm);
    gemm_f64(s_, m, n, m, 1., M2inv_.get(), ldm, 0, F.Kmn_.get(), ldm, 0, 0., G_.get(), ldm);
    gemm_f64(s_, m, n, m, 1., M2inv_.get(), ldm, 0, C_.get(), ldm, 0, 0., CM, ldm);
    // the reference's covariance gradient evaluates the location-dependent terms at mode + F in data order
    // (SetGradOffset); the F-gradient (CalcGradFLaplace) at the model-order offsets
    static const bool consistent = std::getenv("GPBOOST_AMD_VIF_OFFSET_CONSISTENT") != nullptr;
    const bool ref_order = has_goff_ && has_off_ && grad_f == nullptr && !consistent;
    const double* loc_off = ref_order ? goff_.get() : off;
    const double* d1_aux = d1_.get();
    const double* w_aux = w_.get();
    if (ref_order) {
      hipLaunchKernelGGL(vl_prep_kernel, dim3(nb), dim3(kT), 0, s_, n, lik, aux_, y_.get(), goff_.get(), mode_.get(),
                         gd1_.get(), gw_.get(), dw_.get(), static_cast<double*>(nullptr), static_cast<double*>(nullptr));
      HIP_CHECK(hipGetLastError());
      d1_aux = gd1_.get();
      w_aux = gw_.get();
    }
    // d_mll_d_mode = 1/2 diag((Sigma^-1 + W)^-1) dW, diag = diag A^-1 + (A^-1 C)_i . Y_i (:4740-4744);
    // v = (Sigma^-1 + W)^-1 d_mll (the reference's :4746-4753 form, same matrix)
    double* cd = vec_.get() + 4 * (size_t)n;
    double* full = vec_.get() + 5 * (size_t)n;
    V_->ColDot(AiC_.get(), nullptr, Y_.get(), cd);
    hipLaunchKernelGGL(vl_dmll_kernel, dim3((n + kT - 1) / kT), dim3(kT), 0, s_, n, diagS_.get(), cd, dw_.get(), full,
                       dmll_.get());
    HIP_CHECK(hipGetLastError());
    SolveSW(dmll_.get(), vS_.get(), x);
    if (want_grad) {
      // m x m traces: t[0] tr(Ks^-1 Kmm), t[1] tr(M2^-1 Kmm), t[2] tr(Ks^-1 dKmm), t[3] tr(M2^-1 dKmm)
      double* a6 = mv_.get() + 6 * (size_t)ldm;   // (fitc_mm_terms' quadratic forms are not used here)
      fitc_mm_terms(s_, F.Kinv_.get(), M2inv_.get(), F.Kmm_.get(), F.dKmm_.get(), a6, m, ldm, F.part_.get(), red + 16);
      // Frobenius products <X, Y> over the point-major sets -> red slots
      double* cdot = vec_.get() + 6 * (size_t)n;
      auto frob = [&](const double* X, const double* Y, int slot) {
        V_->ColDot(X, nullptr, Y, cdot);
        hipLaunchKernelGGL(vl_dot_kernel, dim3(nb), dim3(kT), 0, s_, n, cdot, static_cast<const double*>(nullptr),
                           static_cast<const double*>(nullptr), part_.get() + 2048);
        launch_sum_blocks(part_.get() + 2048, nb, 1, red + slot, s_);
        HIP_CHECK(hipGetLastError());
      };
      auto vdot = [&](const double* a, const double* b, const double* c, int slot) {
        hipLaunchKernelGGL(vl_dot_kernel, dim3(nb), dim3(kT), 0, s_, n, a, b, c, part_.get() + 3072);
        launch_sum_blocks(part_.get() + 3072, nb, 1, red + slot, s_);
        HIP_CHECK(hipGetLastError());
      };
      // sum D^-1 dD_k (:4790)
      vdot(dinv_.get(), V_->dD0_.get(), nullptr, 22);
      vdot(dinv_.get(), V_->dD1_.get(), nullptr, 23);
      // k = 0: S' = -R, dK = K (re_comps_cross_cov GetZSigmaZtGrad(0)), dK_mm = K_mm
      RMat(AiC_.get(), T1_.get(), T2_.get());     // R A^-1 C
      frob(G_.get(), C_.get(), 24);                // <M2^-1 K, C>          (K^T S' K = -K^T C)
      frob(CM, F.Kmn_.get(), 25);                  // <M2^-1 C, K>
      frob(Y_.get(), T1_.get(), 26);               // <Y, R A^-1 C>
      // k = 1: S'_1, dK = dK_mn / dlog phi
      SpMat(F.Kmn_.get(), T1_.get(), T2_.get(), T3_.get());   // S'_1 K
      frob(G_.get(), T1_.get(), 27);               // <M2^-1 K, S'_1 K>
      frob(Y_.get(), T1_.get(), 28);               // <Y, S'_1 K>
      frob(CM, V_->dK_.get(), 29);                 // <M2^-1 C, dK>
      RMat(V_->dK_.get(), T1_.get(), T2_.get());   // R dK
      frob(Y_.get(), T1_.get(), 30);               // <Y, R dK>
      SpMat(AiC_.get(), T1_.get(), T2_.get(), T3_.get());     // S'_1 A^-1 C
      frob(Y_.get(), T1_.get(), 31);               // <Y, S'_1 A^-1 C>
      // dSigma^-1 m (the reference's SigmaI_deriv_mode, :4775-4783) and its products with m and v
      double* q = vec_.get() + 7 * (size_t)n;
      double* rm = vec_.get() + 8 * (size_t)n;
      double* s1 = vec_.get() + 9 * (size_t)n;
      double* s2 = vec_.get() + 10 * (size_t)n;
      double* s3 = vec_.get() + 11 * (size_t)n;
      double* c2 = vec_.get() + 12 * (size_t)n;
      double* c3 = vec_.get() + 13 * (size_t)n;
      double* mv = mv_.get();
      double* a1 = mv + 6 * (size_t)ldm;
      double* b1 = mv + 7 * (size_t)ldm;
      double* b2 = mv + 8 * (size_t)ldm;
      double* a4 = mv + 9 * (size_t)ldm;
      double* b4 = mv + 10 * (size_t)ldm;
      double* e = mv + 11 * (size_t)ldm;
      double* e2 = mv + 12 * (size_t)ldm;
      double* b5 = mv + 13 * (size_t)ldm;
      double* mtmp = mv + 14 * (size_t)ldm;
      const double* mode = mode_.get();
      RVec(mode, rm, t);                                                     // R m
      V_->Gemv(F.Kmn_.get(), rm, a1);                                        // K^T R m
      fitc_chol_solve(s_, F.Wi_.get(), F.WiT_.get(), a1, m, ldm, mtmp, b2);  // b2 = M^-1 K^T R m
      V_->ColDot(F.Kmn_.get(), b2, nullptr, c2);                             // c2 = K b2
      for (int k = 0; k < 2; ++k) {
        const double* dK = k == 0 ? F.Kmn_.get() : V_->dK_.get();
        const double* dKmm = k == 0 ? F.Kmm_.get() : F.dKmm_.get();
        auto sp = [&](const double* xx, double* out) {   // S'_k x
          if (k == 0) {
            RVec(xx, out, t);
            launch_axpby(n, -1., out, 0., out, out, s_);
          } else {
            SpVec(xx, out, t, x);
          }
        };
        sp(mode, q);                                                          // q = S' m
        // term1: R K M^-1 K^T S' m
        V_->Gemv(F.Kmn_.get(), q, a1);
        fitc_chol_solve(s_, F.Wi_.get(), F.WiT_.get(), a1, m, ldm, mtmp, b1);
        V_->ColDot(F.Kmn_.get(), b1, nullptr, s1);
        RVec(s1, s2, t);
        launch_axpby(n, -1., s2, 1., q, q, s_);
        // term2: S' K M^-1 K^T R m = S' c2
        sp(c2, s2);
        launch_axpby(n, -1., s2, 1., q, q, s_);
        // term3: R dK M^-1 K^T R m
        V_->ColDot(dK, b2, nullptr, c3);
        RVec(c3, s3, t);
        launch_axpby(n, -1., s3, 1., q, q, s_);
        // term4: R K M^-1 dK^T R m
        V_->Gemv(dK, rm, a4);
        fitc_chol_solve(s_, F.Wi_.get(), F.WiT_.get(), a4, m, ldm, mtmp, b4);
        V_->ColDot(F.Kmn_.get(), b4, nullptr, s1);
        RVec(s1, s3, t);
        launch_axpby(n, -1., s3, 1., q, q, s_);
        // term5: R K M^-1 dM M^-1 K^T R m, dM b2 = dK_mm b2 + K^T S' K b2 + C^T dK b2 + dK^T C b2
        fitc_symv(s_, dKmm, b2, m, ldm, e);
        V_->Gemv(F.Kmn_.get(), s2, e2);    // s2 = S' c2 = S' K b2
        launch_axpby(m, 1., e2, 1., e, e, s_);
        V_->Gemv(C_.get(), c3, e2);        // c3 = dK b2
        launch_axpby(m, 1., e2, 1., e, e, s_);
        V_->ColDot(C_.get(), b2, nullptr, s1);   // C b2
        V_->Gemv(dK, s1, e2);
        launch_axpby(m, 1., e2, 1., e, e, s_);
        fitc_chol_solve(s_, F.Wi_.get(), F.WiT_.get(), e, m, ldm, mtmp, b5);
        V_->ColDot(F.Kmn_.get(), b5, nullptr, s1);
        RVec(s1, s3, t);
        launch_axpby(n, 1., s3, 1., q, q, s_);
        vdot(mode, q, nullptr, 32 + 2 * k);      // m^T dSigma^-1 m
        vdot(vS_.get(), q, nullptr, 33 + 2 * k); // v^T dSigma^-1 m
      }
      HIP_CHECK(hipMemcpyAsync(h_red_, red, 40 * sizeof(double), hipMemcpyDeviceToHost, s_));
      HIP_CHECK(hipStreamSynchronize(s_));
      const double* mt = h_red_ + 16;   // [tr Ks^-1 Kmm, tr M2^-1 Kmm, tr Ks^-1 dKmm, tr M2^-1 dKmm, ., .]
      const double* g = h_red_;
      // variance: 1/2 (m^T dSI m - tr(S R)) + 1/2 sum D^-1 dD_0 - 1/2 tr(Ks^-1 Kmm)
      //           + 1/2 [tr(M2^-1 Kmm) - <G, C> + 2 <CM, K> - <Y, R A^-1 C>] - v^T dSI m
      const double tr0 = mt[1] - g[24] + 2. * g[25] - g[26];
      const double g0 = 0.5 * (g[32] - tr_R) + 0.5 * g[22] - 0.5 * mt[0] + 0.5 * tr0 - g[33];
      // range: tr(M2^-1 dM2) = tr(M2^-1 dKmm) + <G, S'K> + 2 <CM, dK> - 2 <Y, R dK> - 2 <Y, S'K> + <Y, S' A^-1 C>
      const double tr1 = mt[3] + g[27] + 2. * g[29] - 2. * g[30] - 2. * g[28] + g[31];
      const double g1 = 0.5 * (g[34] + tr_Sp1) + 0.5 * g[23] - 0.5 * mt[2] + 0.5 * tr1 - g[35];
      res.grad = {g0, g1};
    }
    if (grad_f != nullptr) {   // wrt the fixed effects F (:4885-4893)
      hipLaunchKernelGGL(vl_gradf_kernel, dim3((n + kT - 1) / kT), dim3(kT), 0, s_, n, d1_.get(), dmll_.get(), w_.get(),
                         vS_.get(), t);
      HIP_CHECK(hipGetLastError());
      HIP_CHECK(hipMemcpyAsync(grad_f, t, sizeof(double) * n, hipMemcpyDeviceToHost, s_));
      HIP_CHECK(hipStreamSynchronize(s_));
    }
    if (want_aux) {   // gamma shape on the log scale (:4896-4922; diag(A^-1) counted twice, see the oracle)
      hipLaunchKernelGGL(vl_gamma_kernel, dim3(nb), dim3(kT), 0, s_, n, y_.get(), loc_off, mode_.get(), w_aux, full,
                         diagS_.get(), d1_aux, vS_.get(), part_.get());
      HIP_CHECK(hipGetLastError());
      launch_sum_blocks(part_.get(), nb, 3, red + 40, s_);
      HIP_CHECK(hipMemcpyAsync(h_red_ + 40, red + 40, 3 * sizeof(double), hipMemcpyDeviceToHost, s_));
      HIP_CHECK(hipStreamSynchronize(s_));
      const double a = aux_;
      const double neg = a * (h_red_[40] - n * (std::log(a) + 1. - digamma_asa103(a)) - sum_log_y_);
      res.grad.push_back(neg + 0.5 * h_red_[41] + h_red_[42]);
    }
  }
  mark("gradient other");
  HIP_CHECK(hipEventRecord(ev_[1], s_));
  HIP_CHECK(hipEventSynchronize(ev_[1]));
  float ms = 0.f;
  HIP_CHECK(hipEventElapsedTime(&ms, ev_[0], ev_[1]));
  res.ms_total = ms;
  if (timing) {
    std::fprintf(stderr, "[vif laplace] %.2f ms: %d Newton steps (last factorization %.2f ms)\n", ms, res.newton_its,
                 chol_->last_factor_ms());
    std::vector<std::pair<std::string, double>> sums;
    hipEvent_t prev = ev_[0];
    for (auto& mk : marks) {
      float d = 0.f;
      HIP_CHECK(hipEventElapsedTime(&d, prev, mk.second));
      auto it = std::find_if(sums.begin(), sums.end(), [&](const auto& q) { return q.first == mk.first; });
      if (it == sums.end()) sums.emplace_back(mk.first, d);
      else it->second += d;
      prev = mk.second;
    }
    for (auto& q : sums) std::fprintf(stderr, "    %-34s %8.2f ms\n", q.first.c_str(), q.second);
    for (auto& mk : marks) HIP_CHECK(hipEventDestroy(mk.second));
  }
  return res;
}


// PredictLaplaceApproxFSVA, Cholesky branch (likelihoods.h:6060-6130, 6478-6548), at the mode of the last Eval:
//   s = mode - K M^-1 C^T mode (sigma_inv_mode), mean = -Bpo s [Bp^-1] + K_pm K_mm,s^-1 C^T s
//   SRW = A^-1 (W K), Mw2 = K_mm,s + C^T SRW, Sig = K_mm,s^-1 K_mp, X1 = M_aux_1^T = (C^T SRW)^T Sig,
//   X2 = Mw2^-1 X1, X3 = M_aux_3^T = SRW^T Bpo^T [Bp^-T], X4 = Mw2^-1 X3, Maux = L_A^-1 P Bpo^T [Bp^-T]
//   var = Dp [diag Bp^-1 Dp Bp^-T] + |Maux_p|^2 + |Vp_p|^2 - Sig.X1 + X2.X1 + 2 Sig.X3 - 2 X2.X3 + X4.X3
//   cov = [Dp | Bp^-1 Dp Bp^-T] + Maux^T Maux + Vp^T Vp - X1^T Sig + X1^T X2 + X3^T Sig + Sig^T X3 - X3^T X2
//         - X2^T X3 + X3^T X4
void VifLaplace::Predict(int cov_type, double var, double phi, const double* Xp, int np, const int* nbr, int mp,
                         bool cond_all, double* mean, double* pvar, double* pcov) {
  if (np <= 0) return;
  if (!evaluated_) Fatal("VifLaplace::Predict: no mode (evaluate the model at the parameters first)");
  if (cond_all && (pcov != nullptr || pvar != nullptr) && np > 20000)
    Fatal("latent_order_obs_first_cond_all with predictive (co)variances is limited to num_data_pred <= 20000 in "
          "gpboost_amd");
  FitcSolver& F = *V_->F_;
  const int n = n_, m = m_, ldm = ldm_;
  const long mm = (long)ldm * ldm;
  DevBuf<double> KP, Va, Bvp, Dp;
  DevBuf<int> dnb;
  V_->PredRows(cov_type, var, phi, Xp, np, nbr, mp, KP, Va, Bvp, Dp, dnb);
  double* sv = vec_.get();
  double* ku = vec_.get() + (size_t)n;
  double* mt = mv_.get();
  double* mu = mv_.get() + ldm;
  double* mtmp = mv_.get() + 2 * (size_t)ldm;
  double* u2 = mv_.get() + 3 * (size_t)ldm;
  // sigma_inv_mode (:6107)
  V_->Gemv(C_.get(), mode_.get(), mt);
  fitc_chol_solve(s_, F.Wi_.get(), F.WiT_.get(), mt, m, ldm, mtmp, mu);
  V_->ColDot(F.Kmn_.get(), mu, nullptr, ku);
  launch_axpby(n, 1., mode_.get(), -1., ku, sv, s_);
  // mean (:6108-6115)
  DevBuf<double> mo(np), kpw(np), Qscr((size_t)ldm * np);
  V_->PredBpo(np, mp, dnb.get(), Bvp.get(), sv, F.Kmn_.get(), mo.get(), Qscr.get());
  V_->Gemv(C_.get(), sv, mt);
  fitc_symv(s_, F.Kinv_.get(), mt, m, ldm, u2);
  V_->ColDotN(KP.get(), u2, nullptr, np, kpw.get());
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
  std::vector<double> mu_h(np);
  for (int p = 0; p < np; ++p) mu_h[p] = -hmo[p];
  if (cond_all) bp_solve(mu_h.data(), 1, 1);
  for (int p = 0; p < np; ++p) mean[p] = mu_h[p] + hkpw[p];
  if (pvar == nullptr && pcov == nullptr) return;
  std::vector<double> Binv;
  if (cond_all) {
    Binv.assign((size_t)np * np, 0.);   // row-major: row p = e_p^T Bp^-1
    for (int p = 0; p < np; ++p) Binv[(size_t)p * np + p] = 1.;
    bp_solve(Binv.data(), np, np);
  }
  const size_t mnp = (size_t)ldm * np, mn = (size_t)ldm * n;
  const double* Vp = Va.get() + (size_t)ldm * n;
  DevBuf<double> Sig(mnp), X1(mnp), X2(mnp), X3(mnp), X4(mnp), CS(mm), mo2(np);
  for (DevBuf<double>* b : {&Sig, &X1, &X2, &X3, &X4}) HIP_CHECK(hipMemsetAsync(b->get(), 0, sizeof(double) * mnp, s_));
  gemm_f64(s_, m, np, m, 1., F.Kinv_.get(), ldm, 0, KP.get(), ldm, 0, 0., Sig.get(), ldm);
  // SRW = A^-1 (W o K) (sigma_resid_plus_W_inv_cross_cov, :6480), point-major in T2_
  for (DevBuf<double>* b : {&T1_, &T2_})
    if (b->size() < mn) {
      b->alloc(mn);
      HIP_CHECK(hipMemsetAsync(b->get(), 0, sizeof(double) * mn, s_));
    }
  hipLaunchKernelGGL(vl_colscale_kernel, dim3((n + 3) / 4), dim3(kT), 0, s_, n, m, ldm, F.Kmn_.get(), w_.get(), T1_.get());
  HIP_CHECK(hipGetLastError());
  ToNM(T1_.get(), CL_.get());
  chol_->SolveMulti(CL_.get(), CL_.get(), m);
  double* SRW = T2_.get();
  ToMN(CL_.get(), SRW);
  // CS = C^T SRW; Mw2 = K_mm,s + CS (sigma_woodbury_2, :6481-6483): factor and inverse in M2_ / M2i_ / M2inv_
  const int chunks = gemm_f64_splitk(s_, m, m, n, C_.get(), ldm, 0, SRW, ldm, 1, F.part_.get(), ldm, mm, 2048,
                                     F.max_chunks_);
  hipLaunchKernelGGL(vl_psum_kernel, dim3((m + 63) / 64, (m + 3) / 4), dim3(kT), 0, s_, F.part_.get(), chunks, mm, m, ldm,
                     static_cast<const double*>(nullptr), CS.get());
  hipLaunchKernelGGL(vl_psum_kernel, dim3((m + 63) / 64, (m + 3) / 4), dim3(kT), 0, s_, F.part_.get(), chunks, mm, m, ldm,
                     F.Ks_.get(), M2_.get());
  HIP_CHECK(hipGetLastError());
  HIP_CHECK(hipMemsetAsync(info_.get(), 0, sizeof(int), s_));
  chol_lower(s_, M2_.get(), M2i_.get(), m, ldm, info_.get());
  trtri_lower(s_, M2_.get(), M2i_.get(), F.T_.get(), 0, m, ldm);
  gemm_f64(s_, m, m, m, 1., M2i_.get(), ldm, 1, M2i_.get(), ldm, 0, 0., M2inv_.get(), ldm, 0, 0, 1, 1);
  // X1 = CS^T Sig, X2 = Mw2^-1 X1, X3 = SRW^T Bpo^T [Bp^-T] (columns of M_aux_3^T), X4 = Mw2^-1 X3
  gemm_f64(s_, m, np, m, 1., CS.get(), ldm, 1, Sig.get(), ldm, 0, 0., X1.get(), ldm);
  gemm_f64(s_, m, np, m, 1., M2inv_.get(), ldm, 0, X1.get(), ldm, 0, 0., X2.get(), ldm);
  V_->PredBpo(np, mp, dnb.get(), Bvp.get(), sv, SRW, mo2.get(), X3.get());
  if (cond_all) {
    std::vector<double> hQ(mnp);
    HIP_CHECK(hipMemcpyAsync(hQ.data(), X3.get(), sizeof(double) * mnp, hipMemcpyDeviceToHost, s_));
    HIP_CHECK(hipStreamSynchronize(s_));
    bp_solve(hQ.data(), ldm, m);
    HIP_CHECK(hipMemcpyAsync(X3.get(), hQ.data(), sizeof(double) * mnp, hipMemcpyHostToDevice, s_));
  }
  gemm_f64(s_, m, np, m, 1., M2inv_.get(), ldm, 0, X3.get(), ldm, 0, 0., X4.get(), ldm);
  int info = 0;
  HIP_CHECK(hipMemcpyAsync(&info, info_.get(), sizeof(int), hipMemcpyDeviceToHost, s_));
  HIP_CHECK(hipStreamSynchronize(s_));
  if (info != 0) Fatal("full_scale_vecchia prediction: the Woodbury matrix K_mm + C^T (Sigma_resid^-1 + W)^-1 W K is not "
                       "positive definite");
  // Maux = L_A^-1 P Bpo^T [Bp^-T] (n x np columns; :6492-6505): Bpo^T over the observed neighbours
  std::vector<int> nb_obs((size_t)np * mp);
  for (size_t e = 0; e < nb_obs.size(); ++e) nb_obs[e] = nbr[e] >= 0 && nbr[e] < n ? nbr[e] : -1;
  DevBuf<int> dnbo(nb_obs.size());
  HIP_CHECK(hipMemcpyAsync(dnbo.get(), nb_obs.data(), sizeof(int) * nb_obs.size(), hipMemcpyHostToDevice, s_));
  DevBuf<double> dvar(np);
  const bool all_at_once = cond_all || pcov != nullptr;
  const int chunk = all_at_once ? np : std::max(1, std::min(np, 256));
  DevBuf<double> cols((size_t)n * chunk), Maux((size_t)n * chunk);
  DevBuf<double> dcov;
  if (pcov != nullptr) {
    dcov.alloc((size_t)np * np);
    HIP_CHECK(hipMemsetAsync(dcov.get(), 0, sizeof(double) * dcov.size(), s_));
  }
  DevBuf<double> dX;
  if (cond_all) {   // the row-major Bp^-1 read column-major is X = Bp^-T
    dX.alloc((size_t)np * np);
    HIP_CHECK(hipMemcpyAsync(dX.get(), Binv.data(), sizeof(double) * Binv.size(), hipMemcpyHostToDevice, s_));
  }
  for (int p0 = 0; p0 < np; p0 += chunk) {
    const int c = std::min(chunk, np - p0);
    launch_chol_pred_cols(n, c, mp, dnbo.get() + (size_t)p0 * mp, Bvp.get() + (size_t)p0 * mp, cols.get(), s_);
    if (cond_all) {
      gemm_f64(s_, n, np, np, 1., cols.get(), n, 0, dX.get(), np, 0, 0., Maux.get(), n);
      HIP_CHECK(hipMemcpyAsync(cols.get(), Maux.get(), sizeof(double) * (size_t)n * np, hipMemcpyDeviceToDevice, s_));
    }
    chol_->ForwardCols(cols.get(), Maux.get(), c);
    hipLaunchKernelGGL(vl_colsq_kernel, dim3(c), dim3(kT), 0, s_, n, Maux.get(), dvar.get() + p0);
    HIP_CHECK(hipGetLastError());
    if (pcov != nullptr) gemm_f64(s_, np, np, n, 1., Maux.get(), n, 1, Maux.get(), n, 0, 0., dcov.get(), np);
  }
  if (pvar != nullptr) {
    DevBuf<double> dv2(np);
    hipLaunchKernelGGL(vl_pvar_kernel, dim3((np + 3) / 4), dim3(kT), 0, s_, np, m, ldm, Vp, Sig.get(), X1.get(), X2.get(),
                       X3.get(), X4.get(), dv2.get());
    HIP_CHECK(hipGetLastError());
    launch_axpby(np, 1., dv2.get(), 1., dvar.get(), dvar.get(), s_);
    HIP_CHECK(hipMemcpyAsync(pvar, dvar.get(), sizeof(double) * np, hipMemcpyDeviceToHost, s_));
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
    double* C = dcov.get();
    gemm_f64(s_, np, np, m, 1., Vp, ldm, 1, Vp, ldm, 0, 1., C, np);
    gemm_f64(s_, np, np, m, -1., X1.get(), ldm, 1, Sig.get(), ldm, 0, 1., C, np);
    gemm_f64(s_, np, np, m, 1., X1.get(), ldm, 1, X2.get(), ldm, 0, 1., C, np);
    gemm_f64(s_, np, np, m, 1., X3.get(), ldm, 1, Sig.get(), ldm, 0, 1., C, np);
    gemm_f64(s_, np, np, m, 1., Sig.get(), ldm, 1, X3.get(), ldm, 0, 1., C, np);
    gemm_f64(s_, np, np, m, -1., X3.get(), ldm, 1, X2.get(), ldm, 0, 1., C, np);
    gemm_f64(s_, np, np, m, -1., X2.get(), ldm, 1, X3.get(), ldm, 0, 1., C, np);
    gemm_f64(s_, np, np, m, 1., X3.get(), ldm, 1, X4.get(), ldm, 0, 1., C, np);
    if (cond_all) {   // + Bp^-1 Dp Bp^-T = (D X)^T X with X = Bp^-T
      std::vector<double> XD(Binv);
      for (int p = 0; p < np; ++p)
        for (int k = 0; k < np; ++k) XD[(size_t)p * np + k] *= hD[k];
      DevBuf<double> dXD((size_t)np * np);
      HIP_CHECK(hipMemcpyAsync(dXD.get(), XD.data(), sizeof(double) * XD.size(), hipMemcpyHostToDevice, s_));
      gemm_f64(s_, np, np, np, 1., dXD.get(), np, 1, dX.get(), np, 0, 1., C, np);
      HIP_CHECK(hipMemcpyAsync(pcov, C, sizeof(double) * (size_t)np * np, hipMemcpyDeviceToHost, s_));
      HIP_CHECK(hipStreamSynchronize(s_));
    } else {
      HIP_CHECK(hipMemcpyAsync(pcov, C, sizeof(double) * (size_t)np * np, hipMemcpyDeviceToHost, s_));
      HIP_CHECK(hipStreamSynchronize(s_));
      for (int p = 0; p < np; ++p) pcov[(size_t)p * np + p] += hD[p];
    }
  }
}

}  // namespace gpb_amd
