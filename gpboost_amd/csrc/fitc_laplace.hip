// Laplace approximation with the FITC approximation (fitc_laplace.h gives the model and the
// reference lines). Per Newton step (n observations, m inducing points, K = K_mn column-major, ld ldm):
//   d1, W, DW = (W d + 1)^-1, rhs = W mode + d1          one thread per observation
//   M = K_mm,s + K diag(W DW) K^T                        split-K MFMA Gram (2 m^2 n) + POTRF / TRTRI
//   Sigma rhs, K^T M^-1 K (W DW Sigma rhs), Sigma a      five matrix-vector passes over K
//   Armijo line search on -1/2 a^T mode + sum log p(y | mode + F)
// and for the gradient A = K_mm,s^-1 K, G = M^-1 K, dK_mm A (three MFMA GEMMs) and three fused passes
// per observation (the range derivative of K recomputed from the coordinates).
// Solves with K_mm,s and M apply the inverse Cholesky factor twice (L^-T (L^-1 x), fitc_chol_solve) rather
// than an explicit inverse: Poisson / probit information makes M ill-conditioned enough (cond ~1e6..1e12)
// that S^-1 x formed with the explicit S^-1 moves the Newton fixed point by ~cond(S) eps (measured 1e-7
// relative in the nll against the reference's Cholesky solves; 1e-11 with the factor form).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <limits>

#include "cov.h"
#include "dense.h"
#include "fitc_laplace.h"
#include "kernels.h"
#include "lik_device.h"

namespace gpb_amd {
namespace {

constexpr int kT = 256;
constexpr int kChunk = 64;                  // observations per gemv partial
constexpr double kJitterMult = 1. + 1e-6;   // JITTER_MULT_IP_FITC_FSA (utils.h:39)
enum { kMv = 18 };                          // m-vector slots in mv_

struct Vec4 {
  const double* p[4];
};
struct OutVec4 {
  double* p[4];
};

__device__ __forceinline__ double wsum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// fixed-order sum of the 4 waves' (wave-uniform) values of a 256-thread block
__device__ __forceinline__ double block4(double v, double* red) {
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  const double s = (red[0] + red[1]) + (red[2] + red[3]);
  __syncthreads();
  return s;
}

// fixed-order sum over the 256 threads of a block (per-thread values), written by thread 0
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

// d_i = sigma1^2 jitter - |V[:, i]|^2 (re_model_template.h:7358-7377, no nugget); one wave per observation
__global__ void __launch_bounds__(kT) fl_diag_kernel(const double* __restrict__ V, int n, int m, int ldm, double dvar,
                                                    double* __restrict__ dvec) {
  const int lane = threadIdx.x & 63;
  const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (i >= n) return;
  double s = 0.;
  for (int j = lane; j < m; j += 64) {
    const double v = V[(size_t)j + (size_t)i * ldm];
    s += v * v;
  }
  s = wsum(s);
  if (lane == 0) dvec[i] = dvar - s;
}

// Newton step quantities (likelihoods.h:3130-3150): d1, W (when w_update), DW = (W d + 1)^-1,
// wdw = sqrt(W)^2 DW, rhs = W mode + d1
__global__ void __launch_bounds__(kT) fl_prep_kernel(int n, int lik, double aux, const double* __restrict__ y,
                                                    const double* __restrict__ off, const double* __restrict__ mode,
                                                    const double* __restrict__ dvec, int w_update,
                                                    double* __restrict__ d1, double* __restrict__ w,
                                                    double* __restrict__ wdw, double* __restrict__ DW,
                                                    double* __restrict__ rhs) {
  const int i = blockIdx.x * kT + threadIdx.x;
  if (i >= n) return;
  const double mi = mode[i];
  const double l = off ? mi + off[i] : mi;
  const double g = lik_d1(lik, aux, y[i], l);
  d1[i] = g;
  double wi;
  if (w_update) {
    wi = lik_info(lik, aux, y[i], l);
    w[i] = wi;
  } else {
    wi = w[i];
  }
  const double dw = 1. / (wi * dvec[i] + 1.);
  const double ws = sqrt(wi);
  DW[i] = dw;
  wdw[i] = ws * ws * dw;
  if (rhs) rhs[i] = wi * mi + g;
}

// Kd[j + i ldm] = K[j + i ldm] s_i (j < m)
__global__ void __launch_bounds__(kT) fl_colscale_kernel(const double* __restrict__ K, const double* __restrict__ s,
                                                        int n, int m, int ldm, double* __restrict__ Kd) {
  const int j = blockIdx.x * 64 + (threadIdx.x & 63);
  const int i = blockIdx.y * 4 + (threadIdx.x >> 6);
  if (i >= n || j >= m) return;
  const size_t e = (size_t)j + (size_t)i * ldm;
  Kd[e] = K[e] * s[i];
}

// part[(b NV + v) ldm + j] = sum_{i in chunk b} M[j, i] x_v[i]
template <int NV>
__global__ void __launch_bounds__(kT) fl_gemv_part_kernel(const double* __restrict__ M, Vec4 x, int n, int m, int ldm,
                                                         double* __restrict__ part) {
  const int i0 = blockIdx.x * kChunk, i1 = min(n, i0 + kChunk);
  for (int j = threadIdx.x; j < m; j += kT) {
    double acc[NV];
#pragma unroll
    for (int v = 0; v < NV; ++v) acc[v] = 0.;
    for (int i = i0; i < i1; ++i) {
      const double mj = M[(size_t)j + (size_t)i * ldm];
#pragma unroll
      for (int v = 0; v < NV; ++v) acc[v] += mj * x.p[v][i];
    }
#pragma unroll
    for (int v = 0; v < NV; ++v) part[((size_t)blockIdx.x * NV + v) * ldm + j] = acc[v];
  }
}

// out_v[j] = sum_b part[(b NV + v) ldm + j]: one wave per (v, j), lane-strided, fixed-order wave sum
__global__ void __launch_bounds__(kT) fl_gemv_reduce_kernel(const double* __restrict__ part, int nb, int nv, int m,
                                                           int ldm, OutVec4 out) {
  const int lane = threadIdx.x & 63;
  const int q = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (q >= nv * m) return;
  const int v = q / m, j = q - v * m;
  double s = 0.;
  for (int b = lane; b < nb; b += 64) s += part[((size_t)b * nv + v) * ldm + j];
  s = wsum(s);
  if (lane == 0) out.p[v][j] = s;
}

// c_i = sum_j M[j, i] v_j (v = nullptr: sum_j M[j, i]^2; and c2 with v2); one wave per observation
__global__ void __launch_bounds__(kT) fl_coldot_kernel(const double* __restrict__ M, const double* __restrict__ v,
                                                      const double* __restrict__ v2, int n, int m, int ldm,
                                                      double* __restrict__ c, double* __restrict__ c2) {
  const int lane = threadIdx.x & 63;
  const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (i >= n) return;
  double s = 0., s2 = 0.;
  for (int j = lane; j < m; j += 64) {
    const double x = M[(size_t)j + (size_t)i * ldm];
    s += v ? x * v[j] : x * x;
    if (v2) s2 += x * v2[j];
  }
  s = wsum(s);
  if (v2) s2 = wsum(s2);
  if (lane == 0) {
    c[i] = s;
    if (v2) c2[i] = s2;
  }
}

// out_i = c_i + d_i x_i (Sigma x); z_i = s_i out_i (nullable)
__global__ void __launch_bounds__(kT) fl_sigma_kernel(int n, const double* __restrict__ c, const double* __restrict__ d,
                                                     const double* __restrict__ x, const double* __restrict__ s,
                                                     double* __restrict__ out, double* __restrict__ z) {
  const int i = blockIdx.x * kT + threadIdx.x;
  if (i >= n) return;
  const double o = c[i] + d[i] * x[i];
  out[i] = o;
  if (z) z[i] = s[i] * o;
}

// SigmaI_mode_update = rhs - sqrt(W) DW (sqrt(W) Sigma rhs - sqrt(W) K^T M^-1 K (...)) (likelihoods.h:3158-3162)
__global__ void __launch_bounds__(kT) fl_aupd_kernel(int n, const double* __restrict__ rhs, const double* __restrict__ w,
                                                    const double* __restrict__ DW, const double* __restrict__ sig,
                                                    const double* __restrict__ kv, double* __restrict__ aupd) {
  const int i = blockIdx.x * kT + threadIdx.x;
  if (i >= n) return;
  const double ws = sqrt(w[i]);
  double t = DW[i] * (sig[i] * ws - ws * kv[i]);
  t *= ws;
  aupd[i] = rhs[i] + (-t);
}

// Armijo slope: sum_i dir_i (aupd_i - a_i + W_i dir_i), dir = mupd - mode (likelihoods.h:3166-3169)
__global__ void __launch_bounds__(kT) fl_gdd_kernel(int n, const double* __restrict__ mode,
                                                   const double* __restrict__ a, const double* __restrict__ mupd,
                                                   const double* __restrict__ aupd, const double* __restrict__ w,
                                                   double* __restrict__ part) {
  __shared__ double red[kT];
  double acc = 0.;
  for (int i = blockIdx.x * kT + threadIdx.x; i < n; i += gridDim.x * kT) {
    const double dir = mupd[i] - mode[i];
    acc += dir * (aupd[i] - a[i] + w[i] * dir);
  }
  const double s = block_sum(acc, red);
  if (threadIdx.x == 0) part[blockIdx.x] = s;
}

// one line-search trial (likelihoods.h:3171-3190): the new state mixed at learning rate lam (lam = 1:
// the update itself), partials of [a^T mode, sum log p(y | mode + F)]
__global__ void __launch_bounds__(kT) fl_trial_kernel(int n, int lik, double aux, double lam, const double* __restrict__ mode,
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

// after the mode finding (likelihoods.h:3200-3232): d1, W at the mode, DW = (W d + 1)^-1,
// dpwi = (d + W^-1)^-1; partials of [sum log dpwi, sum log W, #(W == 0)]
__global__ void __launch_bounds__(kT) fl_final_kernel(int n, int lik, double aux, const double* __restrict__ y,
                                                     const double* __restrict__ off, const double* __restrict__ mode,
                                                     const double* __restrict__ dvec, double* __restrict__ d1,
                                                     double* __restrict__ w, double* __restrict__ DW,
                                                     double* __restrict__ dpwi, double* __restrict__ part) {
  __shared__ double red[kT];
  double s0 = 0., s1 = 0., s2 = 0.;
  for (int i = blockIdx.x * kT + threadIdx.x; i < n; i += gridDim.x * kT) {
    const double mi = mode[i];
    const double l = off ? mi + off[i] : mi;
    d1[i] = lik_d1(lik, aux, y[i], l);
    const double wi = lik_info(lik, aux, y[i], l);
    w[i] = wi;
    const double di = dvec[i];
    DW[i] = 1. / (wi * di + 1.);
    const double p = 1. / (di + 1. / wi);
    dpwi[i] = p;
    s0 += log(p);
    s1 += log(wi);
    s2 += wi == 0. ? 1. : 0.;
  }
  const double a0 = block_sum(s0, red);
  const double a1 = block_sum(s1, red);
  const double a2 = block_sum(s2, red);
  if (threadIdx.x == 0) {
    part[3 * blockIdx.x] = a0;
    part[3 * blockIdx.x + 1] = a1;
    part[3 * blockIdx.x + 2] = a2;
  }
}

// gradient pass 0: part of [A a, A g, K g, dK g] (dK = dK_mn / dlog phi recomputed from the coordinates)
template <int COV>
__global__ void __launch_bounds__(kT) fl_grad_p0_kernel(const double* __restrict__ X, const double* __restrict__ Z,
                                                       int n, int m, int d, int ldm, double var, double phi,
                                                       const double* __restrict__ K, const double* __restrict__ A,
                                                       const double* __restrict__ a, const double* __restrict__ g,
                                                       double* __restrict__ part) {
  const int i0 = blockIdx.x * kChunk, i1 = min(n, i0 + kChunk);
  for (int j = threadIdx.x; j < m; j += kT) {
    double zj[3] = {0., 0., 0.};
    for (int q = 0; q < d; ++q) zj[q] = Z[(size_t)j * d + q];
    double s0 = 0., s1 = 0., s2 = 0., s3 = 0.;
    for (int i = i0; i < i1; ++i) {
      const size_t e = (size_t)j + (size_t)i * ldm;
      const double av = A[e], kv = K[e], ai = a[i], gi = g[i];
      double s = 0.;
      for (int q = 0; q < d; ++q) {
        const double t = X[(size_t)i * d + q] - zj[q];
        s += t * t;
      }
      double c, dk;
      cov_dcov<COV>(sqrt(s), var, phi, c, dk);
      s0 += av * ai;
      s1 += av * gi;
      s2 += kv * gi;
      s3 += dk * gi;
    }
    double* p = part + (size_t)blockIdx.x * 4 * ldm + j;
    p[0] = s0;
    p[ldm] = s1;
    p[2 * (size_t)ldm] = s2;
    p[3 * (size_t)ldm] = s3;
  }
}

// gradient pass 1 (likelihoods.h:5455-5525), one wave per observation, k = var / range:
//   fdg_k  = dvar_k - 2 sum_j A_ji dK_ji + sum_j A_ji (dK_mm A)_ji                  (fitc_diag_grad)
//   expl_k = -a_i sum_j dK_ji b_j - fdg_k a_i^2 / 2 + fdg_k p_i / 2 + p_i e_k - p_i^2 fdg_k f_i / 2
//            (b = A a, p = (d + W^-1)^-1, e_k = sum_j G_ji dK_ji, f = sum_j G_ji K_ji, G = M^-1 K)
//   sg_k   = sum_j dK_ji u1_j + sum_j A_ji h_k,j + fdg_k g_i   (Sigma_k' d1: u1 = A g, h_k = dK_k g - dK_mm,k u1)
//   dmll_i = 1/2 (DW_i^2 f_i + W_i^-1 - DW_i W_i^-1) dW_i/dmode     (d mll / d mode)
// For k = var, dK = K and dK_mm A = K - delta A (K_mm = K_mm,s - delta I).
template <int COV>
__global__ void __launch_bounds__(kT) fl_grad_p1_kernel(
    const double* __restrict__ X, const double* __restrict__ Z, int n, int m, int d, int ldm, int lik, double aux, double var,
    double phi, double delta, const double* __restrict__ K, const double* __restrict__ A, const double* __restrict__ G,
    const double* __restrict__ Mr, const double* __restrict__ b, const double* __restrict__ u1,
    const double* __restrict__ u2v, const double* __restrict__ u3v, const double* __restrict__ u2r,
    const double* __restrict__ u3r, const double* __restrict__ avec, const double* __restrict__ g,
    const double* __restrict__ w, const double* __restrict__ DW, const double* __restrict__ dpwi,
    const double* __restrict__ mode, const double* __restrict__ off, const double* __restrict__ y,
    double* __restrict__ sgv,
    double* __restrict__ sgr, double* __restrict__ dmll, double* __restrict__ sdiag, double* __restrict__ part) {
  __shared__ double red[4];
  const int lane = threadIdx.x & 63;
  const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
  double c1v = 0., sa2 = 0., c1r = 0., c2r = 0., f = 0., er = 0., hbv = 0., hbr = 0., huv = 0., hur = 0.;
  if (i < n) {
    double xi[3] = {0., 0., 0.};
    for (int q = 0; q < d; ++q) xi[q] = X[(size_t)i * d + q];
    for (int j = lane; j < m; j += 64) {
      const size_t e = (size_t)j + (size_t)i * ldm;
      const double kv = K[e], av = A[e], gv = G[e], mr = Mr[e];
      double s = 0.;
      for (int q = 0; q < d; ++q) {
        const double t = xi[q] - Z[(size_t)j * d + q];
        s += t * t;
      }
      double c, dk;
      cov_dcov<COV>(sqrt(s), var, phi, c, dk);
      c1v += av * kv;
      sa2 += av * av;
      c1r += av * dk;
      c2r += av * mr;
      f += gv * kv;
      er += gv * dk;
      const double bj = b[j], uj = u1[j];
      hbv += kv * bj;
      hbr += dk * bj;
      huv += kv * uj + av * (u2v[j] - u3v[j]);
      hur += dk * uj + av * (u2r[j] - u3r[j]);
    }
  }
  c1v = wsum(c1v);
  sa2 = wsum(sa2);
  c1r = wsum(c1r);
  c2r = wsum(c2r);
  f = wsum(f);
  er = wsum(er);
  hbv = wsum(hbv);
  hbr = wsum(hbr);
  huv = wsum(huv);
  hur = wsum(hur);
  double ev = 0., erng = 0.;
  if (i < n) {
    const double fdv = var - 2. * c1v + (c1v - delta * sa2);
    const double fdr = -2. * c1r + c2r;
    const double ai = avec[i], gi = g[i], p = dpwi[i], wi = w[i], dw = DW[i];
    ev = -ai * hbv - 0.5 * fdv * ai * ai + 0.5 * fdv * p + p * f - 0.5 * p * p * fdv * f;
    erng = -ai * hbr - 0.5 * fdr * ai * ai + 0.5 * fdr * p + p * er - 0.5 * p * p * fdr * f;
    if (lane == 0) {
      sgv[i] = huv + fdv * gi;
      sgr[i] = hur + fdr * gi;
      const double wi_inv = 1. / wi;
      const double sw = f * dw * dw + wi_inv - dw * wi_inv;   // diag of (Sigma^-1 + W)^-1 (:5447-5449)
      const double mi = mode[i];
      dmll[i] = 0.5 * sw * lik_dinfo(lik, aux, y[i], off ? mi + off[i] : mi);
      sdiag[i] = sw;
    }
  }
  ev = block4(ev, red);
  erng = block4(erng, red);
  if (threadIdx.x == 0) {
    part[2 * (size_t)blockIdx.x] = ev;
    part[2 * (size_t)blockIdx.x + 1] = erng;
  }
}

// gradient pass 3: the implicit derivative (likelihoods.h:5476-5482):
//   d mode / d par_k = W^-1 (p o sg_k - p o K^T vaux_k), grad_k += sum_i dmll_i (d mode / d par_k)_i
__global__ void __launch_bounds__(kT) fl_grad_p3_kernel(const double* __restrict__ K, int n, int m, int ldm,
                                                       const double* __restrict__ vv, const double* __restrict__ vr,
                                                       const double* __restrict__ sgv, const double* __restrict__ sgr,
                                                       const double* __restrict__ w, const double* __restrict__ dpwi,
                                                       const double* __restrict__ dmll, double* __restrict__ part) {
  __shared__ double red[4];
  const int lane = threadIdx.x & 63;
  const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
  double kv = 0., kr = 0.;
  if (i < n)
    for (int j = lane; j < m; j += 64) {
      const double x = K[(size_t)j + (size_t)i * ldm];
      kv += x * vv[j];
      kr += x * vr[j];
    }
  kv = wsum(kv);
  kr = wsum(kr);
  double iv = 0., ir = 0.;
  if (i < n) {
    const double wi_inv = 1. / w[i], p = dpwi[i], dm = dmll[i];
    iv = dm * (wi_inv * (p * sgv[i] - p * kv));
    ir = dm * (wi_inv * (p * sgr[i] - p * kr));
  }
  iv = block4(iv, red);
  ir = block4(ir, red);
  if (threadIdx.x == 0) {
    part[2 * (size_t)blockIdx.x] = iv;
    part[2 * (size_t)blockIdx.x + 1] = ir;
  }
}

// gradient wrt F (likelihoods.h:5510-5531): (Sigma^-1 + W)^-1 dmll = W^-1 dmll - DW^-1 W^-1 dmll
// + DW o K^T M^-1 K (DW o dmll); grad_F = -d1 + dmll - W o that. kq = K^T M^-1 K (DW o dmll) (coldot).
__global__ void __launch_bounds__(kT) fl_gradf_kernel(int n, const double* __restrict__ d1, const double* __restrict__ dmll,
                                                     const double* __restrict__ w, const double* __restrict__ DW,
                                                     const double* __restrict__ kq, double* __restrict__ out) {
  const int i = blockIdx.x * kT + threadIdx.x;
  if (i >= n) return;
  const double wi_inv = 1. / w[i], dm = dmll[i], dw = DW[i];
  const double wdm = wi_inv * dm;
  const double s = wdm - (1. / dw) * wdm + dw * kq[i];
  out[i] = -d1[i] + (dm - s * w[i]);
}

// gamma shape gradient records [l + y e^-l, W o diag((Sigma^-1 + W)^-1), d1 o (Sigma^-1 + W)^-1 dmll] with the
// implicit vector as in fl_gradf_kernel (likelihoods.h:5536-5540, 5560-5590)
__global__ void __launch_bounds__(kT) fl_aux_rec_kernel(int n, const double* __restrict__ y, const double* __restrict__ off,
                                                       const double* __restrict__ mode, const double* __restrict__ w,
                                                       const double* __restrict__ sdiag, const double* __restrict__ d1,
                                                       const double* __restrict__ dmll, const double* __restrict__ DW,
                                                       const double* __restrict__ kq, double* __restrict__ rec) {
  const int i = blockIdx.x * kT + threadIdx.x;
  if (i >= n) return;
  const double l = off ? mode[i] + off[i] : mode[i];
  const double wi_inv = 1. / w[i], dm = dmll[i], dw = DW[i];
  const double wdm = wi_inv * dm;
  const double sv = wdm - (1. / dw) * wdm + dw * kq[i];
  rec[3 * (size_t)i] = l + y[i] * exp(-l);
  rec[3 * (size_t)i + 1] = w[i] * sdiag[i];
  rec[3 * (size_t)i + 2] = d1[i] * sv;
}

__global__ void __launch_bounds__(kT) fl_mul_kernel(int n, const double* __restrict__ a, const double* __restrict__ b,
                                                   double* __restrict__ out) {
  const int i = blockIdx.x * kT + threadIdx.x;
  if (i < n) out[i] = a[i] * b[i];
}

// prediction correction per matched pair (prediction point p, training point o), CalcPredFITC_FSA
// re_model_template.h:10681 and likelihoods.h:7196-7199: corr = sigma1^2 - (L^-1 K_mp)_p . (L^-1 K_mn)_o;
// Maux[:, p] -= K_mn[:, o] (d_o + W_o^-1)^-1 corr (one wave per pair; a prediction point has at most one pair)
__global__ void __launch_bounds__(64) fl_pred_corr_kernel(const int* __restrict__ pairs, int npairs,
                                                         const double* __restrict__ Vp, const double* __restrict__ V,
                                                         const double* __restrict__ K, const double* __restrict__ dpwi,
                                                         int m, int ldm, double sii, double* __restrict__ Maux,
                                                         double* __restrict__ corr) {
  const int q = blockIdx.x;
  if (q >= npairs) return;
  const int p = pairs[2 * q], o = pairs[2 * q + 1];
  const int lane = threadIdx.x;
  double s = 0.;
  for (int j = lane; j < m; j += 64) s += Vp[(size_t)j + (size_t)p * ldm] * V[(size_t)j + (size_t)o * ldm];
  s = wsum(s);
  const double c = sii - s;
  const double f = dpwi[o] * c;
  for (int j = lane; j < m; j += 64) Maux[(size_t)j + (size_t)p * ldm] -= K[(size_t)j + (size_t)o * ldm] * f;
  if (lane == 0) corr[q] = c;
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

FitcLaplace::FitcLaplace(FitcSolver* fitc, hipStream_t stream)
    : F_(fitc), s_(stream), n_(fitc->n_), m_(fitc->m_), ldm_(fitc->ldm_) {
  const int n = n_, ldm = ldm_;
  for (DevBuf<double>* b : {&y_, &off_, &mode_, &a_, &mode_prev_, &a_prev_, &mode_upd_, &a_upd_, &d1_, &w_, &wdw_, &dw_,
                            &rhs_, &sig_, &c_, &z_, &sgv_, &sgr_, &dmll_, &sdiag_})
    b->alloc(n);
  auxrec_.alloc((size_t)3 * n);
  mv_.alloc((size_t)kMv * ldm);
  HIP_CHECK(hipMemsetAsync(mv_.get(), 0, sizeof(double) * kMv * ldm, s_));
  const size_t nbg = (size_t)(n + kChunk - 1) / kChunk;
  part_.alloc(std::max<size_t>({nbg * 4 * ldm, (size_t)((n + 3) / 4) * 2, (size_t)nb_red(n) * 3, (size_t)6 * ((m_ + 3) / 4)}));
  red_.alloc(32);
  HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&h_red_), 32 * sizeof(double), hipHostMallocDefault));
  HIP_CHECK(hipMemsetAsync(mode_.get(), 0, sizeof(double) * n, s_));
  HIP_CHECK(hipMemsetAsync(a_.get(), 0, sizeof(double) * n, s_));
  HIP_CHECK(hipStreamSynchronize(s_));
}

FitcLaplace::~FitcLaplace() {
  if (h_red_) (void)hipHostFree(h_red_);
}

void FitcLaplace::SetY(const double* y) {
  sum_log_y_ = 0.;   // aux_log_normalizing_constant_ of likelihood 'gamma' (likelihoods.h:8181-8191)
  for (int i = 0; i < n_; ++i) sum_log_y_ += y[i] > 0. ? std::log(y[i]) : 0.;
  HIP_CHECK(hipMemcpyAsync(y_.get(), y, sizeof(double) * n_, hipMemcpyHostToDevice, s_));
  HIP_CHECK(hipStreamSynchronize(s_));
  y_set_ = true;
}

void FitcLaplace::SetOffset(const double* off) {
  has_off_ = off != nullptr;
  if (has_off_) {
    HIP_CHECK(hipMemcpyAsync(off_.get(), off, sizeof(double) * n_, hipMemcpyHostToDevice, s_));
    HIP_CHECK(hipStreamSynchronize(s_));
  }
}

void FitcLaplace::GetMode(double* mode) {
  HIP_CHECK(hipMemcpyAsync(mode, mode_.get(), sizeof(double) * n_, hipMemcpyDeviceToHost, s_));
  HIP_CHECK(hipStreamSynchronize(s_));
}

void FitcLaplace::ResetModeToPrevious() {
  if (!prev_valid_) return;
  HIP_CHECK(hipMemcpyAsync(mode_.get(), mode_prev_.get(), sizeof(double) * n_, hipMemcpyDeviceToDevice, s_));
  HIP_CHECK(hipMemcpyAsync(a_.get(), a_prev_.get(), sizeof(double) * n_, hipMemcpyDeviceToDevice, s_));
  HIP_CHECK(hipStreamSynchronize(s_));
}

void FitcLaplace::Gemv(const double* M, int nv, const double* const* x, double* const* out) {
  const int n = n_, m = m_, ldm = ldm_;
  const int nb = (n + kChunk - 1) / kChunk;
  Vec4 xv{};
  OutVec4 ov{};
  for (int v = 0; v < nv; ++v) {
    xv.p[v] = x[v];
    ov.p[v] = out[v];
  }
  switch (nv) {
    case 1: hipLaunchKernelGGL(fl_gemv_part_kernel<1>, dim3(nb), dim3(kT), 0, s_, M, xv, n, m, ldm, part_.get()); break;
    case 2: hipLaunchKernelGGL(fl_gemv_part_kernel<2>, dim3(nb), dim3(kT), 0, s_, M, xv, n, m, ldm, part_.get()); break;
    default: Fatal("FitcLaplace::Gemv: %d vectors", nv);
  }
  hipLaunchKernelGGL(fl_gemv_reduce_kernel, dim3((nv * m + 3) / 4), dim3(kT), 0, s_, part_.get(), nb, nv, m, ldm, ov);
  HIP_CHECK(hipGetLastError());
}

void FitcLaplace::SigmaApply(const double* x, double* out) {
  // Sigma x = K^T (K_mm,s^-1 (K x)) + d o x  (likelihoods.h:3153-3154, chol_fact_sigma_ip.solve)
  double* t1 = mv_.get();
  double* t2 = t1 + ldm_;
  Gemv(F_->Kmn_.get(), 1, &x, &t1);
  fitc_chol_solve(s_, F_->Li_.get(), F_->LiT_.get(), t1, m_, ldm_, t1 + 4 * (size_t)ldm_, t2);
  hipLaunchKernelGGL(fl_coldot_kernel, dim3((n_ + 3) / 4), dim3(kT), 0, s_, F_->Kmn_.get(), t2, nullptr, n_, m_, ldm_,
                     c_.get(), nullptr);
  const double* dvec = F_->vec_.get();
  hipLaunchKernelGGL(fl_sigma_kernel, dim3(nb_thread(n_)), dim3(kT), 0, s_, n_, c_.get(), dvec, x, nullptr, out, nullptr);
  HIP_CHECK(hipGetLastError());
}

void FitcLaplace::Woodbury(const double* s, double* logdet_dev, bool full_inverse) {
  FitcSolver& F = *F_;
  const int n = n_, m = m_, ldm = ldm_;
  hipLaunchKernelGGL(fl_colscale_kernel, dim3((m + 63) / 64, (n + 3) / 4), dim3(kT), 0, s_, F.Kmn_.get(), s, n, m, ldm,
                     F.Kd_.get());
  HIP_CHECK(hipGetLastError());
  const long mm = (long)ldm * ldm;
  const int chunks = gemm_f64_splitk(s_, m, m, n, F.Kmn_.get(), ldm, 0, F.Kd_.get(), ldm, 1, F.part_.get(), ldm, mm,
                                     2048, F.max_chunks_);
  fitc_wsum(s_, F.part_.get(), chunks, mm, m, ldm, F.Ks_.get(), F.W_.get());
  chol_lower(s_, F.W_.get(), F.Wi_.get(), m, ldm, F.info_.get());
  launch_logdet_chol(s_, F.W_.get(), ldm, m, logdet_dev);
  trtri_lower(s_, F.W_.get(), F.Wi_.get(), F.T_.get(), 0, m, ldm);
  fitc_lower_t(s_, F.Wi_.get(), m, ldm, F.WiT_.get());
  // M^-1 itself only for the gradient's trace terms (fitc_mm_terms)
  if (full_inverse)
    gemm_f64(s_, m, m, m, 1., F.Wi_.get(), ldm, 1, F.Wi_.get(), ldm, 0, 0., F.Winv_.get(), ldm, 0, 0, 1, 1);
}

LatentResult FitcLaplace::Eval(int cov_type, int lik, const double* trafo, double aux, const IterativeConfig& cfg,
                               bool want_grad, bool want_aux_grad, double* grad_f, ModeStart start) {
  if (!y_set_) Fatal("response variable y has not been set");
  aux_ = lik == kLikGamma ? aux : 1.;
  const bool want_aux = want_aux_grad && want_grad && lik == kLikGamma;
  if (lik == kLikGaussian) Fatal("FitcLaplace: the Gaussian likelihood uses the exact FITC path");
  FitcSolver& F = *F_;
  const int n = n_, m = m_, ldm = ldm_, d = F.d_;
  const double var = trafo[0], phi = trafo[1];
  const double* off = has_off_ ? off_.get() : nullptr;
  double* red = red_.get();
  double* dvec = F.vec_.get();
  hipEvent_t e0 = F.ev_[0], e1 = F.ev_[2];
  HIP_CHECK(hipEventRecord(e0, s_));
  // Sigma components (CalcSigmaComps :7341-7378): K_mn, K_mm,s, L^-1, V = L^-1 K_mn, K_mm,s^-1; d
  F.Prior(cov_type, var, phi, red + 0);
  hipLaunchKernelGGL(fl_diag_kernel, dim3((n + 3) / 4), dim3(kT), 0, s_, F.V_.get(), n, m, ldm, var * kJitterMult, dvec);
  HIP_CHECK(hipGetLastError());
  auto info_failed = [&]() {
    int info = 0;
    HIP_CHECK(hipMemcpyAsync(&info, F.info_.get(), sizeof(int), hipMemcpyDeviceToHost, s_));
    HIP_CHECK(hipStreamSynchronize(s_));
    return info != 0;
  };
  const int nbr = nb_red(n);
  // objective -1/2 a^T mode + log p(y | mode + F) of the state (mode_, a_)
  auto objective = [&](double lam, const double* mu, const double* au, double* mnew, double* anew) {
    hipLaunchKernelGGL(fl_trial_kernel, dim3(nbr), dim3(kT), 0, s_, n, lik, aux_, lam, mode_.get(), a_.get(), mu, au, y_.get(),
                       off, mnew, anew, part_.get());
    HIP_CHECK(hipGetLastError());
    launch_sum_blocks(part_.get(), nbr, 2, red + 4, s_);
    HIP_CHECK(hipMemcpyAsync(h_red_ + 4, red + 4, 2 * sizeof(double), hipMemcpyDeviceToHost, s_));
    HIP_CHECK(hipStreamSynchronize(s_));
    return -0.5 * h_red_[4] + (h_red_[5] + loglik_const_);
  };
  LatentResult res;
  if (info_failed()) throw LatentNan("the inducing-point covariance is not positive definite (Cholesky failed)");
  // mode start (likelihoods.h:3106-3115): zero, or mode = Sigma a of the previous a
  if (start == ModeStart::kZero || !evaluated_) {
    HIP_CHECK(hipMemsetAsync(mode_.get(), 0, sizeof(double) * n, s_));
    HIP_CHECK(hipMemsetAsync(a_.get(), 0, sizeof(double) * n, s_));
    prev_valid_ = false;
  } else if (start == ModeStart::kWarm) {
    HIP_CHECK(hipMemcpyAsync(mode_prev_.get(), mode_.get(), sizeof(double) * n, hipMemcpyDeviceToDevice, s_));
    HIP_CHECK(hipMemcpyAsync(a_prev_.get(), a_.get(), sizeof(double) * n, hipMemcpyDeviceToDevice, s_));
    prev_valid_ = true;
    SigmaApply(a_.get(), mode_.get());
  }
  double* logdet_M = red + 1;
  int it = 0;
  if (start != ModeStart::kKeep || !evaluated_) {
    double obj = objective(1., mode_.get(), a_.get(), mode_upd_.get(), a_upd_.get());
    const int maxit = 1000;                                // maxit_mode_newton_ (likelihoods.h:12721)
    const double delta = cfg.delta_conv_mode_finding;       // :12723
    bool terminate = false, has_nan = false;
    double* vaux = mv_.get() + 2 * (size_t)ldm;
    double* vaux2 = mv_.get() + 3 * (size_t)ldm;
    for (it = 0; it < maxit; ++it) {
      // information changes in every step for the supported likelihoods (information_changes_during_mode_finding_)
      hipLaunchKernelGGL(fl_prep_kernel, dim3(nb_thread(n)), dim3(kT), 0, s_, n, lik, aux_, y_.get(), off, mode_.get(), dvec, 1,
                         d1_.get(), w_.get(), wdw_.get(), dw_.get(), rhs_.get());
      HIP_CHECK(hipGetLastError());
      Woodbury(wdw_.get(), logdet_M, false);
      // Sigma rhs, vaux = K (W DW Sigma rhs), vaux2 = M^-1 vaux, K^T vaux2 (likelihoods.h:3152-3157)
      SigmaApply(rhs_.get(), sig_.get());
      hipLaunchKernelGGL(fl_mul_kernel, dim3(nb_thread(n)), dim3(kT), 0, s_, n, wdw_.get(), sig_.get(), z_.get());
      const double* zp = z_.get();
      Gemv(F.Kmn_.get(), 1, &zp, &vaux);
      fitc_chol_solve(s_, F.Wi_.get(), F.WiT_.get(), vaux, m, ldm, mv_.get() + 4 * (size_t)ldm, vaux2);
      hipLaunchKernelGGL(fl_coldot_kernel, dim3((n + 3) / 4), dim3(kT), 0, s_, F.Kmn_.get(), vaux2, nullptr, n, m, ldm,
                         c_.get(), nullptr);
      hipLaunchKernelGGL(fl_aupd_kernel, dim3(nb_thread(n)), dim3(kT), 0, s_, n, rhs_.get(), w_.get(), dw_.get(),
                         sig_.get(), c_.get(), a_upd_.get());
      HIP_CHECK(hipGetLastError());
      SigmaApply(a_upd_.get(), mode_upd_.get());   // mode_update = Sigma SigmaI_mode_update
      if (info_failed()) {   // the Woodbury matrix is not positive definite
        has_nan = true;
        break;
      }
      hipLaunchKernelGGL(fl_gdd_kernel, dim3(nbr), dim3(kT), 0, s_, n, mode_.get(), a_.get(), mode_upd_.get(),
                         a_upd_.get(), w_.get(), part_.get());
      launch_sum_blocks(part_.get(), nbr, 1, red + 6, s_);
      HIP_CHECK(hipMemcpyAsync(h_red_ + 6, red + 6, sizeof(double), hipMemcpyDeviceToHost, s_));
      HIP_CHECK(hipStreamSynchronize(s_));
      const double gdd = h_red_[6];
      // backtracking (:3171-3192); the last trial is kept when none is accepted
      double lam = 1., obj_new = obj;
      for (int ih = 0; ih < 20; ++ih) {   // max_number_lr_shrinkage_steps_newton_ (:12725)
        obj_new = objective(lam, mode_upd_.get(), a_upd_.get(), sig_.get(), c_.get());
        if (obj_new < obj + 1e-4 * lam * gdd || std::isnan(obj_new) || std::isinf(obj_new)) lam *= 0.5;   // c_armijo_ 1e-4
        else break;
      }
      std::swap(mode_, sig_);   // mode_ = mode_new, SigmaI_mode_ = SigmaI_mode_new
      std::swap(a_, c_);
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
    if (has_nan) throw LatentNan("NaN or Inf occurred in the FITC mode finding");
    res.newton_its = it;
    cached_obj_ = obj;
  }
  evaluated_ = true;
  // after the mode finding (:3200-3232): d1, W at the mode; M = K_mm,s + K diag((d + W^-1)^-1) K^T
  hipLaunchKernelGGL(fl_final_kernel, dim3(nbr), dim3(kT), 0, s_, n, lik, aux_, y_.get(), off, mode_.get(), dvec, d1_.get(),
                     w_.get(), dw_.get(), wdw_.get(), part_.get());
  HIP_CHECK(hipGetLastError());
  launch_sum_blocks(part_.get(), nbr, 3, red + 8, s_);
  Woodbury(wdw_.get(), logdet_M, want_grad || grad_f != nullptr);
  HIP_CHECK(hipMemcpyAsync(h_red_, red, 12 * sizeof(double), hipMemcpyDeviceToHost, s_));
  HIP_CHECK(hipStreamSynchronize(s_));
  if (h_red_[10] > 0.)
    Fatal("FindModePostRandEffCalcMLLFITC: 0's found in the (diagonal) Hessian (or Fisher information) of the negative "
          "log-likelihood. This is not permitted when using the FITC approximation ");
  if (info_failed()) throw LatentNan("the FITC Woodbury matrix is not positive definite (Cholesky failed)");
  // mll = obj - sum log diag chol(M) + sum log diag chol(K_mm,s) + 1/2 sum log (d + W^-1)^-1 - 1/2 sum log W
  const double mll = cached_obj_ - 0.5 * h_red_[1] + 0.5 * h_red_[0] + 0.5 * h_red_[8] - 0.5 * h_red_[9];
  res.nll = -mll;
  res.logdet = 0.5 * h_red_[1] - 0.5 * h_red_[0] - 0.5 * h_red_[8] + 0.5 * h_red_[9];
  if (!std::isfinite(res.nll)) throw LatentNan("NaN or Inf in the FITC approximate marginal likelihood");
  if (want_grad || grad_f != nullptr) {
    const double delta_j = var * kJitterMult - var;
    double* mv = mv_.get();
    double* b = mv + 6 * (size_t)ldm;
    double* u1 = mv + 7 * (size_t)ldm;
    double* u2v = mv + 8 * (size_t)ldm;
    double* u2r = mv + 9 * (size_t)ldm;
    double* u3v = mv + 10 * (size_t)ldm;
    double* u3r = mv + 11 * (size_t)ldm;
    double* rv = mv + 12 * (size_t)ldm;
    double* rr = mv + 13 * (size_t)ldm;
    double* xv = mv + 14 * (size_t)ldm;
    double* xr = mv + 15 * (size_t)ldm;
    // A = K_mm,s^-1 K = L^-T V (A_), G = M^-1 K (Kd_), M_r = dK_mm A (V_)
    gemm_f64(s_, m, n, m, 1., F.Li_.get(), ldm, 1, F.V_.get(), ldm, 0, 0., F.A_.get(), ldm, 0, 0, 1, 0);
    // G = M^-1 K (fitc_solve_kmn; V_ is scratch until M_r below)
    fitc_solve_kmn(s_, F.Wi_.get(), F.Winv_.get(), F.Kmn_.get(), m, n, ldm, F.V_.get(), F.Kd_.get());
    gemm_f64(s_, m, n, m, 1., F.dKmm_.get(), ldm, 0, F.A_.get(), ldm, 0, 0., F.V_.get(), ldm);
    const int nbg = (n + kChunk - 1) / kChunk;
    dispatch_cov(cov_type, [&](auto c) {
      hipLaunchKernelGGL((fl_grad_p0_kernel<decltype(c)::value>), dim3(nbg), dim3(kT), 0, s_, F.d_X_, F.dZ_.get(), n, m, d,
                         ldm, var, phi, F.Kmn_.get(), F.A_.get(), a_.get(), d1_.get(), part_.get());
    });
    OutVec4 ov{{b, u1, u2v, u2r}};
    hipLaunchKernelGGL(fl_gemv_reduce_kernel, dim3((4 * m + 3) / 4), dim3(kT), 0, s_, part_.get(), nbg, 4, m, ldm, ov);
    HIP_CHECK(hipGetLastError());
    fitc_symv(s_, F.Kmm_.get(), u1, m, ldm, u3v);
    fitc_symv(s_, F.dKmm_.get(), u1, m, ldm, u3r);
    // m x m terms (into red[12..17]) before part_ is reused
    fitc_mm_terms(s_, F.Kinv_.get(), F.Winv_.get(), F.Kmm_.get(), F.dKmm_.get(), b, m, ldm, part_.get(), red + 12);
    const int nb4 = (n + 3) / 4;
    double* part1 = F.part_.get();   // pass-1 partials (the split-K Gram scratch is free now)
    dispatch_cov(cov_type, [&](auto c) {
      hipLaunchKernelGGL((fl_grad_p1_kernel<decltype(c)::value>), dim3(nb4), dim3(kT), 0, s_, F.d_X_, F.dZ_.get(), n, m, d,
                         ldm, lik, aux_, var, phi, delta_j, F.Kmn_.get(), F.A_.get(), F.Kd_.get(), F.V_.get(), b, u1, u2v, u3v,
                         u2r, u3r, a_.get(), d1_.get(), w_.get(), dw_.get(), wdw_.get(), mode_.get(), off, y_.get(), sgv_.get(),
                         sgr_.get(), dmll_.get(), sdiag_.get(), part1);
    });
    HIP_CHECK(hipGetLastError());
    launch_sum_blocks(part1, nb4, 2, red + 18, s_);
    // rhs_k = K (p o sg_k), vaux_k = M^-1 rhs_k
    hipLaunchKernelGGL(fl_mul_kernel, dim3(nb_thread(n)), dim3(kT), 0, s_, n, wdw_.get(), sgv_.get(), z_.get());
    hipLaunchKernelGGL(fl_mul_kernel, dim3(nb_thread(n)), dim3(kT), 0, s_, n, wdw_.get(), sgr_.get(), rhs_.get());
    const double* zx[2] = {z_.get(), rhs_.get()};
    double* zo[2] = {rv, rr};
    Gemv(F.Kmn_.get(), 2, zx, zo);
    fitc_chol_solve(s_, F.Wi_.get(), F.WiT_.get(), rv, m, ldm, mv + 4 * (size_t)ldm, xv);
    fitc_chol_solve(s_, F.Wi_.get(), F.WiT_.get(), rr, m, ldm, mv + 4 * (size_t)ldm, xr);
    hipLaunchKernelGGL(fl_grad_p3_kernel, dim3(nb4), dim3(kT), 0, s_, F.Kmn_.get(), n, m, ldm, xv, xr, sgv_.get(),
                       sgr_.get(), w_.get(), wdw_.get(), dmll_.get(), part1);
    HIP_CHECK(hipGetLastError());
    launch_sum_blocks(part1, nb4, 2, red + 20, s_);
    if (grad_f != nullptr || want_aux) {   // kq = K^T M^-1 K (DW o dmll) for (Sigma^-1 + W)^-1 dmll
      double* q = mv + 16 * (size_t)ldm;
      double* q2 = mv + 17 * (size_t)ldm;
      hipLaunchKernelGGL(fl_mul_kernel, dim3(nb_thread(n)), dim3(kT), 0, s_, n, dw_.get(), dmll_.get(), z_.get());
      const double* zp = z_.get();
      Gemv(F.Kmn_.get(), 1, &zp, &q);
      fitc_chol_solve(s_, F.Wi_.get(), F.WiT_.get(), q, m, ldm, mv + 4 * (size_t)ldm, q2);
      hipLaunchKernelGGL(fl_coldot_kernel, dim3(nb4), dim3(kT), 0, s_, F.Kmn_.get(), q2, nullptr, n, m, ldm, c_.get(),
                         nullptr);
    }
    if (want_aux) {
      hipLaunchKernelGGL(fl_aux_rec_kernel, dim3(nb_thread(n)), dim3(kT), 0, s_, n, y_.get(), off, mode_.get(), w_.get(),
                         sdiag_.get(), d1_.get(), dmll_.get(), dw_.get(), c_.get(), auxrec_.get());
      HIP_CHECK(hipGetLastError());
      launch_sum_blocks(auxrec_.get(), n, 3, red + 24, s_);
    }
    if (grad_f != nullptr) {
      hipLaunchKernelGGL(fl_gradf_kernel, dim3(nb_thread(n)), dim3(kT), 0, s_, n, d1_.get(), dmll_.get(), w_.get(),
                         dw_.get(), c_.get(), z_.get());
      HIP_CHECK(hipGetLastError());
      HIP_CHECK(hipMemcpyAsync(grad_f, z_.get(), sizeof(double) * n, hipMemcpyDeviceToHost, s_));
    }
    HIP_CHECK(hipMemcpyAsync(h_red_ + 12, red + 12, 10 * sizeof(double), hipMemcpyDeviceToHost, s_));
    HIP_CHECK(hipStreamSynchronize(s_));
    const double* t = h_red_ + 12;   // KinvKmm, MinvKmm, KinvdK, MinvdK, bKmmb, bdKb
    const double* ex = h_red_ + 18;  // explicit per-observation sums (var, range)
    const double* im = h_red_ + 20;  // implicit sums
    res.grad = {ex[0] + 0.5 * t[4] + 0.5 * t[1] - 0.5 * t[0] + im[0], ex[1] + 0.5 * t[5] + 0.5 * t[3] - 0.5 * t[2] + im[1]};
    if (want_aux) {   // gamma shape on the log scale (likelihoods.h:10514-10524 + the two trace terms)
      HIP_CHECK(hipMemcpyAsync(h_red_ + 24, red + 24, 3 * sizeof(double), hipMemcpyDeviceToHost, s_));
      HIP_CHECK(hipStreamSynchronize(s_));
      const double a = aux_;
      const double neg = a * (h_red_[24] - n * (std::log(a) + 1. - digamma_asa103(a)) - sum_log_y_);
      res.grad.push_back(neg + 0.5 * h_red_[25] + h_red_[26]);
    }
  }
  HIP_CHECK(hipEventRecord(e1, s_));
  HIP_CHECK(hipEventSynchronize(e1));
  float ms = 0.f;
  HIP_CHECK(hipEventElapsedTime(&ms, e0, e1));
  res.ms_total = ms;
  return res;
}

void FitcLaplace::Predict(int cov_type, double var, double phi, const double* Xp, int np, const std::vector<int>& match,
                          bool want_var, bool want_cov, double* mean, double* pvar, double* pcov) {
  FitcSolver& F = *F_;
  const int n = n_, m = m_, ldm = ldm_, d = F.d_;
  if (!evaluated_) Fatal("FitcLaplace::Predict needs an evaluation at the prediction parameters");
  DevBuf<double> dXp((size_t)np * d), Kmp((size_t)ldm * np), out((size_t)3 * np);
  HIP_CHECK(hipMemcpyAsync(dXp.get(), Xp, sizeof(double) * np * d, hipMemcpyHostToDevice, s_));
  fitc_kmn(s_, cov_type, dXp.get(), F.dZ_.get(), np, m, d, ldm, var, phi, Kmp.get());
  // mean = K_pm (K_mm,s^-1 (K_mn d1)) (likelihoods.h:7183)
  double* t1 = mv_.get();
  double* t2 = t1 + ldm;
  const double* g = d1_.get();
  Gemv(F.Kmn_.get(), 1, &g, &t1);
  fitc_chol_solve(s_, F.Li_.get(), F.LiT_.get(), t1, m, ldm, t1 + 4 * (size_t)ldm, t2);
  const int nb4 = (np + 3) / 4;
  hipLaunchKernelGGL(fl_coldot_kernel, dim3(nb4), dim3(kT), 0, s_, Kmp.get(), t2, nullptr, np, m, ldm, out.get(), nullptr);
  HIP_CHECK(hipGetLastError());
  std::vector<int> pairs;
  for (int p = 0; p < np; ++p)
    if (match[p] >= 0) {
      pairs.push_back(p);
      pairs.push_back(match[p]);
    }
  const int npairs = (int)pairs.size() / 2;
  DevBuf<double> Vp, U, Maux, dcorr(std::max(npairs, 1));
  DevBuf<int> dpairs(std::max<size_t>(pairs.size(), 2));
  std::vector<double> h_corr(npairs);
  const bool need_v = want_var || want_cov || npairs > 0;
  if (need_v) {
    // Vp = L^-1 K_mp (resid = sigma1^2 - |Vp_p|^2, re_model_template.h:10741-10759); Maux = K_mp - corrections
    Vp.alloc((size_t)ldm * np);
    Maux.alloc((size_t)ldm * np);
    gemm_f64(s_, m, np, m, 1., F.Li_.get(), ldm, 0, Kmp.get(), ldm, 0, 0., Vp.get(), ldm, 0, 1, 0, 0);
    HIP_CHECK(hipMemcpyAsync(Maux.get(), Kmp.get(), sizeof(double) * ldm * np, hipMemcpyDeviceToDevice, s_));
    if (npairs > 0) {
      HIP_CHECK(hipMemcpyAsync(dpairs.get(), pairs.data(), sizeof(int) * pairs.size(), hipMemcpyHostToDevice, s_));
      hipLaunchKernelGGL(fl_pred_corr_kernel, dim3(npairs), dim3(64), 0, s_, dpairs.get(), npairs, Vp.get(), F.V_.get(),
                         F.Kmn_.get(), wdw_.get(), m, ldm, var, Maux.get(), dcorr.get());
      HIP_CHECK(hipGetLastError());
      HIP_CHECK(hipMemcpyAsync(h_corr.data(), dcorr.get(), sizeof(double) * npairs, hipMemcpyDeviceToHost, s_));
    }
  }
  if (want_var || want_cov) {
    // U = Lm^-1 Maux (TriangularSolveGivenCholesky(chol_fact_dense_Newton_), likelihoods.h:7201)
    U.alloc((size_t)ldm * np);
    gemm_f64(s_, m, np, m, 1., F.Wi_.get(), ldm, 0, Maux.get(), ldm, 0, 0., U.get(), ldm, 0, 1, 0, 0);
    hipLaunchKernelGGL(fl_coldot_kernel, dim3(nb4), dim3(kT), 0, s_, Vp.get(), nullptr, nullptr, np, m, ldm,
                       out.get() + np, nullptr);
    hipLaunchKernelGGL(fl_coldot_kernel, dim3(nb4), dim3(kT), 0, s_, U.get(), nullptr, nullptr, np, m, ldm,
                       out.get() + 2 * (size_t)np, nullptr);
    HIP_CHECK(hipGetLastError());
  }
  std::vector<double> h((size_t)3 * np), g_h(npairs > 0 ? n : 0), dp_h(npairs > 0 ? n : 0);
  HIP_CHECK(hipMemcpyAsync(h.data(), out.get(), sizeof(double) * h.size(), hipMemcpyDeviceToHost, s_));
  if (npairs > 0) {
    HIP_CHECK(hipMemcpyAsync(g_h.data(), d1_.get(), sizeof(double) * n, hipMemcpyDeviceToHost, s_));
    HIP_CHECK(hipMemcpyAsync(dp_h.data(), wdw_.get(), sizeof(double) * n, hipMemcpyDeviceToHost, s_));
  }
  HIP_CHECK(hipStreamSynchronize(s_));
  std::copy(h.begin(), h.begin() + np, mean);
  for (int q = 0; q < npairs; ++q) mean[pairs[2 * q]] += h_corr[q] * g_h[pairs[2 * q + 1]];   // :7184-7186
  if (want_var) {
    for (int p = 0; p < np; ++p) pvar[p] = (var - h[np + p]) + h[2 * (size_t)np + p];
    for (int q = 0; q < npairs; ++q) {   // - corr (d + W^-1)^-1 corr (:7215-7219)
      const double c = h_corr[q];
      pvar[pairs[2 * q]] -= c * (dp_h[pairs[2 * q + 1]] * c);
    }
  }
  if (want_cov) {
    DevBuf<double> C((size_t)np * np);
    gemm_f64(s_, np, np, m, 1., U.get(), ldm, 1, U.get(), ldm, 0, 0., C.get(), np);
    HIP_CHECK(hipMemcpyAsync(pcov, C.get(), sizeof(double) * np * np, hipMemcpyDeviceToHost, s_));
    HIP_CHECK(hipStreamSynchronize(s_));
    for (int p = 0; p < np; ++p) pcov[(size_t)p * np + p] += var - h[np + p];
    // - fitc_resid_pred_obs diag(p) fitc_resid_pred_obs^T (:7205-7210): a training point's pairs together
    std::vector<int> order(npairs);
    for (int q = 0; q < npairs; ++q) order[q] = q;
    std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return pairs[2 * a + 1] < pairs[2 * b + 1]; });
    for (int g0 = 0; g0 < npairs;) {
      int g1 = g0 + 1;
      while (g1 < npairs && pairs[2 * order[g1] + 1] == pairs[2 * order[g0] + 1]) ++g1;
      const double dpo = dp_h[pairs[2 * order[g0] + 1]];
      for (int a = g0; a < g1; ++a)
        for (int b = g0; b < g1; ++b) {
          const int q = order[a], r = order[b];
          pcov[(size_t)pairs[2 * r] * np + pairs[2 * q]] -= h_corr[q] * dpo * h_corr[r];
        }
      g0 = g1;
    }
  }
}

}  // namespace gpb_amd
