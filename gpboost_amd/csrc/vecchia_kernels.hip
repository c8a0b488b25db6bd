// Vecchia factor + likelihood/gradient row kernel for gfx950 (CDNA4, wave64).
//
// Reference path replaced: CalcCovFactorGradientVecchia (Vecchia_utils.cpp:1307-1632,
// per-row loop :1405-1617) fused with CalcYAux / CalcYTPsiIInvY
// (re_model_template.h:8885-9120) and the Vecchia branch of CalcGradPars (:1768-1791).
//
// Mapping: one Vecchia row i (k_i = min(i, m) neighbours) is owned by a group of K
// lanes of one wavefront (K = 16/32/64 -> 4/2/1 rows per wave); lane r owns row r of
// the k x k between-neighbour covariance C_i. Rows >= k_i are identity padding, which
// leaves the factor unchanged. All synchronisation is wave-local (no block barrier
// in the factor part).
//
// Per-row LDS image (K x (K+1) doubles, padded so row and column sweeps are
// bank-conflict free):   strictly lower = C_i, diagonal = C_ii + nugget,
//                        strictly upper = dC_i/dlog(phi)  (both symmetric)
// 1. the k(k-1)/2 covariance pairs (the exp-heavy part) are computed ONCE, spread
//    evenly over the K lanes, and written to both triangles;
// 2. lane r pulls row r of C into registers, right-looking Cholesky in registers
//    (pivot by lane shuffle, column j broadcast through a K-double LDS slot);
// 3. forward solves in registers; L is written back over the lower triangle and the
//    backward solves read its columns from LDS;
// 4. t = dC a is read from the upper triangle.
// Instead of forming B, D and their derivatives, the row emits six partial sums
// (logD, (By)^2/D, and per parameter s1 = uk*u - u^2 dD/2, s2 = dD/D; DESIGN.md
// "reduction contract") using a = C^-1 c, v = C^-1 y_nbr and t (O(k^2) per parameter).
// Optional outputs D^-1 and B(i, nbr) = -a are written for the factor API.
#include <hip/hip_runtime.h>

#include "common.h"
#include "cov.h"
#include "kernels.h"

namespace gpb_amd {
namespace {

constexpr int kDMax = 3;

// Orders a wave's own LDS writes before its subsequent LDS reads (and vice versa).
__device__ __forceinline__ void wave_lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

template <int K>
__device__ __forceinline__ double group_sum(double v) {
#pragma unroll
  for (int off = K / 2; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

template <int K>
constexpr int block_threads() { return K == 64 ? 64 : 256; }

template <int K>
constexpr int group_lds_doubles() {
  return K * (K + 1) + (kDMax + 1) * K;   // C/dC/L image + neighbour coords + broadcast slot
}

template <int K, int COV>
__global__ void __launch_bounds__(block_threads<K>()) vecchia_rows_kernel(VecchiaRowsArgs a) {
  extern __shared__ __attribute__((aligned(16))) double smem[];
  constexpr int BT = block_threads<K>();
  constexpr int G = 64 / K;                 // rows per wave
  constexpr int KP = K + 1;                 // padded row stride
  constexpr int rows_per_block = (BT / 64) * G;
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int g = lane / K;
  const int r = lane - g * K;
  const int gbase = g * K;
  const int group_id = wave * G + g;
  const int i = a.r0 + blockIdx.x * rows_per_block + group_id;
  const bool active = i < a.r1;
  const int k = active ? min(i, a.m) : 0;
  const bool rv = r < k;
  const int d = a.d;

  double* img = smem + group_id * group_lds_doubles<K>();
  double* nbx = img + K * KP;              // K x kDMax
  double* bcast = nbx + K * kDMax;         // K

  // ---- gather: neighbour index, coordinates, response (Vecchia order)
  const int nb = rv ? a.nbr[(size_t)i * a.m + r] : 0;
  const int irow = active ? i : 0;
  double xi[kDMax], xr[kDMax];
#pragma unroll
  for (int q = 0; q < kDMax; ++q) {
    xi[q] = (q < d) ? a.X[(size_t)irow * d + q] : 0.;
    xr[q] = (q < d && rv) ? a.X[(size_t)nb * d + q] : 0.;
    nbx[r * kDMax + q] = xr[q];
  }
  const bool want_like = a.Y != nullptr;
  const double yi = want_like ? a.Y[irow] : 0.;
  const double ynb = (want_like && rv) ? a.Y[nb] : 0.;

  const double var = a.var, phi = a.phi;
  const double cdiag = var * a.diag_mult + a.diag_add;
  // ---- observation-neighbour covariance c_r and its range derivative
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
  img[r * KP + r] = rv ? cdiag : 1.;
  wave_lds_sync();

  // ---- 1. between-neighbour pairs (rr > cc), each computed once, spread over the lanes
  constexpr int npairs = K * (K - 1) / 2;
  for (int p = r; p < npairs; p += K) {
    int rr = (int)((1.f + sqrtf(1.f + 8.f * (float)p)) * 0.5f);
    if (rr * (rr - 1) / 2 > p) --rr;
    if ((rr + 1) * rr / 2 <= p) ++rr;
    const int cc = p - rr * (rr - 1) / 2;
    double cv = 0., dcv = 0.;
    if (rr < k) {  // cc < rr < k
      double s = 0.;
#pragma unroll
      for (int q = 0; q < kDMax; ++q) {
        const double t = nbx[rr * kDMax + q] - nbx[cc * kDMax + q];
        s += t * t;
      }
      cov_dcov<COV>(sqrt(s), var, phi, cv, dcv);
    }
    img[rr * KP + cc] = cv;    // lower: C
    img[cc * KP + rr] = dcv;   // upper: dC
  }
  wave_lds_sync();

  // ---- 2. Cholesky C = L L^T; lane r keeps row r of L in registers
  double Lrow[K];
#pragma unroll
  for (int c = 0; c < K; ++c) Lrow[c] = (c <= r) ? img[r * KP + c] : img[c * KP + r];
  double mydiag = 1.;
#pragma unroll
  for (int j = 0; j < K; ++j) {
    const double piv = __shfl(Lrow[j], gbase + j, 64);
    const double ljj = sqrt(piv);
    const double lrj = (r > j) ? Lrow[j] / ljj : 0.;
    Lrow[j] = (r == j) ? ljj : ((r > j) ? lrj : Lrow[j]);
    mydiag = (r == j) ? ljj : mydiag;
    if (j < K - 1) {
      bcast[r] = lrj;
      wave_lds_sync();
#pragma unroll
      for (int c = j + 1; c < K; ++c) Lrow[c] = fma(-lrj, bcast[c], Lrow[c]);
      wave_lds_sync();
    }
  }
  const double invd = 1. / mydiag;

  // ---- 3a. forward solves L w = c and L w = y_nbr (registers)
  double acc1 = cvec, acc2 = ynb;
#pragma unroll
  for (int j = 0; j < K; ++j) {
    const double w1 = __shfl(acc1 * invd, gbase + j, 64);
    const double w2 = __shfl(acc2 * invd, gbase + j, 64);
    if (r > j) {
      acc1 = fma(-Lrow[j], w1, acc1);
      acc2 = fma(-Lrow[j], w2, acc2);
    }
  }
  acc1 *= invd;
  acc2 *= invd;
  // L (strictly lower part) back into the lower triangle of the image
#pragma unroll
  for (int c = 0; c < K; ++c)
    if (c < r) img[r * KP + c] = Lrow[c];
  wave_lds_sync();

  // ---- 3b. backward solves L^T x = w: lane r reads L[j][r] (column r) from LDS
  for (int j = K - 1; j >= 0; --j) {
    const double x1 = __shfl(acc1 * invd, gbase + j, 64);
    const double x2 = __shfl(acc2 * invd, gbase + j, 64);
    if (r < j) {
      const double l = img[j * KP + r];
      acc1 = fma(-l, x1, acc1);
      acc2 = fma(-l, x2, acc2);
    }
  }
  const double av_r = acc1 * invd;   // a = C^-1 c
  const double vv_r = acc2 * invd;   // v = C^-1 y_nbr

  if (active && a.B_out != nullptr && r < a.m) a.B_out[(size_t)i * a.m + r] = rv ? -av_r : 0.;

  // ---- 4. t = dC a from the upper triangle (a broadcast through LDS)
  bcast[r] = av_r;
  wave_lds_sync();
  double t = 0.;
  for (int c = 0; c < K; ++c) {
    if (c == r) continue;
    const double dcrc = (c > r) ? img[r * KP + c] : img[c * KP + r];
    t = fma(dcrc, bcast[c], t);
  }

  // ---- group reductions
  const double ac = group_sum<K>(av_r * cvec);
  const double ay = group_sum<K>(av_r * ynb);
  const double aa = group_sum<K>(av_r * av_r);
  const double avv = group_sum<K>(av_r * vv_r);
  const double dca = group_sum<K>(dcvec * av_r);
  const double dcv = group_sum<K>(dcvec * vv_r);
  const double ta = group_sum<K>(t * av_r);
  const double tv = group_sum<K>(t * vv_r);

  const double D = var + a.d_nugget - ac;          // Vecchia_utils.cpp:1351, 1507, 1562
  const double Dinv = 1. / D;
  if (active && r == 0 && a.Dinv_out != nullptr) a.Dinv_out[i] = Dinv;
  if (!want_like) return;

  double sums[kVecchiaSums] = {0., 0., 0., 0., 0., 0.};
  if (active) {
    const double delta = cdiag - var;                  // C - C_nonugget on the diagonal
    const double By = yi - ay;                         // (B y)_i
    const double u = By * Dinv;                        // (D^-1 B y)_i
    const double dD_var = var - delta * aa - ac;       // dD/dlog var
    const double uk_var = -delta * avv;                // (dB_var y)_i
    const double dD_rng = -(2. * dca - ta);            // dD/dlog phi
    const double uk_rng = -(dcv - tv);                 // (dB_range y)_i
    sums[0] = log(D);
    sums[1] = By * u;
    sums[2] = uk_var * u - 0.5 * u * u * dD_var;
    sums[3] = uk_rng * u - 0.5 * u * u * dD_rng;
    sums[4] = Dinv * dD_var;
    sums[5] = Dinv * dD_rng;
  }

  // ---- block reduction of the per-row sums (fixed order -> deterministic)
  __syncthreads();
  double* red = smem;  // reuse: rows_per_block x kVecchiaSums
  if (r == 0) {
#pragma unroll
    for (int s = 0; s < kVecchiaSums; ++s) red[group_id * kVecchiaSums + s] = sums[s];
  }
  __syncthreads();
  if (threadIdx.x < kVecchiaSums) {
    double acc = 0.;
    for (int gi = 0; gi < rows_per_block; ++gi) acc += red[gi * kVecchiaSums + threadIdx.x];
    a.block_sums[(size_t)blockIdx.x * kVecchiaSums + threadIdx.x] = acc;
  }
}

__global__ void __launch_bounds__(256) sum_blocks_kernel(const double* __restrict__ in, int nblocks, int width,
                                                       double* __restrict__ out) {
  __shared__ double red[256];
  for (int s = 0; s < width; ++s) {
    double acc = 0.;
    for (int b = threadIdx.x; b < nblocks; b += 256) acc += in[(size_t)b * width + s];
    red[threadIdx.x] = acc;
    __syncthreads();
    for (int off = 128; off > 0; off >>= 1) {
      if ((int)threadIdx.x < off) red[threadIdx.x] += red[threadIdx.x + off];
      __syncthreads();
    }
    if (threadIdx.x == 0) out[s] = red[0];
    __syncthreads();
  }
}

int lanes_for_m(int m) {
  if (m <= 16) return 16;
  if (m <= 32) return 32;
  if (m <= 64) return 64;
  return 0;
}

template <int K>
int rows_per_block() { return (block_threads<K>() / 64) * (64 / K); }

template <int K, int COV>
void launch_k(const VecchiaRowsArgs& a, hipStream_t s) {
  const int rpb = rows_per_block<K>();
  const int rows = a.r1 - a.r0;
  const int blocks = (rows + rpb - 1) / rpb;
  size_t lds = (size_t)rpb * group_lds_doubles<K>() * sizeof(double);
  const size_t red = (size_t)rpb * kVecchiaSums * sizeof(double);
  if (lds < red) lds = red;
  static bool attr_set = false;
  if (!attr_set && lds > 65536) {
    HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&vecchia_rows_kernel<K, COV>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    attr_set = true;
  }
  hipLaunchKernelGGL((vecchia_rows_kernel<K, COV>), dim3(blocks), dim3(block_threads<K>()), lds, s, a);
  HIP_CHECK(hipGetLastError());
}

template <int K>
void launch_cov(int cov, const VecchiaRowsArgs& a, hipStream_t s) {
  switch (cov) {
    case kMatern05: launch_k<K, kMatern05>(a, s); break;
    case kMatern15: launch_k<K, kMatern15>(a, s); break;
    case kMatern25: launch_k<K, kMatern25>(a, s); break;
    case kGaussian: launch_k<K, kGaussian>(a, s); break;
    default: Fatal("unsupported covariance type %d", cov);
  }
}

}  // namespace

int vecchia_rows_blocks(int rows, int m) {
  int rpb = 0;
  switch (lanes_for_m(m)) {
    case 16: rpb = rows_per_block<16>(); break;
    case 32: rpb = rows_per_block<32>(); break;
    case 64: rpb = rows_per_block<64>(); break;
    default: Fatal("num_neighbors = %d > 64 is not supported by the GPU Vecchia kernel", m);
  }
  return (rows + rpb - 1) / rpb;
}

void launch_vecchia_rows(int cov_type, const VecchiaRowsArgs& a, hipStream_t s) {
  if (a.d < 1 || a.d > kDMax) Fatal("GPU Vecchia kernel supports 1 <= dim_gp_coords <= %d, got %d", kDMax, a.d);
  if (a.r1 <= a.r0) return;
  switch (lanes_for_m(a.m)) {
    case 16: launch_cov<16>(cov_type, a, s); break;
    case 32: launch_cov<32>(cov_type, a, s); break;
    case 64: launch_cov<64>(cov_type, a, s); break;
    default: Fatal("num_neighbors = %d > 64 is not supported by the GPU Vecchia kernel", a.m);
  }
}

void launch_sum_blocks(const double* block_sums, int nblocks, int width, double* out, hipStream_t s) {
  hipLaunchKernelGGL(sum_blocks_kernel, dim3(1), dim3(256), 0, s, block_sums, nblocks, width, out);
  HIP_CHECK(hipGetLastError());
}

}  // namespace gpb_amd
