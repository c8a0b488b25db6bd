// Vecchia neighbour search on the GPU.
//
// Reference replaced: find_nearest_neighbors_Vecchia_fast / _fast_internal
// (Vecchia_utils.cpp:732-1058; neighbour lists by ascending squared distance, insertion sort
// with stable ties, utils.h:245-257). The reference sweeps, for row i, the points in the order
// of their coordinate sums outward from i's position (one step down, one step up), skips
// candidates that are not earlier than i, stops a direction once (sum_c - sum_i)^2 > d * r_k^2
// and keeps the m best by insertion. That walk is serial per row but independent across rows:
// here one thread runs it for one row, with the same candidate order, the same fp64
// operations (contraction into FMA disabled, so products and sums round exactly as on the
// host) and the same insertion, so the lists are bit-identical to the host search
// (vecchia_host.cpp) and to the reference — including ties. The host computes the coordinate
// sums and the std::sort sweep order once (same code as vecchia_host.cpp).
//
// Per-thread best lists live in LDS, slot-major ([k][thread]) so a wave's accesses to slot k
// are consecutive words. Rows i <= m take all earlier points in index order (host side).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <limits>
#include <numeric>
#include <vector>

#include "common.h"
#include "vecchia_host.h"

#pragma clang fp contract(off)

namespace gpb_amd {
namespace {

constexpr int kKnnThreads = 64;
constexpr int kKnnMaxM = 64;

__global__ void __launch_bounds__(kKnnThreads) knn_kernel(const double* __restrict__ x,
                                                         const double* __restrict__ csum,
                                                         const int* __restrict__ order,
                                                         const int* __restrict__ pos, int n, int d, int m,
                                                         int r0, int r1, int last_cand, int* __restrict__ out) {
  __shared__ double bd_s[kKnnMaxM * kKnnThreads];
  __shared__ int bi_s[kKnnMaxM * kKnnThreads];
  const int tid = threadIdx.x;
  double* bd = bd_s + tid;   // slot k at bd[k * kKnnThreads]
  int* bi = bi_s + tid;
  const int i = r0 + blockIdx.x * kKnnThreads + tid;
  if (i >= r1 || i <= m) return;   // rows i <= m: all earlier points (host)
  for (int k = 0; k < m; ++k) {
    bd[k * kKnnThreads] = INFINITY;
    bi[k * kKnnThreads] = 0;
  }
  double xi[3];
  for (int q = 0; q < d; ++q) xi[q] = x[(size_t)i * d + q];
  const double si = csum[i];
  const double dd = (double)d;
  bool go_down = true, go_up = true;
  int lo = pos[i], hi = pos[i];
  double worst = INFINITY;   // bd[m - 1]
  auto visit = [&](int cand, bool& alive) {
    if (cand >= i || cand > last_cand) return;
    const double ds = csum[cand] - si;
    if (ds * ds > dd * worst) { alive = false; return; }
    double sq = 0.;
    for (int q = 0; q < d; ++q) {
      const double t = x[(size_t)cand * d + q] - xi[q];
      sq += t * t;
    }
    if (sq < worst) {
      int j = m - 1;
      // insertion from the end: shift larger entries up (same result as the swap loop)
      while (j > 0 && sq < bd[(j - 1) * kKnnThreads]) {
        bd[j * kKnnThreads] = bd[(j - 1) * kKnnThreads];
        bi[j * kKnnThreads] = bi[(j - 1) * kKnnThreads];
        --j;
      }
      bd[j * kKnnThreads] = sq;
      bi[j * kKnnThreads] = cand;
      worst = bd[(m - 1) * kKnnThreads];
    }
  };
  while (go_up || go_down) {
    if (lo == 0) go_down = false;
    if (hi == n - 1) go_up = false;
    if (go_down) visit(order[--lo], go_down);
    if (go_up) visit(order[++hi], go_up);
  }
  int* o = out + (size_t)(i - r0) * m;
  for (int k = 0; k < m; ++k) o[k] = bi[k * kKnnThreads];
}

}  // namespace

void vecchia_neighbors_gpu(const double* x, int n, int d, int m, int row_begin, int row_end, int* nbr,
                           hipStream_t s, int end_search_at) {
  const int last_cand = end_search_at < 0 ? n - 2 : end_search_at;
  if (m > kKnnMaxM) Fatal("GPU neighbour search supports num_neighbors <= %d", kKnnMaxM);
  if (d < 1 || d > 3) Fatal("GPU neighbour search supports 1 <= dim_gp_coords <= 3");
  const int rows = row_end - row_begin;
  if (rows <= 0) return;
  // coordinate sums and the sweep order: same code as the host search (utils.h:228-236)
  std::vector<double> csum(n);
  for (int i = 0; i < n; ++i) {
    double v = 0.;
    for (int q = 0; q < d; ++q) v += x[(size_t)i * d + q];
    csum[i] = v;
  }
  std::vector<int> order(n);
  std::iota(order.begin(), order.end(), 0);
  std::sort(order.begin(), order.end(), [&](int a, int b) { return csum[a] < csum[b]; });
  std::vector<int> pos(n);
  for (int i = 0; i < n; ++i) pos[order[i]] = i;
  // rows i <= m (and i = 0) on the host: all earlier points in index order, the rest -1
  for (int i = row_begin; i < row_end; ++i) {
    int* o = nbr + (size_t)(i - row_begin) * m;
    if (i <= m) {
      std::fill(o, o + m, -1);
      for (int j = 0; j < i; ++j) o[j] = j;
    }
  }
  const int g0 = std::max(row_begin, m + 1);
  if (g0 >= row_end) return;
  DevBuf<double> dx, dcs;
  DevBuf<int> dord, dpos, dout;
  dx.alloc((size_t)n * d);
  dcs.alloc(n);
  dord.alloc(n);
  dpos.alloc(n);
  dout.alloc((size_t)(row_end - g0) * m);
  HIP_CHECK(hipMemcpyAsync(dx.get(), x, sizeof(double) * (size_t)n * d, hipMemcpyHostToDevice, s));
  HIP_CHECK(hipMemcpyAsync(dcs.get(), csum.data(), sizeof(double) * n, hipMemcpyHostToDevice, s));
  HIP_CHECK(hipMemcpyAsync(dord.get(), order.data(), sizeof(int) * n, hipMemcpyHostToDevice, s));
  HIP_CHECK(hipMemcpyAsync(dpos.get(), pos.data(), sizeof(int) * n, hipMemcpyHostToDevice, s));
  const int blocks = (row_end - g0 + kKnnThreads - 1) / kKnnThreads;
  hipLaunchKernelGGL(knn_kernel, dim3(blocks), dim3(kKnnThreads), 0, s, dx.get(), dcs.get(), dord.get(), dpos.get(),
                     n, d, m, g0, row_end, last_cand, dout.get());
  HIP_CHECK(hipGetLastError());
  HIP_CHECK(hipMemcpyAsync(nbr + (size_t)(g0 - row_begin) * m, dout.get(), sizeof(int) * (size_t)(row_end - g0) * m,
                           hipMemcpyDeviceToHost, s));
  HIP_CHECK(hipStreamSynchronize(s));
}

}  // namespace gpb_amd
