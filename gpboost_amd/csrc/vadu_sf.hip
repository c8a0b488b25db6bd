// Sync-free triangular solves of the VADU preconditioner, one resident wave per CU slot.
//
// Reference replaced: the two sparse triangular solves of CGVecchiaLaplaceVec /
// CGTridiagVecchiaLaplace (CG_utils.cpp:56-60, 131-136, 181-186): B^T Y = R (unit upper),
// then Z = ((D^-1 + W) B)^-1 Y, i.e. Z_i = Y_i / dw_i - sum_r B(i, nbr_r) Z_nbr_r.
//
// The level-set form pays a kernel boundary (~1.5 us) plus the gather round trip per level
// (~400 levels per solve at n = 100k, m = 30). Here one launch per solve runs the whole DAG:
//  * Positions q (rows in the solve's level order) are dealt round-robin to a FIXED grid of
//    single-wave workgroups, all resident (grid <= CU count x waves the occupancy allows), so
//    at any time the waves work on about one level set: little polling, no deep run-ahead.
//    A wave only ever waits for smaller positions, every smaller position is owned by a
//    resident wave that reaches it, so the solve cannot deadlock.
//  * Hand-off = the value itself (MI355X_MICROARCH.md "Valid forms", 8-byte granules): the
//    output block is pre-filled with an all-ones NaN sentinel, a solved value is published by
//    one relaxed agent-scope 8-byte store (global_store sc1), every read of the output block
//    is a relaxed agent-scope load (global_load sc1). Lane = column for t >= 2 (each lane
//    waits only for its own column); lane = entry for t = 1 (fixed shuffle-tree sum).
//  * A row first polls its critical dependency (highest level: finished last), then gathers
//    all entries, re-polling any still-missing one. Sums run in entry order (t >= 2) or a
//    fixed tree (t = 1): results are bitwise reproducible.
//  * Every spin is bounded; giving up sets the error word (the host raises a Fatal error).
#include <hip/hip_runtime.h>

#include "common.h"
#include "latent_kernels.h"

namespace gpb_amd {
namespace {

constexpr unsigned long long kSentinel = ~0ull;
constexpr unsigned kSpinLimit = 1u << 16;   // ~1 us per spin: a broken DAG, not a slow one
constexpr int kSfChunk = 32;   // entries gathered per round trip (t >= 2)

__device__ __forceinline__ double poll(const double* p) {
  return __longlong_as_double(
      (long long)__hip_atomic_load(reinterpret_cast<const unsigned long long*>(p), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT));
}
__device__ __forceinline__ bool ready(double v) {
  return (unsigned long long)__double_as_longlong(v) != kSentinel;
}
// Called on every spin: gives up (and raises the error word) past the spin limit, and exits
// early once any other wave has given up, so a failure never cascades into long waits.
__device__ __forceinline__ bool give_up(unsigned& spins, int* err) {
  ++spins;
  if (spins > kSpinLimit) {
    __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return true;
  }
  if ((spins & 255u) == 0 && __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) return true;
  __builtin_amdgcn_s_sleep(1);
  return false;
}
__device__ __forceinline__ void publish(double* p, double v) {
  __hip_atomic_store(reinterpret_cast<unsigned long long*>(p), (unsigned long long)__double_as_longlong(v),
                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// row structure of position q
template <bool LOWER>
__device__ __forceinline__ void row_of(const SfArgs& a, int q, int i, const int*& idx, const double*& val, int& cnt) {
  if (LOWER) {
    idx = a.eidx + (size_t)q * a.m;
    val = a.eval + (size_t)q * a.m;
    cnt = i < a.m ? i : a.m;
  } else {
    const int e0 = a.eoff[q];
    idx = a.eidx + e0;
    val = a.eval + e0;
    cnt = a.eoff[q + 1] - e0;
  }
}

// t >= 2: lane = column c (blockIdx.y selects the 64-column chunk).
template <bool LOWER>
__global__ void __launch_bounds__(64) vadu_sf_kernel(SfArgs a) {
  const int lane = threadIdx.x;
  const int c = lane + blockIdx.y * 64;
  const int t = a.t;
  const int cc = c < t ? c : t - 1;   // lanes beyond t shadow a valid column, never publish
  double* X = a.X;
  for (int q = blockIdx.x; q < a.n; q += gridDim.x) {
    const int i = a.lrows[q];
    const int crit = a.crit[q];
    const int* idx;
    const double* val;
    int cnt;
    row_of<LOWER>(a, q, i, idx, val, cnt);
    double x = a.in[(size_t)i * t + cc];
    if (LOWER) x /= a.dw[i];
    if (crit >= 0) {   // the dependency that finishes last: one load per poll
      unsigned spins = 0;
      while (!ready(poll(X + (size_t)crit * t + cc)))
        if (give_up(spins, a.err)) return;
    }
    double acc = 0.;
    for (int b0 = 0; b0 < cnt; b0 += kSfChunk) {
      int id[kSfChunk];
      double w[kSfChunk], g[kSfChunk];
#pragma unroll
      for (int e = 0; e < kSfChunk; ++e) {
        const bool ok = b0 + e < cnt;
        id[e] = ok ? idx[b0 + e] : -1;
        w[e] = ok ? val[b0 + e] : 0.;
      }
#pragma unroll
      for (int e = 0; e < kSfChunk; ++e) g[e] = id[e] >= 0 ? poll(X + (size_t)id[e] * t + cc) : 0.;
#pragma unroll
      for (int e = 0; e < kSfChunk; ++e) {
        if (id[e] >= 0 && !ready(g[e])) {   // rare: a dependency other than crit still running
          unsigned spins = 0;
          do {
            if (give_up(spins, a.err)) return;
            g[e] = poll(X + (size_t)id[e] * t + cc);
          } while (!ready(g[e]));
        }
      }
#pragma unroll
      for (int e = 0; e < kSfChunk; ++e) acc = fma(w[e], g[e], acc);
    }
    if (c < t) publish(X + (size_t)i * t + c, x - acc);
  }
}

// t = 1: lane r = entry r of the row (rows with more than 64 entries loop over chunks).
template <bool LOWER>
__global__ void __launch_bounds__(64) vadu_sf1_kernel(SfArgs a) {
  const int lane = threadIdx.x;
  double* X = a.X;
  for (int q = blockIdx.x; q < a.n; q += gridDim.x) {
    const int i = a.lrows[q];
    const int* idx;
    const double* val;
    int cnt;
    row_of<LOWER>(a, q, i, idx, val, cnt);
    double x = a.in[i];
    if (LOWER) x /= a.dw[i];
    double acc = 0.;
    for (int b0 = 0; b0 < cnt; b0 += 64) {
      const bool ok = b0 + lane < cnt;
      double prod = 0.;
      if (ok) {
        const int j = idx[b0 + lane];
        const double w = val[b0 + lane];
        double g = poll(X + j);
        unsigned spins = 0;
        bool failed = false;
        while (!ready(g)) {
          if (give_up(spins, a.err)) { failed = true; break; }
          g = poll(X + j);
        }
        if (failed) g = 0.;
        prod = w * g;
      }
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) prod += __shfl_xor(prod, off, 64);
      acc += prod;
    }
    if (lane == 0) publish(X + i, x - acc);
  }
}

}  // namespace

void launch_vadu_sf(const SfArgs& a, bool lower, int grid, hipStream_t s) {
  if (a.n <= 0) return;
  HIP_CHECK(hipMemsetAsync(a.X, 0xFF, sizeof(double) * (size_t)a.n * a.t, s));
  const int g = grid < a.n ? grid : a.n;
  if (a.t == 1) {
    if (lower) hipLaunchKernelGGL(vadu_sf1_kernel<true>, dim3(g), dim3(64), 0, s, a);
    else hipLaunchKernelGGL(vadu_sf1_kernel<false>, dim3(g), dim3(64), 0, s, a);
  } else {
    const dim3 gr(g, (a.t + 63) / 64);
    if (lower) hipLaunchKernelGGL(vadu_sf_kernel<true>, gr, dim3(64), 0, s, a);
    else hipLaunchKernelGGL(vadu_sf_kernel<false>, gr, dim3(64), 0, s, a);
  }
  HIP_CHECK(hipGetLastError());
}

}  // namespace gpb_amd
