// Sync-free ("dataflow") triangular solves of the VADU preconditioner on gfx950.
//
// Reference replaced: the two sparse triangular solves of CGVecchiaLaplaceVec /
// CGTridiagVecchiaLaplace (CG_utils.cpp:56-60, 131-136): B^T Y = R (unit upper), then
// Z = ((D^-1 + W) B)^-1 Y, i.e. Z_i = Y_i / dw_i - sum_r B(i, nbr_r) Z_nbr_r.
//
// Why not one launch per level: at n = 100k, m = 30 each solve has ~400 dependent level
// sets of ~250 rows; a kernel boundary costs ~1.5-1.9 us plus the gathers' round trip, so
// the level form is latency-bound at ~5 us per level. Here ONE launch per solve runs the
// whole DAG: every lane is an independent state machine for one (row, column) pair of the
// solve, and each solved value is its own readiness flag.
//
//  * Handoff (MI355X_MICROARCH.md "Valid forms", R2 granules): the output block X is
//    filled with the all-ones bit pattern (a NaN no arithmetic produces) before the launch;
//    a finished value is published with ONE 8-byte relaxed agent-scope atomic store
//    (global_store sc1, write-through) and every read of X in the launch is a relaxed
//    agent-scope atomic load (global_load sc1). A lane re-polls only the entries of its
//    chunk that still read as the sentinel, then sums the chunk in index order (the
//    summation order is fixed, so results are bitwise reproducible).
//  * Work assignment: positions p in the solve's level order are dealt round-robin to lane
//    groups (one group of T = pow2 >= min(t, 64) lanes per row, lane = column). All
//    dependencies of p have smaller positions, and every workgroup is resident (the grid is
//    capped at 2 blocks per CU), so the smallest unfinished (p, column) can always proceed:
//    no deadlock. A lane never waits for another lane of its own wave, because each lane
//    steps its own state machine (the wave loops until all its lanes are finished).
//  * Every spin is bounded: a lane that polls one chunk more than kSpinLimit times writes
//    the error word and gives up (the host turns that into a Fatal error).
#include <hip/hip_runtime.h>

#include "common.h"
#include "latent_kernels.h"

namespace gpb_amd {
namespace {

constexpr int kFlowThreads = 256;
constexpr int kFlowChunk = 32;                    // entries polled per round trip
constexpr unsigned kSpinLimit = 1u << 22;         // ~seconds of polling: a broken DAG, not a slow one
constexpr int kFlowInflightRows = 2048;         // rows (lane groups) in flight per column chunk
constexpr unsigned long long kSentinel = ~0ull;   // all-ones: a NaN that arithmetic never produces

__device__ __forceinline__ unsigned long long poll_load(const unsigned long long* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void publish(unsigned long long* p, double v) {
  __hip_atomic_store(p, (unsigned long long)__double_as_longlong(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <bool LOWER, bool PROF>
__global__ void __launch_bounds__(kFlowThreads) vadu_flow_kernel(FlowArgs a) {
  const int lane = threadIdx.x & 63;
  const int T = 1 << a.shift;
  const int c = (lane & (T - 1)) + blockIdx.y * 64;
  if (c >= a.t) return;
  const int G = 64 >> a.shift;
  const int gwave = blockIdx.x * (kFlowThreads / 64) + (threadIdx.x >> 6);
  const int stride = gridDim.x * (kFlowThreads / 64) * G;
  const int t = a.t;
  unsigned long long* X = reinterpret_cast<unsigned long long*>(a.X);

  int q = gwave * G + (lane >> a.shift);   // position within this solve
  int i = 0, k = 0, e0 = 0, cnt = 0, crit = -1;
  const int* ip = nullptr;
  const double* vp = nullptr;
  double x = 0., acc = 0.;
  unsigned mask = 0, full = 0, spins = 0;
  bool have = false;
  int id[kFlowChunk];
  double w[kFlowChunk], v[kFlowChunk];
  while (q < a.n) {
    if (!have) {   // set up row p = q: structure pointers, own input, its critical dependency
      i = a.lrows[q];
      crit = a.crit[q];
      if (LOWER) {
        k = i < a.m ? i : a.m;
        ip = a.eidx + (size_t)q * a.m;
        vp = a.eval + (size_t)q * a.m;
        x = a.in[(size_t)i * t + c] / a.dw[i];
      } else {
        const int b0 = a.eoff[q];
        k = a.eoff[q + 1] - b0;
        ip = a.eidx + b0;
        vp = a.eval + b0;
        x = a.in[(size_t)i * t + c];
      }
      acc = 0.;
      e0 = 0;
      have = true;
      cnt = -1;
      if (PROF && c == 0) a.prof[(size_t)q * 4 + 0] = __builtin_amdgcn_s_memrealtime();
    }
    bool progress;
    if (crit >= 0) {   // one load per poll until the last-finishing dependency has arrived
      progress = poll_load(X + (size_t)crit * t + c) != kSentinel;
      if (progress) {
        crit = -1;
        if (PROF && c == 0) a.prof[(size_t)q * 4 + 1] = __builtin_amdgcn_s_memrealtime();
      }
    } else {
      if (cnt < 0) {   // new chunk: its structure, then one load per entry
        cnt = k - e0 < kFlowChunk ? k - e0 : kFlowChunk;
        full = cnt == 32 ? ~0u : ((1u << cnt) - 1u);
        mask = 0;
#pragma unroll
        for (int e = 0; e < kFlowChunk; ++e) {
          id[e] = e < cnt ? ip[e0 + e] : 0;
          w[e] = e < cnt ? vp[e0 + e] : 0.;
        }
      }
#pragma unroll
      for (int e = 0; e < kFlowChunk; ++e) {
        if (e < cnt && !(mask & (1u << e))) {
          const unsigned long long u = poll_load(X + (size_t)id[e] * t + c);
          v[e] = __longlong_as_double((long long)u);
          if (u != kSentinel) mask |= 1u << e;
        }
      }
      progress = mask == full;
      if (progress) {
#pragma unroll
        for (int e = 0; e < kFlowChunk; ++e)
          if (e < cnt) acc = fma(w[e], v[e], acc);
        e0 += cnt;
        cnt = -1;
        if (e0 >= k) {
          publish(X + (size_t)i * t + c, x - acc);
          if (PROF && c == 0) a.prof[(size_t)q * 4 + 2] = __builtin_amdgcn_s_memrealtime();
          q += stride;
          have = false;
        }
      }
    }
    if (progress) {
      spins = 0;
    } else {
      if (++spins > kSpinLimit) {
        __hip_atomic_store(a.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return;
      }
      __builtin_amdgcn_s_sleep(2);
    }
  }
}

}  // namespace

void launch_vadu_flow(const FlowArgs& a0, bool lower, int max_blocks, hipStream_t s) {
  if (a0.n <= 0) return;
  FlowArgs a = a0;
  int T = 1, shift = 0;
  const int tc = a.t < 64 ? a.t : 64;
  while (T < tc) { T <<= 1; ++shift; }
  a.shift = shift;
  const int gy = (a.t + 63) / 64;
  const int rows_per_block = (kFlowThreads / 64) * (64 >> shift);
  int gx = (a.n + rows_per_block - 1) / rows_per_block;
  int cap = max_blocks / gy > 0 ? max_blocks / gy : 1;   // every block resident
  // rows in flight: a few levels ahead of the frontier is enough; more only adds polling
  const int inflight_cap = (kFlowInflightRows + rows_per_block - 1) / rows_per_block;
  if (cap > inflight_cap) cap = inflight_cap;
  if (gx > cap) gx = cap;
  HIP_CHECK(hipMemsetAsync(a.X, 0xFF, sizeof(double) * (size_t)a.n * a.t, s));
  if (a.prof) {
    if (lower)
      hipLaunchKernelGGL((vadu_flow_kernel<true, true>), dim3(gx, gy), dim3(kFlowThreads), 0, s, a);
    else
      hipLaunchKernelGGL((vadu_flow_kernel<false, true>), dim3(gx, gy), dim3(kFlowThreads), 0, s, a);
  } else if (lower) {
    hipLaunchKernelGGL((vadu_flow_kernel<true, false>), dim3(gx, gy), dim3(kFlowThreads), 0, s, a);
  } else {
    hipLaunchKernelGGL((vadu_flow_kernel<false, false>), dim3(gx, gy), dim3(kFlowThreads), 0, s, a);
  }
  HIP_CHECK(hipGetLastError());
}

}  // namespace gpb_amd
