// VADU preconditioner application on gfx950: Z = P^-1 R, P = B^T (D^-1 + W) B
// (reference CGVecchiaLaplaceVec / CGTridiagVecchiaLaplace, CG_utils.cpp:56-60, 131-136:
// B^T unit-upper solve, then the (D^-1 + W) B lower solve, one column at a time).
//
// The two solves are sequences of dependent level sets (~390 levels each at n = 100k,
// m = 30), so the cost is latency, not bandwidth. One workgroup owns one column and walks
// all steps of both solves with a workgroup barrier between steps: no per-level launches
// and no inter-CU synchronisation. Per step each thread owns one row; its entries (index,
// value) come from LDS, so the only global-memory round trip on the critical path is the
// gather of already-solved values (the column's vectors stay in L2). The next step's blob
// is copied global -> LDS with global_load_lds (no VGPR staging) while the current step
// computes, into the other half of a double buffer; the barrier's vmcnt(0) wait orders it.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#include "common.h"
#include "latent_kernels.h"
#include "wave_ops.h"

namespace gpb_amd {
namespace {

constexpr int kThreads = kSweepRows;
constexpr int kChunk = 32;   // gathers in flight per thread (a typical row needs one round trip)

typedef __attribute__((address_space(3))) void lds_void;

// Copy `words` 32-bit words from global src to LDS dst (both word aligned) with the
// direct-to-LDS load path; every wave copies 64-word slices (LDS dst = base + lane * 4).
template <bool DMA>
__device__ __forceinline__ void stage_async(const int* __restrict__ src, int* dst, int words) {
  if (words <= 0) return;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  constexpr int kWaves = kThreads / 64;
  for (int base = wave * 64; base < words; base += kWaves * 64) {
    const int w = base + lane < words ? base + lane : words - 1;   // clamp: stays in-bounds
    if constexpr (DMA) __builtin_amdgcn_global_load_lds(src + w, (lds_void*)(dst + base), 4, 0, 0);
    else dst[base + lane] = src[w];
  }
}

__device__ __forceinline__ int sweep_column(int t) {
  // blocks are dispatched round-robin over the 8 XCDs: give each XCD a contiguous range of
  // columns so that neighbouring columns share row-major cache lines in its L2
  const int cpx = (t + 7) / 8;
  return (blockIdx.x & 7) * cpx + (blockIdx.x >> 3);
}

__device__ unsigned long long g_sweep_prof[8];

template <bool DMA, int MODE>
__global__ void __launch_bounds__(kThreads) vadu_sweep_kernel(SweepPlan plan, const double* __restrict__ dw,
                                                              const double* R, double* Y, double* Z, int t) {
  unsigned long long tp[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  unsigned long long t0 = 0;
  extern __shared__ __attribute__((aligned(16))) int lds[];
  const int c = sweep_column(t);
  if (c >= t) return;
  const int tid = threadIdx.x;
  const int W = plan.max_words;
  // every blob starts with its header (kSweepHdr words): rows, entries, values offset,
  // own size, next blob's size, phase; all step metadata travels with the staged blob
  int off = 0;
  stage_async<DMA>(plan.blob, lds, plan.first_words);
  for (int s = 0; s < plan.nsteps; ++s) {
    if (MODE == 4) t0 = __builtin_amdgcn_s_memrealtime();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // step s staged, previous stores done
    if (MODE == 4) { unsigned long long t1 = __builtin_amdgcn_s_memrealtime(); tp[0] += t1 - t0; t0 = t1; }
    __syncthreads();
    if (MODE == 4) { unsigned long long t1 = __builtin_amdgcn_s_memrealtime(); tp[1] += t1 - t0; t0 = t1; }
    const int* buf = lds + (s & 1) * W;
    const int rows = buf[0], ents = buf[1], v0 = buf[2], words = buf[3], next_words = buf[4];
    const bool lower = buf[5] != 0;
    if (MODE < 3 || MODE == 4) stage_async<DMA>(plan.blob + off + words, lds + ((s + 1) & 1) * W, next_words);
    if (MODE == 4) { unsigned long long t1 = __builtin_amdgcn_s_memrealtime(); tp[2] += t1 - t0; t0 = t1; }
    off += words;
    const double* X = lower ? Z : Y;     // vector being solved for
    double* out = lower ? Z : Y;
    const double* in = lower ? Y : R;
    if ((MODE < 2 || MODE == 4) && tid < rows) {
      const int i = buf[kSweepHdr + tid];
      const int e0 = buf[kSweepHdr + rows + tid], e1 = buf[kSweepHdr + rows + tid + 1];
      const double* vals = reinterpret_cast<const double*>(buf + v0);
      const int* idx = buf + v0 + 2 * ents;
      double x = in[(size_t)i * t + c];
      const double d = lower ? dw[i] : 1.;
      double acc = 0.;
      for (int e = e0; e < e1; e += kChunk) {
        // branch-free chunk: all LDS reads, then all gathers, then the FMAs (padding lanes
        // re-read the last entry and contribute 0)
        int id[kChunk];
        double v[kChunk], g[kChunk];
#pragma unroll
        for (int q = 0; q < kChunk; ++q) {
          const int ee = min(e + q, e1 - 1);
          id[q] = idx[ee];
          v[q] = (e + q < e1) ? vals[ee] : 0.;
        }
#pragma unroll
        for (int q = 0; q < kChunk; ++q) g[q] = (MODE == 0 || MODE == 4) ? X[(size_t)id[q] * t + c] : 0.;
        if (MODE == 4) { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); unsigned long long t1 = __builtin_amdgcn_s_memrealtime(); tp[3] += t1 - t0; t0 = t1; }
#pragma unroll
        for (int q = 0; q < kChunk; ++q) acc = fma(v[q], g[q], acc);
      }
      out[(size_t)i * t + c] = x / d - acc;
      if (MODE == 4) { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); unsigned long long t1 = __builtin_amdgcn_s_memrealtime(); tp[4] += t1 - t0; t0 = t1; }
    }
  }
  if (MODE == 4 && tid == 0 && blockIdx.x == 0)
    for (int q = 0; q < 5; ++q) g_sweep_prof[q] += tp[q];
}

// One level of either solve; T lanes (columns) per row, rows of the level over all blocks.
// Per row: the structure loads (one round trip), then every gather of already-solved values
// issued together (one round trip), then the store.
template <int CH>
__device__ __forceinline__ double level_dot(const int* __restrict__ idx, const double* __restrict__ val, int cnt,
                                            const double* X, int t, int c) {
  double acc = 0.;
  for (int e = 0; e < cnt; e += CH) {
    int id[CH];
    double v[CH], g[CH];
#pragma unroll
    for (int q = 0; q < CH; ++q) {
      const int ee = min(e + q, cnt - 1);
      id[q] = idx[ee];
      v[q] = (e + q < cnt) ? val[ee] : 0.;
    }
#pragma unroll
    for (int q = 0; q < CH; ++q) g[q] = X[(size_t)id[q] * t + c];
#pragma unroll
    for (int q = 0; q < CH; ++q) acc = fma(v[q], g[q], acc);
  }
  return acc;
}


template <bool LOWER, bool EMPTY>
__global__ void __launch_bounds__(256) vadu_level_kernel(LevelPlan lp, int p0, int cnt, const double* __restrict__ dw,
                                                         const double* in, double* X, int t, int shift) {
  const int T = 1 << shift;
  const int c = (threadIdx.x & (T - 1)) + blockIdx.y * 64;
  const int task = blockIdx.x * (256 >> shift) + (threadIdx.x >> shift);
  if (task >= cnt || c >= t) return;
  const int p = p0 + task;
  const int i = lp.lrows[p];
  if (EMPTY) {   // timing experiment: no gathers
    X[(size_t)i * t + c] = in[(size_t)i * t + c];
    return;
  }
  double acc;
  if (LOWER) {
    const size_t q = (size_t)(p - lp.n) * lp.m;
    acc = level_dot<32>(lp.fidx + q, lp.fval + q, lp.m, X, t, c);
  } else {
    const int e0 = lp.beoff[p], e1 = lp.beoff[p + 1];
    acc = e1 > e0 ? level_dot<32>(lp.beidx + e0, lp.beval + e0, e1 - e0, X, t, c) : 0.;
  }
  double x = in[(size_t)i * t + c];
  if (LOWER) x /= dw[i];
  X[(size_t)i * t + c] = x - acc;
}

__global__ void sweep_values_kernel(int count, const int* __restrict__ vpos, const int* __restrict__ eslot,
                                    const double* __restrict__ Bv, double* __restrict__ blob) {
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < count; e += gridDim.x * blockDim.x)
    blob[vpos[e]] = Bv[eslot[e]];
}

}  // namespace

void launch_vadu_sweep(const SweepPlan& plan, const double* dw, const double* R, double* Y, double* Z, int t,
                       hipStream_t s) {
  if (plan.nsteps <= 0) return;
  const int grid = 8 * ((t + 7) / 8);
  const size_t lds = (size_t)2 * plan.max_words * sizeof(int);
  static const bool dma = std::getenv("GPBOOST_AMD_SWEEP_NODMA") == nullptr;
  static const int mode = std::getenv("GPBOOST_AMD_SWEEP_MODE") ? std::atoi(std::getenv("GPBOOST_AMD_SWEEP_MODE")) : 0;
  static size_t lds_attr = 0;   // dynamic LDS above 64 KB must be opted into per kernel
  auto kern = [&]() -> const void* {
    switch (mode) {
      case 1: return reinterpret_cast<const void*>(dma ? vadu_sweep_kernel<true, 1> : vadu_sweep_kernel<false, 1>);
      case 2: return reinterpret_cast<const void*>(dma ? vadu_sweep_kernel<true, 2> : vadu_sweep_kernel<false, 2>);
      case 3: return reinterpret_cast<const void*>(dma ? vadu_sweep_kernel<true, 3> : vadu_sweep_kernel<false, 3>);
      case 4: return reinterpret_cast<const void*>(dma ? vadu_sweep_kernel<true, 4> : vadu_sweep_kernel<false, 4>);
      default: return reinterpret_cast<const void*>(dma ? vadu_sweep_kernel<true, 0> : vadu_sweep_kernel<false, 0>);
    }
  }();
  if (lds > lds_attr) {
    HIP_CHECK(hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    lds_attr = lds;
  }
  void* args[] = {const_cast<SweepPlan*>(&plan), &dw, &R, &Y, &Z, &t};
  HIP_CHECK(hipLaunchKernel(kern, dim3(grid), dim3(kThreads), args, lds, s));
  if (mode == 4) {
    static int calls = 0;
    if (++calls % 50 == 0) {
      unsigned long long h[8];
      HIP_CHECK(hipStreamSynchronize(s));
      HIP_CHECK(hipMemcpyFromSymbol(h, HIP_SYMBOL(g_sweep_prof), sizeof(h)));
      std::fprintf(stderr, "[sweep prof] calls=%d t=%d steps=%d  wait=%llu bar=%llu stage=%llu gather=%llu store=%llu (100MHz ticks, per call)\n",
                   calls, t, plan.nsteps, h[0] / calls, h[1] / calls, h[2] / calls, h[3] / calls, h[4] / calls);
    }
  }
  HIP_CHECK(hipGetLastError());
}

// t = 1: a row's entries are spread over a lane group (G lanes, entry e on lane e mod G),
// so a level's gathers are one instruction per row and the structure loads are coalesced;
// the group then sums its lanes with a fixed shuffle tree (deterministic).
template <bool LOWER, int G>
__global__ void __launch_bounds__(256) vadu_level1_kernel(LevelPlan lp, int p0, int cnt,
                                                          const double* __restrict__ dw, const double* in,
                                                          double* X) {
  const int lane = threadIdx.x & (G - 1);
  const int task = xcd_block(blockIdx.x, gridDim.x) * (256 / G) + threadIdx.x / G;
  if (task >= cnt) return;   // whole groups exit together (cnt is per group)
  const int p = p0 + task;
  const int i = lp.lrows[p];
  double acc = 0.;
  if (LOWER) {
    const size_t q = (size_t)(p - lp.n) * lp.m;
    for (int e = lane; e < lp.m; e += G) acc = fma(lp.fval[q + e], X[lp.fidx[q + e]], acc);
  } else {
    const int e0 = lp.beoff[p], e1 = lp.beoff[p + 1];
    for (int e = e0 + lane; e < e1; e += G) acc = fma(lp.beval[e], X[lp.beidx[e]], acc);
  }
  acc = lane_group_sum<G>(acc);
  if (lane == 0) {
    double x = in[i];
    if (LOWER) x /= dw[i];
    X[i] = x - acc;
  }
}

// t >= 2: one workgroup per row; lane = column (coalesced t-wide gathers of a neighbour's
// row), wave w takes entries w, w + NW, ...; the NW partial sums meet in LDS in a fixed order.
template <bool LOWER, int NW>
__global__ void __launch_bounds__(NW * 64) vadu_levelT_kernel(LevelPlan lp, int p0, const double* __restrict__ dw,
                                                              const double* in, double* X, int t) {
  __shared__ double red[NW][64];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int c = lane + blockIdx.y * 64;
  const int p = p0 + xcd_block(blockIdx.x, gridDim.x);
  const int i = lp.lrows[p];
  int e0, e1;
  const int* idx;
  const double* val;
  if (LOWER) {
    const size_t q = (size_t)(p - lp.n) * lp.m;
    idx = lp.fidx + q;
    val = lp.fval + q;
    e0 = 0;
    e1 = lp.m;
  } else {
    idx = lp.beidx;
    val = lp.beval;
    e0 = lp.beoff[p];
    e1 = lp.beoff[p + 1];
  }
  const int cc = c < t ? c : t - 1;   // lanes beyond t gather a valid column, result unused
  // the row's own input is loaded up front, next to the structure loads (no extra round trip)
  double x = 0.;
  if (wave == 0) {
    x = in[(size_t)i * t + cc];
    if (LOWER) x /= dw[i];
  }
  constexpr int B = 16;
  double acc = 0.;
  for (int e = e0 + wave; e < e1; e += NW * B) {
    int id[B];
    double v[B], g[B];
#pragma unroll
    for (int q = 0; q < B; ++q) {
      const int ee = min(e + q * NW, e1 - 1);
      id[q] = idx[ee];
      v[q] = (e + q * NW < e1) ? val[ee] : 0.;
    }
#pragma unroll
    for (int q = 0; q < B; ++q) g[q] = X[(size_t)id[q] * t + cc];
#pragma unroll
    for (int q = 0; q < B; ++q) acc = fma(v[q], g[q], acc);
  }
  red[wave][lane] = acc;
  __syncthreads();
  if (wave == 0 && c < t) {
    double sum = red[0][lane];
#pragma unroll
    for (int w = 1; w < NW; ++w) sum += red[w][lane];
    X[(size_t)i * t + c] = x - sum;
  }
}

// t >= 2, wave-per-row: one 64-lane workgroup per row (lane = column), the row's structure
// loaded by one coalesced load (lane r = entry r) and broadcast to the gathers by v_readlane,
// all of a typical row's gathers in flight at once (CH = 32). Summation: entries ascending.
template <bool LOWER, int CH>
__global__ void __launch_bounds__(64) vadu_levelW_kernel(LevelPlan lp, int p0, const double* __restrict__ dw,
                                                        const double* in, double* X, int t) {
  const int lane = threadIdx.x;
  const int p = p0 + xcd_block(blockIdx.x, gridDim.x);
  const int i = lp.lrows[p];
  const int c = lane + blockIdx.y * 64;
  const int cc = c < t ? c : t - 1;   // lanes beyond t gather a valid column, result unused
  const int* idx;
  const double* val;
  int cnt;
  if (LOWER) {
    const size_t q = (size_t)(p - lp.n) * lp.m;
    idx = lp.fidx + q;
    val = lp.fval + q;
    cnt = i < lp.m ? i : lp.m;
  } else {
    const int e0 = lp.beoff[p];
    idx = lp.beidx + e0;
    val = lp.beval + e0;
    cnt = lp.beoff[p + 1] - e0;
  }
  double x = in[(size_t)i * t + cc];
  if (LOWER) x /= dw[i];
  double acc = 0.;
  for (int b0 = 0; b0 < cnt; b0 += 64) {
    const int nb = cnt - b0 < 64 ? cnt - b0 : 64;
    const bool ok = lane < nb;
    const int my_id = ok ? idx[b0 + lane] : 0;
    const double my_w = ok ? val[b0 + lane] : 0.;
    acc = wave_dot<CH>(my_id, my_w, nb, X, t, cc, __builtin_amdgcn_readlane(my_id, 0), acc);
  }
  if (c < t) X[(size_t)i * t + c] = x - acc;
}

void launch_vadu_level(const LevelPlan& lp, int l, const double* dw, const double* R, double* Y, double* Z, int t,
                       hipStream_t s) {
  int T = 1, shift = 0;
  const int tc = t < 64 ? t : 64;
  while (T < tc) { T <<= 1; ++shift; }
  const int p0 = lp.lptr[l], cnt = lp.lptr[l + 1] - p0;
  if (cnt <= 0) return;
  if (t == 1 && std::getenv("GPBOOST_AMD_LEVEL_T1_OLD") == nullptr) {
    static const int g_env = std::getenv("GPBOOST_AMD_LEVEL1_G") ? std::atoi(std::getenv("GPBOOST_AMD_LEVEL1_G")) : 0;
    if (l < lp.nlev_b) {
      if (g_env == 32) {
        constexpr int G = 32;
        hipLaunchKernelGGL((vadu_level1_kernel<false, G>), dim3((cnt + 256 / G - 1) / (256 / G)), dim3(256), 0, s,
                           lp, p0, cnt, dw, R, Y);
      } else {
        constexpr int G = 64;
        hipLaunchKernelGGL((vadu_level1_kernel<false, G>), dim3((cnt + 256 / G - 1) / (256 / G)), dim3(256), 0, s,
                           lp, p0, cnt, dw, R, Y);
      }
    } else {
      if (g_env == 16) {
        constexpr int G = 16;
        hipLaunchKernelGGL((vadu_level1_kernel<true, G>), dim3((cnt + 256 / G - 1) / (256 / G)), dim3(256), 0, s,
                           lp, p0, cnt, dw, Y, Z);
      } else {
        constexpr int G = 32;
        hipLaunchKernelGGL((vadu_level1_kernel<true, G>), dim3((cnt + 256 / G - 1) / (256 / G)), dim3(256), 0, s,
                           lp, p0, cnt, dw, Y, Z);
      }
    }
    return;
  }
  // Level form for t >= 2 (GPBOOST_AMD_LEVEL_FORM): 1 (default) = vadu_levelT_kernel (4 waves
  // share a row's entries); 0 / 2 = wave-per-row with 32 / 16 gathers in flight, measured
  // slower on MI355X at n = 100k, t = 51 (7.2 / 7.4 ms against 4.66 ms per application).
  static const int lform = std::getenv("GPBOOST_AMD_LEVEL_FORM") ? std::atoi(std::getenv("GPBOOST_AMD_LEVEL_FORM")) : 1;
  if (lform == 0 || lform == 2) {
    const dim3 g(cnt, (t + 63) / 64);
    if (lform == 0) {
      if (l < lp.nlev_b) hipLaunchKernelGGL((vadu_levelW_kernel<false, 32>), g, dim3(64), 0, s, lp, p0, dw, R, Y, t);
      else hipLaunchKernelGGL((vadu_levelW_kernel<true, 32>), g, dim3(64), 0, s, lp, p0, dw, Y, Z, t);
    } else {
      if (l < lp.nlev_b) hipLaunchKernelGGL((vadu_levelW_kernel<false, 16>), g, dim3(64), 0, s, lp, p0, dw, R, Y, t);
      else hipLaunchKernelGGL((vadu_levelW_kernel<true, 16>), g, dim3(64), 0, s, lp, p0, dw, Y, Z, t);
    }
    return;
  }
  if (std::getenv("GPBOOST_AMD_LEVEL_T_OLD") == nullptr) {
    const dim3 g(cnt, (t + 63) / 64);
    // waves sharing a row's entries: lower rows (m fixed entries) 2 waves — measured at
    // n = 100k, t = 51: lower tail 0.506 -> 0.428 ms vs 4 waves; B^T rows (variable, some
    // long) 4 waves (2 waves: 0.518 vs 0.510 ms). GPBOOST_AMD_LEVELT_NW forces one value.
    static const int nw_env = std::getenv("GPBOOST_AMD_LEVELT_NW") ? std::atoi(std::getenv("GPBOOST_AMD_LEVELT_NW")) : 0;
    const bool lower = l >= lp.nlev_b;
    const int nw = nw_env ? nw_env : (lower ? 2 : 4);
    if (nw == 1) {
      if (!lower)
        hipLaunchKernelGGL((vadu_levelT_kernel<false, 1>), g, dim3(64), 0, s, lp, p0, dw, R, Y, t);
      else
        hipLaunchKernelGGL((vadu_levelT_kernel<true, 1>), g, dim3(64), 0, s, lp, p0, dw, Y, Z, t);
      return;
    }
    if (nw == 2) {
      if (!lower)
        hipLaunchKernelGGL((vadu_levelT_kernel<false, 2>), g, dim3(128), 0, s, lp, p0, dw, R, Y, t);
      else
        hipLaunchKernelGGL((vadu_levelT_kernel<true, 2>), g, dim3(128), 0, s, lp, p0, dw, Y, Z, t);
      return;
    }
    if (!lower)
      hipLaunchKernelGGL((vadu_levelT_kernel<false, 4>), g, dim3(256), 0, s, lp, p0, dw, R, Y, t);
    else
      hipLaunchKernelGGL((vadu_levelT_kernel<true, 4>), g, dim3(256), 0, s, lp, p0, dw, Y, Z, t);
    return;
  }
  const int rpb = 256 >> shift;
  const dim3 grid((cnt + rpb - 1) / rpb, (t + 63) / 64);
  static const bool empty = std::getenv("GPBOOST_AMD_LEVEL_EMPTY") != nullptr;
  if (empty)
    hipLaunchKernelGGL((vadu_level_kernel<false, true>), grid, dim3(256), 0, s, lp, p0, cnt, dw, R, Y, t, shift);
  else if (l < lp.nlev_b)
    hipLaunchKernelGGL((vadu_level_kernel<false, false>), grid, dim3(256), 0, s, lp, p0, cnt, dw, R, Y, t, shift);
  else
    hipLaunchKernelGGL((vadu_level_kernel<true, false>), grid, dim3(256), 0, s, lp, p0, cnt, dw, Y, Z, t, shift);
}

void launch_sweep_values(int count, const int* vpos, const int* eslot, const double* Bv, int* blob, hipStream_t s) {
  if (count <= 0) return;
  int g = (count + 255) / 256;
  if (g > 4096) g = 4096;
  hipLaunchKernelGGL(sweep_values_kernel, dim3(g), dim3(256), 0, s, count, vpos, eslot, Bv,
                     reinterpret_cast<double*>(blob));
  HIP_CHECK(hipGetLastError());
}

}  // namespace gpb_amd
