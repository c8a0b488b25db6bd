// Tail solves of the VADU preconditioner: one launch per merged dependency level.
//
// Reference replaced: the sparse triangular solves of P^-1 = B^-1 (D^-1 + W)^-1 B^-T
// (CG_utils.cpp:56-60, 131-136: B^T unit-upper solve, then the (D^-1 + W) B lower solve) on the
// tail rows (Vecchia index >= K, the wide part of the dependency DAG).
//   B^T solve:   X_j = R_j - sum_{i : j in nbr(i)} B(i, j) X_i
//   lower solve: X_i = Y_i / dw_i - sum_{r < k_i} B(i, nbr_r) X_{nbr_r}
// Rows of g consecutive levels form one merged level: a dependency inside the merged level is
// replaced by its own expression (recursively), so the launch reads only values of earlier merged
// levels and inputs, with coefficients c that are products of B values (latent_kernels.h,
// MergedSolve). The coefficients are refreshed once per factor by merge_numeric_kernel; each
// application then costs one launch per merged level instead of one per level — the launches,
// not the arithmetic, are what a level costs (a copy-only level kernel measured 2.8-4 us of the
// 4.1-4.9 us of a real one at n = 100k, t = 51). Fixed summation orders throughout (bitwise
// repeatable).
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <string>

#include "common.h"
#include "latent_kernels.h"
#include "wave_ops.h"

namespace gpb_amd {
namespace {

// Coefficients of the positions at one level offset (their substituted dependencies sit at lower
// offsets of the same merged level, done by earlier launches). One wave per position: the ops run
// in order, the entries of one substitution in parallel over the lanes (they map to distinct
// positions of the row's list), accumulated in LDS; lists longer than kNumericLds run on one lane
// in global memory. Same order of accumulation either way.
constexpr int kNumericLds = 512;
__global__ void __launch_bounds__(256) merge_numeric_kernel(MergedSolve ms, const int* __restrict__ plist, int cnt,
                                                            const double* __restrict__ Bv) {
  __shared__ double cbuf[4][kNumericLds];
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const int k = blockIdx.x * 4 + w;
  if (k >= cnt) return;
  const int p = plist[k];
  const int base = ms.eoff[p], len = ms.eoff[p + 1] - base;
  const int o0 = ms.opoff[p], o1 = ms.opoff[p + 1];
  if (len > kNumericLds) {   // rare: serial in global memory
    if (lane != 0) return;
    double* c = ms.eval + base;
    c[0] = 1.;
    for (int q = 1; q < len; ++q) c[q] = 0.;
    for (int o = o0; o < o1; ++o) {
      const double wt = -Bv[ms.op_slot[o]];
      const int mo = ms.op_map[o];
      if (mo < 0) {
        c[ms.op_a[o]] += wt;
      } else {
        const double* cj = ms.eval + ms.eoff[ms.op_a[o]];
        const int lj = ms.eoff[ms.op_a[o] + 1] - ms.eoff[ms.op_a[o]];
        for (int q = 0; q < lj; ++q) c[ms.map[mo + q]] = fma(wt, cj[q], c[ms.map[mo + q]]);
      }
    }
    return;
  }
  double* c = cbuf[w];
  for (int q = lane; q < len; q += 64) c[q] = q == 0 ? 1. : 0.;   // c[0]: the row's own input
  for (int o = o0; o < o1; ++o) {
    const double wt = -Bv[ms.op_slot[o]];
    const int mo = ms.op_map[o];
    if (mo < 0) {
      if (lane == 0) c[ms.op_a[o]] += wt;
    } else {
      const int pj = ms.op_a[o];
      const double* cj = ms.eval + ms.eoff[pj];
      const int lj = ms.eoff[pj + 1] - ms.eoff[pj];
      for (int q = lane; q < lj; q += 64) {
        const int at = ms.map[mo + q];
        c[at] = fma(wt, cj[q], c[at]);
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");   // this op's LDS updates before the next op's reads
  }
  for (int q = lane; q < len; q += 64) ms.eval[base + q] = c[q];
}

// t >= 2: one workgroup per row; lane = column (coalesced t-wide gathers of a dependency's row),
// wave w takes entries w, w + NW, ...; the NW partial sums meet in LDS in a fixed order.
template <int NW, int B>
__global__ void __launch_bounds__(NW * 64) merged_levelT_kernel(MergedSolve ms, const double* __restrict__ coef, int p0,
                                                                const double* in, double* X, int t) {
  __shared__ double red[NW][64];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int c = lane + blockIdx.y * 64;
  const int cc = c < t ? c : t - 1;   // lanes beyond t gather a valid column, result unused
  const int p = p0 + xcd_block(blockIdx.x, gridDim.x);
  const int i = ms.rows[p];
  const int e0 = ms.eoff[p], ex = ms.xoff[p], e1 = ms.eoff[p + 1];
  double acc = 0.;
  for (int e = e0 + wave; e < e1; e += NW * B) {
    int id[B];
    double v[B], g[B];
#pragma unroll
    for (int q = 0; q < B; ++q) {
      const int ee = min(e + q * NW, e1 - 1);
      id[q] = ms.eidx[ee];
      v[q] = (e + q * NW < e1) ? coef[ee] : 0.;
    }
#pragma unroll
    for (int q = 0; q < B; ++q) {
      const int ee = min(e + q * NW, e1 - 1);
      g[q] = (ee < ex ? in : X)[(size_t)id[q] * t + cc];
    }
#pragma unroll
    for (int q = 0; q < B; ++q) acc = fma(v[q], g[q], acc);
  }
  red[wave][lane] = acc;
  __syncthreads();
  if (wave == 0 && c < t) {
    double sum = red[0][lane];
#pragma unroll
    for (int w = 1; w < NW; ++w) sum += red[w][lane];
    X[(size_t)i * t + c] = sum;
  }
}

// t >= 2 (default form): one workgroup per row, wave w takes the chunks w, w + NW, ... of CH
// consecutive entries; a chunk's structure is ONE coalesced load per array (lane q = entry q) and
// each gather takes its entry's row and coefficient by v_readlane, so an entry costs one vector
// memory instruction (the gather, from a scalar base) instead of three. CH gathers in flight.
template <int NW, int CH>
__global__ void __launch_bounds__(NW * 64) merged_levelR_kernel(MergedSolve ms, const double* __restrict__ coef, int p0,
                                                                const double* in, double* X, int t) {
  __shared__ double red[NW][64];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int c = lane + blockIdx.y * 64;
  const int cc = c < t ? c : t - 1;   // lanes beyond t gather a valid column, result unused
  const int p = p0 + xcd_block(blockIdx.x, gridDim.x);
  const int i = ms.rows[p];
  const int e0 = ms.eoff[p], ex = ms.xoff[p], e1 = ms.eoff[p + 1];
  const int safe = ms.eidx[e0];       // padding gathers re-read the first entry's row
  double acc = 0.;
  for (int b = e0 + wave * CH; b < e1; b += NW * CH) {
    const int e = b + lane;
    const bool ok = lane < CH && e < e1;
    const int my_id = ok ? ms.eidx[e] : safe;
    const double my_w = ok ? coef[e] : 0.;
    int id[CH];
    double w[CH], g[CH];
#pragma unroll
    for (int q = 0; q < CH; ++q) {
      id[q] = __builtin_amdgcn_readlane(my_id, q);
      w[q] = readlane_f64(my_w, q);
    }
#pragma unroll
    for (int q = 0; q < CH; ++q) g[q] = (b + q < ex ? in : X)[(size_t)id[q] * t + cc];
#pragma unroll
    for (int q = 0; q < CH; ++q) acc = fma(w[q], g[q], acc);
  }
  red[wave][lane] = acc;
  __syncthreads();
  if (wave == 0 && c < t) {
    double sum = red[0][lane];
#pragma unroll
    for (int w = 1; w < NW; ++w) sum += red[w][lane];
    X[(size_t)i * t + c] = sum;
  }
}

// IN-entry coefficients of the lower solve with 1/dw folded in (per system, after SetDiag):
// coef[e] = eval[e] / dw[eidx[e]] for IN entries, eval[e] for X entries. One thread per position.
__global__ void __launch_bounds__(256) merged_scale_kernel(MergedSolve ms, const double* __restrict__ dw,
                                                           double* __restrict__ coef) {
  const int p = blockIdx.x * 256 + threadIdx.x;
  if (p >= ms.npos) return;
  const int e0 = ms.eoff[p], ex = ms.xoff[p], e1 = ms.eoff[p + 1];
  for (int e = e0; e < ex; ++e) coef[e] = ms.eval[e] / dw[ms.eidx[e]];
  for (int e = ex; e < e1; ++e) coef[e] = ms.eval[e];
}

// t >= 2, wave per row (A/B): 4 rows per 256-thread workgroup, lane = column; a chunk of up
// to 64 entries is ONE coalesced structure load (lane r = entry r) and each gather takes its
// entry's index and coefficient by v_readlane, CH gathers in flight (the operator kernels' form,
// sparse_kernels.hip). IN entries first (the lower solve folds 1/dw into their coefficients),
// then X entries, each ascending.
template <int CH>
__global__ void __launch_bounds__(256) merged_levelW_kernel(MergedSolve ms, const double* __restrict__ coef, int p0,
                                                            int cnt, const double* in, double* X, int t) {
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int r = xcd_block(blockIdx.x, gridDim.x) * 4 + wave;
  if (r >= cnt) return;
  const int p = p0 + r;
  const int i = ms.rows[p];
  const int e0 = ms.eoff[p], ex = ms.xoff[p], e1 = ms.eoff[p + 1];
  const int c = lane + blockIdx.y * 64;
  const int cc = c < t ? c : t - 1;   // lanes beyond t gather a valid column, result unused
  double s = 0.;
  for (int b0 = e0; b0 < ex; b0 += 64) {
    const int e = b0 + lane;
    const bool ok = e < ex;
    const int my_id = ok ? ms.eidx[e] : i;
    const double my_w = ok ? coef[e] : 0.;
    s = wave_dot<CH>(my_id, my_w, ex - b0 < 64 ? ex - b0 : 64, in, t, cc, i, s);
  }
  for (int b0 = ex; b0 < e1; b0 += 64) {
    const int e = b0 + lane;
    const bool ok = e < e1;
    const int my_id = ok ? ms.eidx[e] : i;
    const double my_w = ok ? coef[e] : 0.;
    s = wave_dot<CH>(my_id, my_w, e1 - b0 < 64 ? e1 - b0 : 64, X, t, cc, i, s);
  }
  if (c < t) X[(size_t)i * t + c] = s;
}

// t = 1: a row's entries are spread over a lane group (G lanes, entry e on lane e mod G), the
// group sums its lanes with a fixed tree.
template <int G>
__global__ void __launch_bounds__(256) merged_level1_kernel(MergedSolve ms, const double* __restrict__ coef, int p0,
                                                            int cnt, const double* in, double* X) {
  const int lane = threadIdx.x & (G - 1);
  const int task = xcd_block(blockIdx.x, gridDim.x) * (256 / G) + threadIdx.x / G;
  if (task >= cnt) return;   // whole groups exit together (cnt is per group)
  const int p = p0 + task;
  const int i = ms.rows[p];
  const int e0 = ms.eoff[p], ex = ms.xoff[p], e1 = ms.eoff[p + 1];
  double acc = 0.;
  for (int e = e0 + lane; e < e1; e += G) {
    const int id = ms.eidx[e];
    const double g = e < ex ? in[id] : X[id];
    acc = fma(coef[e], g, acc);
  }
  acc = lane_group_sum<G>(acc);
  if (lane == 0) X[i] = acc;
}

// Shape knobs (A/B only): GPBOOST_AMD_LEVELT_FORM = chunk (default: merged_levelR, coalesced
// structure + readlane), gather (merged_levelT: per-entry structure loads) or wave (merged_levelW,
// one wave per row); GPBOOST_AMD_LEVELT_NW = waves per row of the workgroup forms (1, 2, 4 default,
// 8); GPBOOST_AMD_LEVELT_CH = entries per chunk of the chunk form (8, 16 default, 32); GPBOOST_AMD_LEVEL1_G = lanes per row at t = 1 (16, 32 or 64; default 64). Other values:
// error.
struct LevelShape {
  int form = 0, nw = 4, ch = 16, g = 64;   // form 0 chunk, 1 gather, 2 wave
};
const LevelShape& level_shape() {
  static const LevelShape v = [] {
    LevelShape k;
    if (const char* e = std::getenv("GPBOOST_AMD_LEVELT_FORM")) {
      const std::string f(e);
      if (f == "chunk") k.form = 0;
      else if (f == "gather") k.form = 1;
      else if (f == "wave") k.form = 2;
      else Fatal("GPBOOST_AMD_LEVELT_FORM must be chunk, gather or wave (got '%s')", e);
      Info("tail level kernels: form %s", e);
    }
    if (const char* e = std::getenv("GPBOOST_AMD_LEVELT_NW")) {
      k.nw = std::atoi(e);
      if (k.nw != 1 && k.nw != 2 && k.nw != 4 && k.nw != 8)
        Fatal("GPBOOST_AMD_LEVELT_NW must be 1, 2, 4 or 8 (got '%s')", e);
      Info("tail level kernels: %d wave(s) per row at t >= 2", k.nw);
    }
    if (const char* e = std::getenv("GPBOOST_AMD_LEVELT_CH")) {
      k.ch = std::atoi(e);
      if (k.ch != 8 && k.ch != 16 && k.ch != 32) Fatal("GPBOOST_AMD_LEVELT_CH must be 8, 16 or 32 (got '%s')", e);
      Info("tail level kernels: chunks of %d entries", k.ch);
    }
    if (const char* e = std::getenv("GPBOOST_AMD_LEVEL1_G")) {
      k.g = std::atoi(e);
      if (k.g != 16 && k.g != 32 && k.g != 64) Fatal("GPBOOST_AMD_LEVEL1_G must be 16, 32 or 64 (got '%s')", e);
      Info("tail level kernels: %d lanes per row at t = 1", k.g);
    }
    return k;
  }();
  return v;
}

template <int NW>
void launch_chunk_nw(int ch, dim3 g, dim3 b, hipStream_t s, const MergedSolve& ms, const double* coef, int p0,
                     const double* in, double* X, int t) {
  if (ch == 8) hipLaunchKernelGGL((merged_levelR_kernel<NW, 8>), g, b, 0, s, ms, coef, p0, in, X, t);
  else if (ch == 32) hipLaunchKernelGGL((merged_levelR_kernel<NW, 32>), g, b, 0, s, ms, coef, p0, in, X, t);
  else hipLaunchKernelGGL((merged_levelR_kernel<NW, 16>), g, b, 0, s, ms, coef, p0, in, X, t);
}
void launch_chunk(int nw, int ch, dim3 g, dim3 b, hipStream_t s, const MergedSolve& ms, const double* coef, int p0,
                  const double* in, double* X, int t) {
  if (nw == 1) launch_chunk_nw<1>(ch, g, b, s, ms, coef, p0, in, X, t);
  else if (nw == 2) launch_chunk_nw<2>(ch, g, b, s, ms, coef, p0, in, X, t);
  else if (nw == 8) launch_chunk_nw<8>(ch, g, b, s, ms, coef, p0, in, X, t);
  else launch_chunk_nw<4>(ch, g, b, s, ms, coef, p0, in, X, t);
}

void launch_level(const MergedSolve& ms, const double* coef, int p0, int cnt, const double* in, double* X, int t,
                  hipStream_t s) {
  const LevelShape& ks = level_shape();
  if (t == 1) {
    const int G = ks.g;
    const dim3 grid((cnt + 256 / G - 1) / (256 / G));
    if (G == 16) hipLaunchKernelGGL((merged_level1_kernel<16>), grid, dim3(256), 0, s, ms, coef, p0, cnt, in, X);
    else if (G == 32) hipLaunchKernelGGL((merged_level1_kernel<32>), grid, dim3(256), 0, s, ms, coef, p0, cnt, in, X);
    else hipLaunchKernelGGL((merged_level1_kernel<64>), grid, dim3(256), 0, s, ms, coef, p0, cnt, in, X);
    return;
  }
  if (ks.form == 2) {   // wave per row: gathers in flight per batch = LEVELT_CH (16 or 32)
    if (ks.ch == 32)
      hipLaunchKernelGGL((merged_levelW_kernel<32>), dim3((cnt + 3) / 4, (t + 63) / 64), dim3(256), 0, s, ms, coef,
                         p0, cnt, in, X, t);
    else
      hipLaunchKernelGGL((merged_levelW_kernel<16>), dim3((cnt + 3) / 4, (t + 63) / 64), dim3(256), 0, s, ms, coef,
                         p0, cnt, in, X, t);
    return;
  }
  const dim3 g(cnt, (t + 63) / 64);
  const dim3 b(ks.nw * 64);
  if (ks.form == 1) {   // entries in flight per row: NW waves x B gathers (64 for every shape)
    if (ks.nw == 1) hipLaunchKernelGGL((merged_levelT_kernel<1, 64>), g, b, 0, s, ms, coef, p0, in, X, t);
    else if (ks.nw == 2) hipLaunchKernelGGL((merged_levelT_kernel<2, 32>), g, b, 0, s, ms, coef, p0, in, X, t);
    else if (ks.nw == 8) hipLaunchKernelGGL((merged_levelT_kernel<8, 8>), g, b, 0, s, ms, coef, p0, in, X, t);
    else hipLaunchKernelGGL((merged_levelT_kernel<4, 16>), g, b, 0, s, ms, coef, p0, in, X, t);
    return;
  }
  launch_chunk(ks.nw, ks.ch, g, b, s, ms, coef, p0, in, X, t);
}

// ---- persistent tail solve (TailPersist, latent_kernels.h)
//
// Grid barrier between merged levels, bounded: every wave's stores are acknowledged by L2
// (vmcnt(0)), then one thread per workgroup writes back its XCD's L2 (agent-scope release),
// counts in at its group's counter (the last of the W workgroups of a group counts in at the level
// counter) and polls the level counter until all 8 groups are in. No acquire on the way out: the
// values read after the barrier are Tp rows written once in this launch and never read before
// (their lines hold no stale copy anywhere); a foreign XCD's row misses in L2 and is fetched from
// memory, a local one is served by L2. A poll that runs out (a workgroup never became resident)
// poisons this workgroup's results with NaN, which the PCG reports, instead of hanging.
template <int REL>
__device__ __forceinline__ bool tail_grid_barrier(unsigned* ctr, int grp, int W, int* s_ok) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    if constexpr (REL == 0) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    const unsigned old = __hip_atomic_fetch_add(ctr + grp, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (old == (unsigned)W - 1) __hip_atomic_fetch_add(ctr + 8, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    int ok = 1;
    for (int spins = 0; __hip_atomic_load(ctr + 8, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < 8u;) {
      __builtin_amdgcn_s_sleep(1);
      if (++spins > (1 << 22)) {
        ok = 0;
        break;
      }
    }
    *s_ok = ok;
  }
  __syncthreads();
  return *s_ok != 0;
}

// R rows per wave (lane = column), each row's entries in ascending order into its own accumulator
// (the order of merged_levelW_kernel): a chunk of 64 entries of a row is one coalesced structure
// load, each gather takes its row and coefficient by v_readlane, and the R rows' gathers of a
// CH-entry step are issued together (R * CH in flight: the persistent grid has few waves per CU,
// so the memory parallelism has to come from within the wave). IN entries read `in`, X entries on
// tail rows Tp, other X entries (head rows of the lower solve, final before the launch) Xr.
template <int R, int CH, int REL>
__global__ void __launch_bounds__(256) tail_persist_kernel(MergedSolve ms, TailPersist tp, unsigned* ctr,
                                                           const double* __restrict__ coef, const double* in,
                                                           const double* Xr, double* Tp, double* X, int t) {
  __shared__ int s_ok;
  // lines of Tp cached by an earlier launch would be stale: drop this XCD's clean lines first
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int grp = blockIdx.x & 7;
  const int qw = (blockIdx.x >> 3) * 4 + wave;
  const int nwv = tp.W * 4;
  const int cc = lane < t ? lane : t - 1;
  bool good = true;
  for (int L = 0; L < tp.nL; ++L) {
    const int p0 = tp.lptr[L], cnt = tp.lptr[L + 1] - p0;
    const int q0 = p0 + (int)(((long)cnt * grp) >> 3), q1 = p0 + (int)(((long)cnt * (grp + 1)) >> 3);
    for (int pb = q0 + qw; pb < q1; pb += R * nwv) {
      int i[R], e0[R], ex[R], len[R];
      int lmax = 0;
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const int p = pb + r * nwv;
        const bool v = p < q1;
        i[r] = v ? ms.rows[p] : -1;
        e0[r] = v ? ms.eoff[p] : 0;
        ex[r] = v ? ms.xoff[p] : 0;
        len[r] = v ? ms.eoff[p + 1] - e0[r] : 0;
        lmax = max(lmax, len[r]);
      }
      double s[R];
#pragma unroll
      for (int r = 0; r < R; ++r) s[r] = 0.;
      for (int b = 0; b < (tp.diag == 2 ? 0 : lmax); b += 64) {
        int my_id[R];
        double my_w[R];
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const bool ok = b + lane < len[r];
          my_id[r] = ok ? tp.eidx_p[e0[r] + b + lane] : 0;
          my_w[r] = ok ? coef[e0[r] + b + lane] : 0.;
        }
        const int nb = min(64, lmax - b);
        for (int c0 = 0; c0 < nb; c0 += CH) {
          double w[R][CH], g[R][CH];
#pragma unroll
          for (int r = 0; r < R; ++r) {
#pragma unroll
            for (int q = 0; q < CH; ++q) {
              const int k = b + c0 + q;   // entry k of row r
              const bool okq = k < len[r];
              const int id = __builtin_amdgcn_readlane(my_id[r], okq ? c0 + q : 0);
              w[r][q] = okq ? readlane_f64(my_w[r], c0 + q) : 0.;
              const double* src = !okq                 ? in
                                  : e0[r] + k < ex[r]  ? in + (size_t)id * t
                                  : (id & kTailBit)    ? Tp + (size_t)(id & ~kTailBit) * kTailPad
                                                       : Xr + (size_t)id * t;
              g[r][q] = src[cc];
            }
          }
#pragma unroll
          for (int r = 0; r < R; ++r) {
#pragma unroll
            for (int q = 0; q < CH; ++q) s[r] = fma(w[r][q], g[r][q], s[r]);
          }
        }
      }
#pragma unroll
      for (int r = 0; r < R; ++r) {
        if (i[r] < 0) continue;
        const double v = good ? s[r] : __builtin_nan("");
        if (lane < t) {
          // REL 1: written through to memory (agent-scope store), no L2 write-back at the barrier
          if constexpr (REL == 1) __hip_atomic_store(Tp + (size_t)i[r] * kTailPad + lane, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          else Tp[(size_t)i[r] * kTailPad + lane] = v;
          X[(size_t)i[r] * t + lane] = v;
        }
      }
    }
    if (L + 1 < tp.nL && tp.diag != 1) good = tail_grid_barrier<REL>(ctr + (size_t)L * 9, grp, tp.W, &s_ok) && good;
  }
}

}  // namespace

int tail_persist_max_w() {
  static int w = -1;
  if (w < 0) {
    int dev = 0, cus = 0, per_cu = 0;
    HIP_CHECK(hipGetDevice(&dev));
    HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    // the grid barriers need every workgroup resident: take the lowest occupancy over all the
    // instantiations GPBOOST_AMD_TAIL_RCH / _REL can select
    per_cu = 1 << 30;
    auto occ = [&](const void* k) {
      int v = 0;
      HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&v, k, 256, 0));
      per_cu = std::min(per_cu, v);
    };
    occ((const void*)tail_persist_kernel<4, 8, 0>);
    occ((const void*)tail_persist_kernel<4, 8, 1>);
    occ((const void*)tail_persist_kernel<2, 16, 0>);
    occ((const void*)tail_persist_kernel<2, 16, 1>);
    occ((const void*)tail_persist_kernel<8, 4, 0>);
    occ((const void*)tail_persist_kernel<8, 4, 1>);
    occ((const void*)tail_persist_kernel<8, 8, 0>);
    occ((const void*)tail_persist_kernel<8, 8, 1>);
    w = (cus % 8 == 0) ? (per_cu * cus) / 8 : 0;
  }
  return w;
}

void launch_tail_persist(const MergedSolve& ms, const TailPersist& tp, unsigned* counters, const double* coef,
                         const double* in, const double* Xr, double* Tp, double* X, int t, hipStream_t s) {
  if (tp.nL <= 0 || t <= 0) return;
  if (t > kTailPad) Fatal("persistent tail solve: %d columns > %d", t, kTailPad);
  if (tp.W < 1 || tp.W > tail_persist_max_w()) Fatal("persistent tail solve: %d workgroups per XCD not resident", tp.W);
  HIP_CHECK(hipMemsetAsync(counters, 0, sizeof(unsigned) * 9 * (size_t)tp.nL, s));
  // A/B: GPBOOST_AMD_TAIL_REL 0 = L2 write-back at the barrier, 1 = stores written through (default);
  // GPBOOST_AMD_TAIL_RCH = rows per wave x gathers per row step: 4x8 (default), 2x16, 8x4, 8x8
  static const int rel = [] {
    const char* e = std::getenv("GPBOOST_AMD_TAIL_REL");
    return e ? std::atoi(e) : 1;
  }();
  static const std::string rch = [] {
    const char* e = std::getenv("GPBOOST_AMD_TAIL_RCH");
    const std::string v = e ? e : "4x8";
    if (v != "4x8" && v != "2x16" && v != "8x4" && v != "8x8") Fatal("GPBOOST_AMD_TAIL_RCH must be 4x8, 2x16, 8x4 or 8x8");
    return v;
  }();
  const dim3 g(8 * tp.W), b(256);
#define GPB_TAIL_LAUNCH(R, CH)                                                                                   \
  do {                                                                                                          \
    if (rel == 0) hipLaunchKernelGGL((tail_persist_kernel<R, CH, 0>), g, b, 0, s, ms, tp, counters, coef, in, Xr, Tp, X, t); \
    else hipLaunchKernelGGL((tail_persist_kernel<R, CH, 1>), g, b, 0, s, ms, tp, counters, coef, in, Xr, Tp, X, t);      \
  } while (0)
  if (rch == "2x16") GPB_TAIL_LAUNCH(2, 16);
  else if (rch == "8x4") GPB_TAIL_LAUNCH(8, 4);
  else if (rch == "8x8") GPB_TAIL_LAUNCH(8, 8);
  else GPB_TAIL_LAUNCH(4, 8);
#undef GPB_TAIL_LAUNCH
  HIP_CHECK(hipGetLastError());
}

void launch_merged_numeric(const MergedSolve& ms, const double* Bv, hipStream_t s) {
  for (size_t o = 0; o + 1 < ms.offptr.size(); ++o) {
    const int cnt = ms.offptr[o + 1] - ms.offptr[o];
    if (cnt <= 0) continue;
    hipLaunchKernelGGL(merge_numeric_kernel, dim3((cnt + 3) / 4), dim3(256), 0, s, ms, ms.offpos + ms.offptr[o], cnt,
                       Bv);
  }
  HIP_CHECK(hipGetLastError());
}

void launch_merged_scale(const MergedSolve& ms, const double* dw, double* coef, hipStream_t s) {
  if (ms.npos <= 0) return;
  hipLaunchKernelGGL(merged_scale_kernel, dim3((ms.npos + 255) / 256), dim3(256), 0, s, ms, dw, coef);
  HIP_CHECK(hipGetLastError());
}

void launch_merged_level(const MergedSolve& ms, int L, const double* coef, const double* in, double* X, int t,
                         hipStream_t s) {
  const int p0 = ms.lptr[L], cnt = ms.lptr[L + 1] - p0;
  if (cnt <= 0 || t <= 0) return;
  launch_level(ms, coef, p0, cnt, in, X, t, s);
  HIP_CHECK(hipGetLastError());
}

}  // namespace gpb_amd
