// LDS segment kernel and partial-sum kernels of the VADU triangular solves (vadu_precond.cpp).
//
// Reference replaced: the two sparse triangular solves of the VADU preconditioner
// P^-1 = B^-1 (D^-1 + W)^-1 B^-T (CG_utils.cpp:56-60, likelihoods.h:11963-12041 and the
// Lanczos variant CG_utils.cpp:110-217).
//
// Why: in a random Vecchia ordering the dependency DAG is thin at its early end — row i
// depends on its m nearest EARLIER points, which for small i are spread over the whole
// domain. At n = 100k, m = 30 the first 12288 Vecchia rows already span ~280 of the 388
// dependency levels, with ~44 rows per level; the remaining 88% of the rows fit in ~110
// wide levels. One launch per level (launch_vadu_level, ~4.9 us each at t = 51) is pure
// latency on the thin part. Here ONE workgroup per column solves the whole head with that
// column's head values resident in LDS: a level costs an LDS gather + a workgroup barrier,
// and the next pass's structure (global) is loaded while the current one computes.
//
// The rows handled here are Vecchia rows [K0, K) ("head 1"); the first K0 rows are solved by the
// dense block of vadu_dense.hip, and every dependency outside the segment is folded into the
// segment's input beforehand by vadu_partial_kernel, so the kernel itself is direction-agnostic.
//
// Row arithmetic is the reference's: x_i = in_i (/ dw_i) - sum_e v_e x_{idx_e}; the entries
// are split over G = 16 lanes (lane l: entries l, l+16, ...) and combined by a fixed xor
// tree, so repeated runs are bitwise identical.
#include <hip/hip_runtime.h>

#include "common.h"
#include "latent_kernels.h"
#include "wave_ops.h"

namespace gpb_amd {
namespace {

constexpr int kHeadThreads = kHeadRowsPerPass * kHeadG;

// LDS writes of this wave done, then the workgroup barrier. Global accesses are left in
// flight on purpose (prefetched structure; result stores nobody reads inside the launch),
// which a __syncthreads() (workgroup release: vmcnt(0)) would drain.
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// Sum over each slot of kHeadG lanes, result in every lane of the slot: quad swaps, then the
// half-row (and row) mirrors (VALU data movement instead of LDS-crossbar shuffles on the pass's
// critical chain). Fixed order -> bitwise repeatable.
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v) {
  const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), CTRL, 0xF, 0xF, false);
  return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double slot_sum(double v) {
  static_assert(kHeadG == 8 || kHeadG == 16, "a slot is one half or one whole 16-lane DPP row");
  v += dpp_f64<0xB1>(v);    // quad_perm [1,0,3,2]
  v += dpp_f64<0x4E>(v);    // quad_perm [2,3,0,1]
  v += dpp_f64<0x141>(v);   // row_half_mirror: 8-lane sums
  if constexpr (kHeadG == 16) v += dpp_f64<0x140>(v);   // row_mirror
  return v;
}

// Stage of one pass on this thread: its record and this lane's EPL fixed-layout entries.
// Every address is a function of the pass index alone (no dependent loads), so the next
// pass's stage is in flight while this one gathers from LDS; the loop is unrolled by two so
// the stages alternate between two register sets (a copy would force a wait).
template <int EPL>
struct Stage {
  int pend;            // the pass ends its level: workgroup barrier after it
  int rec;             // see HeadSolve (latent_kernels.h)
  int id[EPL];
  double v[EPL];
};

template <int EPL>
__device__ __forceinline__ void load_stage(const HeadSolve& h, int q, int slot, int lane, Stage<EPL>& st) {
  const int r = q * kHeadRowsPerPass + slot;
  st.pend = h.pend[q];
  st.rec = h.rec[r];
#pragma unroll
  for (int k = 0; k < EPL; ++k) {
    const size_t e = ((size_t)r * EPL + k) * kHeadG + lane;
    st.id[k] = h.eidx[e];
    st.v[k] = h.eval[e];
  }
}

// A row spans 1, 2 or 4 slots (kHeadG << lg lanes); group lane gl = sub * kHeadG + lane holds its
// entries gl + k * GL (k < EPL), then overflow entries [ooff[r0], ooff[r0 + 1]) in steps of GL.
template <int EPL>
__device__ __forceinline__ void solve_row(const HeadSolve& h, const Stage<EPL>& st, int q, int slot, int lane,
                                          double* xs) {
  const int lg = (st.rec >> 16) & 3, sub = (st.rec >> 18) & 3;
  double acc = 0.;
#pragma unroll
  for (int k = 0; k < EPL; ++k) acc = fma(st.v[k], xs[st.id[k]], acc);
  if (st.rec < 0) {   // long row: overflow entries
    const int r0 = q * kHeadRowsPerPass + slot - sub;
    const int GL = kHeadG << lg;
    for (int e = h.ooff[r0] + sub * kHeadG + lane; e < h.ooff[r0 + 1]; e += GL) acc = fma(h.oval[e], xs[h.oidx[e]], acc);
  }
  acc = slot_sum(acc);
  if (__ballot(lg >= 1)) {   // wave-uniform: only waves holding a multi-slot row pay the cross-slot steps
    // partner slot: the other half of the 16-lane DPP row (row_mirror) for 8-lane slots
    const double o1 = kHeadG == 8 ? dpp_f64<0x140>(acc) : __shfl_xor(acc, kHeadG, 64);
    if (lg >= 1) acc += o1;
    if (__ballot(lg >= 2)) {
      const double o2 = __shfl_xor(acc, 2 * kHeadG, 64);
      if (lg >= 2) acc += o2;
    }
  }
  if (lane == 0 && sub == 0) xs[st.rec & 0xffff] -= acc;
}

template <int EPL, int NS>
__global__ void __launch_bounds__(kHeadThreads) vadu_head_kernel(HeadSolve h, int t, const double* in,
                                                                 const double* __restrict__ dw, double* X) {
  extern __shared__ double xs[];   // this column's segment values by slot; slot K = scratch
  const int c = blockIdx.x;
  const int lane = threadIdx.x & (kHeadG - 1);
  const int slot = threadIdx.x / kHeadG;
  // inputs of all segment rows first (independent loads): in (/ dw when given)
  constexpr int kPer = (kHeadMaxRows + kHeadThreads - 1) / kHeadThreads;
  {   // all loads of the phase in flight at once (no loop-carried wait)
    int r[kPer];
    double x[kPer], w[kPer];
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
      const int v = threadIdx.x + k * kHeadThreads;
      r[k] = h.hrow[v < h.K ? v : 0];
    }
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
      x[k] = in[(size_t)r[k] * t + c];
      w[k] = dw ? dw[r[k]] : 1.;
    }
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
      const int v = threadIdx.x + k * kHeadThreads;
      if (v < h.K) xs[v] = dw ? x[k] / w[k] : x[k];
    }
  }
  if (threadIdx.x == 0) xs[h.K] = 0.;
  __syncthreads();
  const int last = h.npass - 1;
  // NS stages in flight: pass q + NS's structure is loaded while pass q solves (a pass is a few
  // hundred cycles of LDS work, a structure load an L2 / Infinity-Cache round trip of more)
  Stage<EPL> st[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) load_stage<EPL>(h, min(s, last), slot, lane, st[s]);
  for (int q = 0; q < h.npass; q += NS) {
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      if (q + s <= last) {   // workgroup-uniform
        solve_row<EPL>(h, st[s], q + s, slot, lane, xs);
        // rows of one level are independent: only a level's last pass needs the barrier (a
        // workgroup-uniform flag, so every wave takes the same barriers)
        const int pend = __builtin_amdgcn_readfirstlane(st[s].pend);
        load_stage<EPL>(h, min(q + s + NS, last), slot, lane, st[s]);
        if (pend) lds_barrier();
      }
    }
  }
  // results out after the loop: a global store inside it would make the compiler drain the
  // prefetch (its registers are reused by the next stage's loads)
  __syncthreads();
  int r[kPer];
#pragma unroll
  for (int k = 0; k < kPer; ++k) {
    const int v = threadIdx.x + k * kHeadThreads;
    r[k] = h.hrow[v < h.K ? v : 0];
  }
#pragma unroll
  for (int k = 0; k < kPer; ++k) {
    const int v = threadIdx.x + k * kHeadThreads;
    if (v < h.K) X[(size_t)r[k] * t + c] = xs[v];
  }
}

// ---- one-wave segment solve (SegWave, latent_kernels.h)
//
// Why one wave: the per-pass cost of vadu_head_kernel (1024 threads) was its sixteen waves each
// running the whole pass code (gather, four DPP stages, the row write) between workgroup barriers,
// ~0.55 us per pass. Here the pass is one wave's stream: up to kSegSteps LDS gathers and FMAs per
// lane, a DPP reduction over the row's lane group and one LDS write, with no barrier (a wave's LDS
// operations complete in order). The other three waves of the workgroup only stage the segment
// into LDS and write it back.
constexpr int kSegThreads = 256;

struct SegStage {
  int rec;
  int id[kSegSteps];
  double v[kSegSteps];
};

__device__ __forceinline__ void seg_load(const SegWave& w, int4 m, int lane, SegStage& st) {
  st.rec = w.rec[(size_t)m.w * 64 + lane];   // m.w: the pass index (set by seg_meta)
  const size_t base = (size_t)m.x * 64 + lane;
#pragma unroll
  for (int k0 = 0; k0 < kSegSteps; k0 += 8) {
    if (k0 < m.y) {   // wave-uniform
#pragma unroll
      for (int k = k0; k < k0 + 8; ++k) {
        st.id[k] = w.eidx[base + (size_t)k * 64];
        st.v[k] = w.eval[base + (size_t)k * 64];
      }
    }
  }
}

__device__ __forceinline__ int4 seg_meta(const SegWave& w, int q) {
  int4 m = w.meta[q];
  m.w = q;
  return m;
}

// sum over the row's lane group of 2^lg lanes (lg wave-uniform), every lane of the group gets it
__device__ __forceinline__ double seg_group_sum(double v, int lg) {
  if (lg >= 1) v += dpp_f64<0xB1>(v);    // quad_perm [1,0,3,2]
  if (lg >= 2) v += dpp_f64<0x4E>(v);    // quad_perm [2,3,0,1]
  if (lg >= 3) v += dpp_f64<0x141>(v);   // row_half_mirror
  if (lg >= 4) v += dpp_f64<0x140>(v);   // row_mirror
  if (lg >= 5) v += __shfl_xor(v, 16, 64);
  if (lg >= 6) v += __shfl_xor(v, 32, 64);
  return v;
}

template <int NS>
__global__ void __launch_bounds__(kSegThreads) vadu_seg_wave_kernel(SegWave w, int t, const double* in,
                                                                    const double* __restrict__ dw, double* X) {
  extern __shared__ double xs[];   // this column's segment values by slot; slot K = 0 (padding target)
  const int c = blockIdx.x;
  for (int v = threadIdx.x; v < w.K; v += kSegThreads) {
    const int r = w.hrow[v];
    const double x = in[(size_t)r * t + c];
    xs[v] = dw ? x / dw[r] : x;
  }
  if (threadIdx.x == 0) xs[w.K] = 0.;
  __syncthreads();
  if (threadIdx.x < 64 && w.npass > 0) {
    const int lane = threadIdx.x;
    const char* xb = reinterpret_cast<const char*>(xs);
    const int last = w.npass - 1;
    SegStage st[NS];
    int4 m[NS];
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      m[s] = seg_meta(w, min(s, last));
      seg_load(w, m[s], lane, st[s]);
    }
    for (int q = 0; q <= last; q += NS) {
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        if (q + s <= last) {   // wave-uniform
          const int L = m[s].y, lg = m[s].z;
          double a0 = 0., a1 = 0., a2 = 0., a3 = 0.;
#pragma unroll
          for (int k0 = 0; k0 < kSegSteps; k0 += 8) {
            if (k0 < L) {   // steps k0..k0+7 (padding entries beyond L hold a zero coefficient)
              double g[8];
#pragma unroll
              for (int k = 0; k < 8; ++k)
                g[k] = *reinterpret_cast<const double*>(xb + st[s].id[k0 + k]);
              a0 = fma(st[s].v[k0 + 0], g[0], a0);
              a1 = fma(st[s].v[k0 + 1], g[1], a1);
              a2 = fma(st[s].v[k0 + 2], g[2], a2);
              a3 = fma(st[s].v[k0 + 3], g[3], a3);
              a0 = fma(st[s].v[k0 + 4], g[4], a0);
              a1 = fma(st[s].v[k0 + 5], g[5], a1);
              a2 = fma(st[s].v[k0 + 6], g[6], a2);
              a3 = fma(st[s].v[k0 + 7], g[7], a3);
            }
          }
          const double acc = seg_group_sum((a0 + a1) + (a2 + a3), lg);
          const int rec = st[s].rec;
          if (rec >= 0) xs[rec] = -acc;
          // the next pass's gathers stay behind this write in program order (LDS is in order per wave)
          asm volatile("" ::: "memory");
          m[s] = seg_meta(w, min(q + s + NS, last));
          seg_load(w, m[s], lane, st[s]);
        }
      }
    }
  }
  __syncthreads();
  for (int v = threadIdx.x; v < w.K; v += kSegThreads) X[(size_t)w.hrow[v] * t + c] = xs[v];
}

// Partial sums of the dependencies outside a solve step, for every listed row r:
//   out[r] = (in ? in[r] / (dw ? dw[r] : 1) : out[r]) - sum_e eval[e] src[eidx[e]]
// (entries in list order). t >= 2: one wave per row, lane = column, the row's structure by one
// coalesced load and v_readlane broadcasts; t = 1: 16 lanes per row over its entries.
__global__ void __launch_bounds__(256) vadu_partial_kernel(PartialList p, const double* in,
                                                           const double* __restrict__ dw, const double* src,
                                                           double* out, int t, double* compact, int ncompact) {
  const int lane = threadIdx.x & 63;
  const int w = blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (w >= p.rows) return;
  const int j = p.row[w];
  const int c = lane + blockIdx.y * 64;
  const int cc = c < t ? c : t - 1;
  const int e0 = p.eoff[w], e1 = p.eoff[w + 1];
  double x = in ? in[(size_t)j * t + cc] : out[(size_t)j * t + cc];
  if (dw) x /= dw[j];
  double acc = 0.;
  for (int b0 = e0; b0 < e1; b0 += 64) {
    const int e = b0 + lane;
    const bool ok = e < e1;
    const int my_id = ok ? p.eidx[e] : j;
    const double my_w = ok ? p.eval[e] : 0.;
    const int cnt = e1 - b0 < 64 ? e1 - b0 : 64;
    acc = wave_dot<16>(my_id, my_w, cnt, src, t, cc, j, acc);
  }
  if (c < t) {
    out[(size_t)j * t + c] = x - acc;
    if (w < ncompact) compact[(size_t)w * t + c] = x - acc;
  }
}

__global__ void __launch_bounds__(256) vadu_partial1_kernel(PartialList p, const double* in,
                                                            const double* __restrict__ dw, const double* src,
                                                            double* out, double* compact, int ncompact) {
  const int g = blockIdx.x * 16 + (threadIdx.x >> 4), gl = threadIdx.x & 15;
  if (g >= p.rows) return;   // whole 16-lane groups exit together
  const int j = p.row[g];
  double acc = 0.;
  for (int e = p.eoff[g] + gl; e < p.eoff[g + 1]; e += 16) acc = fma(p.eval[e], src[p.eidx[e]], acc);
  acc = lane_group_sum<16>(acc);
  if (gl == 0) {
    double x = in ? in[j] : out[j];
    if (dw) x /= dw[j];
    out[j] = x - acc;
    if (g < ncompact) compact[g] = x - acc;
  }
}

}  // namespace

// Structure stages in flight in the segment kernel (GPBOOST_AMD_HEAD_NS = 2, 4 or 6; default 4).
int head_stages() {
  static const int v = [] {
    int k = 4;
    if (const char* e = std::getenv("GPBOOST_AMD_HEAD_NS")) {
      k = std::atoi(e);
      if (k != 2 && k != 4 && k != 6) Fatal("GPBOOST_AMD_HEAD_NS must be 2, 4 or 6 (got '%s')", e);
    }
    return k;
  }();
  return v;
}

void launch_vadu_head(const HeadSolve& h, const double* in, const double* dw, double* X, int t, hipStream_t s) {
  if (h.npass <= 0 || t <= 0) return;
  const size_t lds = sizeof(double) * ((size_t)h.K + 1);
  const int ns = head_stages();
  if (ns == 2)
    hipLaunchKernelGGL((vadu_head_kernel<kHeadEpl, 2>), dim3(t), dim3(kHeadThreads), lds, s, h, t, in, dw, X);
  else if (ns == 6)
    hipLaunchKernelGGL((vadu_head_kernel<kHeadEpl, 6>), dim3(t), dim3(kHeadThreads), lds, s, h, t, in, dw, X);
  else
    hipLaunchKernelGGL((vadu_head_kernel<kHeadEpl, 4>), dim3(t), dim3(kHeadThreads), lds, s, h, t, in, dw, X);
  HIP_CHECK(hipGetLastError());
}

void launch_vadu_partial(const PartialList& p, const double* in, const double* dw, const double* src, double* out,
                         int t, hipStream_t s, double* compact, int ncompact) {
  if (p.rows <= 0 || t <= 0) return;
  if (!compact) ncompact = 0;
  if (t == 1)
    hipLaunchKernelGGL(vadu_partial1_kernel, dim3((p.rows + 15) / 16), dim3(256), 0, s, p, in, dw, src, out, compact,
                       ncompact);
  else
    hipLaunchKernelGGL(vadu_partial_kernel, dim3((p.rows + 3) / 4, (t + 63) / 64), dim3(256), 0, s, p, in, dw, src,
                       out, t, compact, ncompact);
  HIP_CHECK(hipGetLastError());
}

// Structure stages in flight in the one-wave segment kernel (GPBOOST_AMD_SEG_NS = 1, 2 or 3; default 2).
int seg_stages() {
  static const int v = [] {
    int k = 2;
    if (const char* e = std::getenv("GPBOOST_AMD_SEG_NS")) {
      k = std::atoi(e);
      if (k < 1 || k > 3) Fatal("GPBOOST_AMD_SEG_NS must be 1, 2 or 3 (got '%s')", e);
    }
    return k;
  }();
  return v;
}

void launch_vadu_seg_wave(const SegWave& w, const double* in, const double* dw, double* X, int t, hipStream_t s) {
  if (w.K <= 0 || t <= 0) return;
  const size_t lds = sizeof(double) * ((size_t)w.K + 1);
  const int ns = seg_stages();
  if (ns == 1)
    hipLaunchKernelGGL((vadu_seg_wave_kernel<1>), dim3(t), dim3(kSegThreads), lds, s, w, t, in, dw, X);
  else if (ns == 3)
    hipLaunchKernelGGL((vadu_seg_wave_kernel<3>), dim3(t), dim3(kSegThreads), lds, s, w, t, in, dw, X);
  else
    hipLaunchKernelGGL((vadu_seg_wave_kernel<2>), dim3(t), dim3(kSegThreads), lds, s, w, t, in, dw, X);
  HIP_CHECK(hipGetLastError());
}

// The limit is per kernel function, not per model: always the largest head any model may use,
// so a later model with a smaller K cannot lower it under an earlier model's launches.
void set_vadu_head_lds_limit(int K) {
  if (K > kHeadMaxRows) Fatal("LDS segment of %d rows exceeds the LDS capacity (%d)", K, kHeadMaxRows);
  const int bytes = (int)(sizeof(double) * ((size_t)kHeadMaxRows + 1));
  for (const void* f : {(const void*)vadu_head_kernel<kHeadEpl, 2>, (const void*)vadu_head_kernel<kHeadEpl, 4>,
                        (const void*)vadu_head_kernel<kHeadEpl, 6>, (const void*)vadu_seg_wave_kernel<1>,
                        (const void*)vadu_seg_wave_kernel<2>, (const void*)vadu_seg_wave_kernel<3>})
    HIP_CHECK(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, bytes));
}

}  // namespace gpb_amd
