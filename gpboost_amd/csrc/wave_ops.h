// Device helpers shared by the sparse operator and triangular-solve kernels (HIP only).
//
// Wave-per-row gathers: lane r holds entry r of a row's structure (index, value), loaded by
// ONE coalesced vector load; each gather takes its entry's index and value from that lane
// with v_readlane (scalar registers). A row then costs one vector-memory instruction per
// entry instead of three (index load, value load, gather), which is what bounds the
// per-entry forms on the TA issue rate.
#pragma once

#include <hip/hip_runtime.h>

namespace gpb_amd {

// Block b runs on XCD b % 8 (round-robin dispatch): give every XCD one contiguous range of
// logical blocks, so rows stored in a locality order share gathered data in that XCD's L2.
__device__ __forceinline__ int xcd_block(int b, int G) {
  const int per = G >> 3;
  if (b >= (per << 3)) return b;
  return (b & 7) * per + (b >> 3);
}

__device__ __forceinline__ double readlane_f64(double v, int l) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), l);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), l);
  return __hiloint2double(hi, lo);
}

// s += sum_{q < cnt} w_q X[id_q * t + cc], entries in ascending q, (id_q, w_q) held by lane q
// of (my_id, my_w); cnt <= 64 and wave-uniform. Padding gathers read row `safe`.
template <int CH>
__device__ __forceinline__ double wave_dot(int my_id, double my_w, int cnt, const double* __restrict__ X, int t,
                                           int cc, int safe, double s) {
  for (int q0 = 0; q0 < cnt; q0 += CH) {
    int id[CH];
    double w[CH], g[CH];
#pragma unroll
    for (int q = 0; q < CH; ++q) {
      const bool ok = q0 + q < cnt;
      id[q] = ok ? __builtin_amdgcn_readlane(my_id, q0 + q) : safe;
      w[q] = ok ? readlane_f64(my_w, q0 + q) : 0.;
    }
#pragma unroll
    for (int q = 0; q < CH; ++q) g[q] = X[(size_t)id[q] * t + cc];
#pragma unroll
    for (int q = 0; q < CH; ++q) s = fma(w[q], g[q], s);
  }
  return s;
}

// Sum over groups of G consecutive lanes (G a power of two <= 64), result in every lane of the
// group: inside 16-lane DPP rows by VALU data movement (quad swaps, half-row and row mirrors),
// across rows through the LDS crossbar. Fixed order -> bitwise repeatable.
template <int CTRL>
__device__ __forceinline__ double dpp_move_f64(double v) {
  const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), CTRL, 0xF, 0xF, false);
  return __hiloint2double(hi, lo);
}
template <int G>
__device__ __forceinline__ double lane_group_sum(double v) {
  if constexpr (G < 16) {
#pragma unroll
    for (int off = G / 2; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
  } else {
    v += dpp_move_f64<0xB1>(v);    // quad_perm [1,0,3,2]
    v += dpp_move_f64<0x4E>(v);    // quad_perm [2,3,0,1]
    v += dpp_move_f64<0x141>(v);   // row_half_mirror
    v += dpp_move_f64<0x140>(v);   // row_mirror
    if constexpr (G >= 32) v += __shfl_xor(v, 16, 64);
    if constexpr (G >= 64) v += __shfl_xor(v, 32, 64);
    return v;
  }
}

}  // namespace gpb_amd
