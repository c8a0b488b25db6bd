// Vecchia factor + likelihood/gradient rows, 16-lane form (m <= 30), gfx950.
//
// Same row math as vecchia_rows_kernel's bordered form (vecchia_kernels.hip; reference:
// CalcCovFactorGradientVecchia Vecchia_utils.cpp:1307-1632 fused with re_model_template.h:8885-9120,
// 1768-1791), laid out so the Gauss-Jordan broadcasts never touch LDS: one row problem (the 32 x 32
// bordered matrix [[C, c, y_nbr], [c^T ...], [y_nbr^T ...]], 30 pivots) per 16-lane DPP row, lane h
// holding matrix rows h and h + 16. Column j of the current matrix is row j by symmetry, and row c's
// entry sits in lane c mod 16 (register set c / 16), so one row_newbcast DPP move (a single 64-bit
// VALU op) hands M[j][c] to the 16 lanes of the problem, where it feeds TWO FMAs (rows h, h + 16).
// Four problems per wave, one per DPP row. The 32-lane form broadcasts every value through an LDS
// slot (a 16-byte read per two values per lane): at 2 waves/SIMD its LDS return traffic, not the FP64
// VALU, set the pace.
//   1. a 31-point circulant over the 30 neighbours and the row's own point (slot 30 = lane 14's second
//      slot): slot v pairs with (v + delta) mod 31, delta = 1..15, so the 465 pairs are each evaluated
//      once (30 kernel evaluations per lane; slot 30's pairs are the border column c). Coordinates in
//      LDS with copies of slots 0..15 at 31..46 (partner v + delta is an immediate-offset read). C to
//      the packed lower triangle, dC/dlog(phi) in registers until the rows are loaded, then over the
//      packed C in the circulant layout W[(delta - 1) 32 + v];
//   2. rows h and h + 16 of the bordered matrix into registers; 30 Gauss-Jordan steps by DPP
//      broadcasts (pivots 16..29 on the B rows only, the A rows finished by one block
//      back-substitution); a_v = M[v][30] / M[v][v], w_v = M[v][31] / M[v][v] (the pivots are captured
//      when broadcast);
//   3. a^T dC a and w^T dC a over each lane's circulant pairs ([a, w] pairs with the same wrap copies);
//   4. the eight group sums by DPP within the 16-lane row, then the six row partials.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <type_traits>

#include "common.h"
#include "cov.h"
#include "kernels.h"

namespace gpb_amd {
namespace {

constexpr int kD3 = 3;   // coordinate dimension bound (VecchiaRowsArgs.d <= 3)
// broadcasts in flight per elimination step (1, 2 or 4): 1 / 2 / 4 measured 0.2193 / 0.2176 / 0.2162 ms
// per launch (profiles/r03/rows_ab_r03o.log, rows_ab_r03p.log)
#ifndef GPB_ROWS16_BCG
#define GPB_ROWS16_BCG 4
#endif
// broadcasts folded into v_fmac_f64_dpp (1, default) vs separate DPP moves + FMAs (0): 0.1968 vs
// 0.2140 ms per launch, 4835 vs 4483 evals/s (profiles/r04/round_r04c.log)
#ifndef GPB_ROWS16_FMAC
#define GPB_ROWS16_FMAC 1
#endif
// pivots 16..29 eliminate only the B rows (h + 16); the A rows' solution is completed by one block
// back-substitution x_A -= M_AB x_B afterwards (28 instead of 119 fused broadcasts per problem)
#ifndef GPB_ROWS16_BACKSUB
#define GPB_ROWS16_BACKSUB 1
#endif

__device__ __forceinline__ void lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
__device__ __forceinline__ void cfence() { asm volatile("" ::: "memory"); }

template <int CTRL>
__device__ __forceinline__ double dpp32x2(double v) {   // all controls used have a source lane for every lane
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), CTRL, 0xF, 0xF, true);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), CTRL, 0xF, 0xF, true);
  return __hiloint2double(hi, lo);
}

template <int L>
__device__ __forceinline__ double bcast16(double v) {   // lane L of each 16-lane row, to the whole row
  const long b = __builtin_amdgcn_mov_dpp(__builtin_bit_cast(long, v), 0x150 + L, 0xF, 0xF, true);
  return __builtin_bit_cast(double, b);
}

// acc += (src of lane L of the 16-lane row) * mul, one instruction. NOP: the VALU-write -> DPP-read
// wait states (2) emitted inside the same asm statement, so no compiler-scheduled VALU op can land
// between them and the DPP read (the hazard recognizer does not see into inline asm). The first
// broadcast of every sequence whose source was just written carries them; tests/test_isa_hazards.py
// disassembles the built kernels and checks every DPP source against the preceding VALU writes.
template <int L, bool NOP = false>
__device__ __forceinline__ void fmac_bcast16(double& acc, double src, double mul) {
  if constexpr (NOP)
    asm volatile("s_nop 1\n\tv_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf"
                 : "+v"(acc)
                 : "v"(src), "v"(mul), "n"(L));
  else
    asm volatile("v_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf"
                 : "+v"(acc)
                 : "v"(src), "v"(mul), "n"(L));
}

__device__ __forceinline__ double sum16(double v) {   // fixed-order sum over the 16-lane row
  v += dpp32x2<0xB1>(v);    // quad_perm [1,0,3,2]
  v += dpp32x2<0x4E>(v);    // quad_perm [2,3,0,1]
  v += dpp32x2<0x141>(v);   // row_half_mirror
  v += dpp32x2<0x140>(v);   // row_mirror
  return v;
}

__device__ __forceinline__ double recip(double x) {   // hardware reciprocal + two Newton steps (~1 ulp)
  double r = __builtin_amdgcn_rcp(x);
  r = fma(r, fma(-x, r, 1.), r);
  return fma(r, fma(-x, r, 1.), r);
}

template <int B, int E, class F>
__device__ __forceinline__ void sfor(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    sfor<B + 1, E>(f);
  }
}

__device__ __forceinline__ int tri(int x) { return x * (x + 1) / 2; }

constexpr int kK = 32, kMK = 30;
constexpr int kPacked = kK * (kK + 1) / 2;   // 528

template <int CS>
constexpr int problem_doubles() { return kPacked + 48 * CS; }   // packed C (then dC) | 48 coordinate rows

template <int COV, int DIM>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2, 2))) vecchia_rows16_kernel(VecchiaRowsArgs a) {
  constexpr int ND = DIM > 0 ? DIM : kD3;
  constexpr int CS = ND;
  constexpr int PD = problem_doubles<CS>();
  static_assert(PD % 2 == 0, "16-byte aligned problems");
  typedef double v2d __attribute__((ext_vector_type(2)));
  extern __shared__ __attribute__((aligned(16))) double smem[];
  const int lane = threadIdx.x;
  const int g = lane >> 4;
  double* Cp = smem + g * PD;
  double* nbx = Cp + kPacked;
  const double var = a.var, phi = a.phi;
  const double cdiag = var * a.diag_mult + a.diag_add;
  const double delta = cdiag - var;
  const bool want_like = a.Y != nullptr;
  const int d = DIM > 0 ? DIM : a.d;

  // the row partials accumulate in LDS (4 problems x 6 doubles after the problems' areas): a register
  // accumulator would be live across the elimination, where the registers run out
  double* acc = smem + 4 * PD + g * kVecchiaSums;
  if ((lane & 15) < kVecchiaSums) acc[lane & 15] = 0.;
  const int total = a.r1 - a.r0;
  // problem sets (4 rows) over the G waves: full rounds w + it G; the last round's E sets either on
  // waves 0..E-1 (sched 0/2) or spread evenly over the grid (sched 1), so its waves do not crowd the
  // first SIMDs the dispatcher fills
  const int nsets = (total + 3) / 4, G = gridDim.x, w = blockIdx.x;
  const int R = (nsets + G - 1) / G, E = nsets - (R - 1) * G;
  int last_set = (R - 1) * G + w;
  if (a.sched == 1) {
    const long lo = (long)w * E / G, hi = (long)(w + 1) * E / G;
    last_set = hi > lo ? (R - 1) * G + (int)lo : nsets;
  }
  for (int it = 0; it < R; ++it) {
    const int set = it + 1 < R ? it * G + w : last_set;
    if (set >= nsets) break;
    const int base = set * 4;
    int h = lane & 15;
    asm volatile("" : "+v"(h));   // lane-dependent addresses / masks recomputed per problem (not hoisted)
    const int v1 = h + 16;
    const int i = a.r0 + base + g;
    const bool active = i < a.r1;
    const int k = active ? min(i, a.m) : 0;
    const bool rv0 = h < k, rv1 = v1 < k;
    const int irow = active ? i : a.r0;

    // ---- gather (rows h and h + 16)
    const int nb0 = rv0 ? a.nbr[(size_t)(i - a.row_base) * a.m + h] : 0;
    const int nb1 = rv1 ? a.nbr[(size_t)(i - a.row_base) * a.m + v1] : 0;
    double xi[ND], x0[ND], x1[ND];
#pragma unroll
    for (int q = 0; q < ND; ++q) {
      xi[q] = (q < d) ? a.X[(size_t)irow * d + q] : 0.;
      x0[q] = (q < d && rv0) ? a.X[(size_t)nb0 * d + q] : 0.;
      x1[q] = (q < d && rv1) ? a.X[(size_t)nb1 * d + q] : 0.;
    }
    const double yi = want_like ? a.Y[irow] : 0.;
    double y0s = (want_like && rv0) ? a.Y[nb0] : 0.;
    double y1s = (want_like && rv1) ? a.Y[nb1] : 0.;
    // padding rows at distinct far-away points: covariances exactly 0 (see vecchia_rows_kernel); slot
    // 30 (lane 14's second slot) is the row's own point, lane 15's second slot (31) holds no point
    const bool own1 = v1 == kMK;
#pragma unroll
    for (int q = 0; q < ND; ++q) x1[q] = own1 ? xi[q] : x1[q];
    x0[0] = rv0 ? x0[0] : 1e30 * (h + 1);
    x1[0] = (rv1 || own1) ? x1[0] : 1e30 * (v1 + 1);
    cfence();   // the previous problem's LDS reads are issued before these writes
#pragma unroll
    for (int q = 0; q < ND; ++q) {
      nbx[h * CS + q] = x0[q];
      nbx[(h + 31) * CS + q] = x0[q];   // partners past slot 30 wrap: copies of slots 0..15 at 31..46
      if (v1 <= kMK) nbx[v1 * CS + q] = x1[q];
    }
    Cp[tri(h) + h] = rv0 ? cdiag : 1.;
    Cp[tri(v1) + v1] = rv1 ? cdiag : 1.;   // slots 30, 31: 1 (border rows, not pivots)
    lds_sync();

    // ---- 1. circulant pairs: slot v with (v + delta) mod 31, delta = 1..15, for v = h and v = h + 16
    double w0[15], w1[15];
    {
      const int b0 = tri(h) + h, b1 = tri(v1) + v1;
#pragma unroll
      for (int dl = 1; dl <= 15; ++dl) {
        const double* xp = nbx + (h + dl) * CS;
        double s = 0.;
#pragma unroll
        for (int q = 0; q < ND; ++q) {
          const double t = x0[q] - xp[q];
          s += t * t;
        }
        double cv, dcv;
        cov_dcov_sq<COV>(s, var, phi, cv, dcv);
        Cp[b0 + h * dl + dl * (dl + 1) / 2] = cv;   // packed(h + dl, h)
        w0[dl - 1] = dcv;
      }
#pragma unroll
      for (int dl = 1; dl <= 15; ++dl) {
        const double* xp = nbx + (v1 + dl) * CS;
        double s = 0.;
#pragma unroll
        for (int q = 0; q < ND; ++q) {
          const double t = x1[q] - xp[q];
          s += t * t;
        }
        double cv, dcv;
        cov_dcov_sq<COV>(s, var, phi, cv, dcv);
        // packed(v1 + dl, v1), or past slot 30 packed(v1, v1 + dl - 31) (slot 31: row 31, overwritten below)
        const int pos = (v1 + dl <= kMK) ? b1 + v1 * dl + dl * (dl + 1) / 2 : b1 + dl - 31;
        Cp[pos] = cv;
        w1[dl - 1] = dcv;
      }
    }
    lds_sync();
    // border row 31 (y_nbr); row 30 (c) came from the slot-30 pairs
    Cp[tri(kMK + 1) + h] = y0s;
    if (v1 < kMK) Cp[tri(kMK + 1) + v1] = y1s;
    else if (v1 == kMK) Cp[tri(kMK + 1) + kMK] = 0.;
    lds_sync();

    // ---- 2. rows h and h + 16 into registers; c and y_nbr (their columns 30, 31) wait out the
    // elimination in the coordinate area; dC over the packed C (circulant layout W[(delta - 1) 32 + v])
    double r0[kK], r1[kK];
#pragma unroll
    for (int c = 0; c < kK; ++c) {
      r0[c] = (c <= h) ? Cp[tri(h) + c] : Cp[tri(c) + h];
      r1[c] = (c <= v1) ? Cp[tri(v1) + c] : Cp[tri(c) + v1];
    }
    double c0, c1, dc0, dc1;
    cfence();
    {
      v2d* st = reinterpret_cast<v2d*>(__builtin_assume_aligned(nbx, 16)) + 2 * h;
      st[0] = v2d{r0[kMK], rv1 ? r1[kMK] : 0.};
      st[1] = v2d{y0s, y1s};
    }
#pragma unroll
    for (int dl = 1; dl <= 15; ++dl) {
      Cp[(dl - 1) * kK + h] = w0[dl - 1];
      Cp[(dl - 1) * kK + v1] = w1[dl - 1];
    }

    // Gauss-Jordan, 30 pivots: M[j][c] = M[c][j] from lane c mod 16 (register set c / 16)
    double dg0 = 1., dg1 = 1.;
    sfor<0, kMK>([&](auto J) {
      constexpr int j = decltype(J)::value;
      constexpr int jl = j & 15;
      constexpr bool jhi = j >= 16;
      const double piv = bcast16<jl>(jhi ? r1[j] : r0[j]);
      const double rinv = recip(piv);
      const bool own = h == jl;
      double f0 = r0[j] * rinv, f1 = r1[j] * rinv;
      if constexpr (jhi) {
        f1 = own ? 0. : f1;
        dg1 = own ? piv : dg1;
      } else {
        f0 = own ? 0. : f0;
        dg0 = own ? piv : dg0;
      }
#if GPB_ROWS16_FMAC
      // each broadcast folded into its two FMAs: v_fmac_f64_dpp row_newbcast (gfx950 takes DPP on the
      // 64-bit fmac; the compiler never folds a 64-bit DPP move into its uses), so a column costs two
      // VALU ops instead of three and no move -> FMA dependency
      constexpr bool upd0 = !GPB_ROWS16_BACKSUB || !jhi;   // A rows take part in pivots 0..15 only
      const double nf0 = upd0 ? -f0 : 0., nf1 = -f1;
      sfor<j + 1, kK>([&](auto C) {
        constexpr int c = decltype(C)::value;
        constexpr bool first = c == j + 1;   // wait states before the step's first DPP read
        const double& src = c >= 16 ? r1[j] : r0[j];
        if constexpr (upd0) fmac_bcast16<c & 15, first>(r0[c], src, nf0);
        fmac_bcast16<c & 15, first && !upd0>(r1[c], src, nf1);
      });
#elif GPB_ROWS16_BCG > 1
      // GPB_ROWS16_BCG broadcasts in flight: a group's DPP moves issue before its FMAs (the compiler
      // otherwise reuses one temporary, a DPP -> FMA dependency per column)
      constexpr int BG = GPB_ROWS16_BCG;
      constexpr int ncol = kK - 1 - j;   // columns j + 1 .. kK - 1
      sfor<0, ncol / BG>([&](auto P) {
        constexpr int c0g = j + 1 + BG * decltype(P)::value;
        double m[BG];
        sfor<0, BG>([&](auto Q) {
          constexpr int c = c0g + decltype(Q)::value;
          m[decltype(Q)::value] = bcast16<c & 15>(c >= 16 ? r1[j] : r0[j]);
        });
        if constexpr (BG == 2) asm volatile("" ::"v"(m[0]), "v"(m[1]));
        if constexpr (BG == 4) asm volatile("" ::"v"(m[0]), "v"(m[1]), "v"(m[2]), "v"(m[3]));
#pragma unroll
        for (int q = 0; q < BG; ++q) {
          r0[c0g + q] = fma(-f0, m[q], r0[c0g + q]);
          r1[c0g + q] = fma(-f1, m[q], r1[c0g + q]);
        }
      });
      sfor<j + 1 + BG * (ncol / BG), kK>([&](auto C) {   // the remainder, one at a time
        constexpr int c = decltype(C)::value;
        const double mc = bcast16<c & 15>(c >= 16 ? r1[j] : r0[j]);
        r0[c] = fma(-f0, mc, r0[c]);
        r1[c] = fma(-f1, mc, r1[c]);
      });
#else
      sfor<j + 1, kK>([&](auto C) {
        constexpr int c = decltype(C)::value;
        const double mc = bcast16<c & 15>(c >= 16 ? r1[j] : r0[j]);
        r0[c] = fma(-f0, mc, r0[c]);
        r1[c] = fma(-f1, mc, r1[c]);
      });
#endif
      // pin this step's updates (otherwise the FMAs are deferred and the broadcasts stay live)
#pragma unroll
      for (int c = j + 1; c < kK; ++c) {
        if (GPB_ROWS16_BACKSUB && jhi) asm volatile("" : "+v"(r1[c]));
        else asm volatile("" : "+v"(r0[c]), "+v"(r1[c]));
      }
    });
#if GPB_ROWS16_FMAC && GPB_ROWS16_BACKSUB
    {   // A rows: M[h][30..31] -= sum_{c=16..29} M[h][c] x_c, x_c = M[c][30..31] / M[c][c] (lane c - 16)
      const double i1 = recip(dg1);
      const double na = rv1 ? -(r1[kMK] * i1) : 0., nw = rv1 ? -(r1[kMK + 1] * i1) : 0.;
      sfor<16, kMK>([&](auto C) {
        constexpr int c = decltype(C)::value;
        fmac_bcast16<c & 15, c == 16>(r0[kMK], na, r0[c]);
        fmac_bcast16<c & 15, c == 16>(r0[kMK + 1], nw, r0[c]);
      });
    }
#endif
    {   // the stashed c, y_nbr back (read before the [a, w] array below overwrites the area); dc_v = dC(v, 30):
        // the slot-30 pair at delta = v + 1 (v <= 14), slot v's pair at delta = 30 - v (v = 15..29)
      lds_sync();
      const v2d* st = reinterpret_cast<const v2d*>(__builtin_assume_aligned(nbx, 16)) + 2 * h;
      const v2d s0 = st[0], s1 = st[1];
      c0 = s0.x;
      c1 = s0.y;
      y0s = s1.x;
      y1s = s1.y;
      dc0 = Cp[h <= 14 ? h * kK + kMK : 14 * kK + 15];
      dc1 = h <= 13 ? Cp[(13 - h) * kK + v1] : 0.;
    }
    const double i0 = recip(dg0), i1 = recip(dg1);
    const double a0 = rv0 ? r0[kMK] * i0 : 0., w0v = rv0 ? r0[kMK + 1] * i0 : 0.;
    const double a1 = rv1 ? r1[kMK] * i1 : 0., w1v = rv1 ? r1[kMK + 1] * i1 : 0.;
    if (active && a.B_out != nullptr) {
      double* Bo = a.B_out + (size_t)(i - a.row_base) * a.m;
      if (h < a.m) Bo[h] = rv0 ? -a0 : 0.;
      if (v1 < a.m) Bo[v1] = rv1 ? -a1 : 0.;
    }

    // ---- 3. a^T dC a, w^T dC a over the circulant pairs (see vecchia_rows_kernel, bordered form)
    double tA, tV;
    {
      v2d* av2 = reinterpret_cast<v2d*>(__builtin_assume_aligned(nbx, 16));
      cfence();
      av2[h] = v2d{a0, w0v};
      if (v1 <= kMK) av2[v1] = v2d{a1, w1v};   // slot 30: a = w = 0
      av2[h + 31] = v2d{a0, w0v};
      lds_sync();
      double s10 = 0., s20 = 0., s11 = 0., s21 = 0.;
#pragma unroll
      for (int dl = 1; dl <= 15; ++dl) {
        const double wa = Cp[(dl - 1) * kK + h], wb = Cp[(dl - 1) * kK + v1];
        const v2d pa = av2[h + dl], pb = av2[v1 + dl];
        s10 = fma(wa, pa.x, s10);
        s20 = fma(wa, pa.y, s20);
        s11 = fma(wb, pb.x, s11);
        s21 = fma(wb, pb.y, s21);
      }
      tA = 2. * (a0 * s10 + a1 * s11);
      tV = w0v * s10 + a0 * s20 + w1v * s11 + a1 * s21;
    }

    // ---- 4. group sums (16 lanes) and the row partials
    const double ac = sum16(a0 * c0 + a1 * c1);
    const double ay = sum16(a0 * y0s + a1 * y1s);
    const double aa = sum16(a0 * a0 + a1 * a1);
    const double avv = sum16(a0 * w0v + a1 * w1v);
    const double dca = sum16(dc0 * a0 + dc1 * a1);
    const double dcv = sum16(dc0 * w0v + dc1 * w1v);
    const double ta = sum16(tA);
    const double tv = sum16(tV);
    const double D = var + a.d_nugget - ac;          // Vecchia_utils.cpp:1351, 1507, 1562
    const double Dinv = 1. / D;
    if (active && h == 0 && a.Dinv_out != nullptr) a.Dinv_out[i - a.row_base] = Dinv;
    if (want_like && active && h == 0) {
      const double By = yi - ay;
      const double u = By * Dinv;
      const double dD_var = var - delta * aa - ac;
      const double uk_var = -delta * avv;
      const double dD_rng = -(2. * dca - ta);
      const double uk_rng = -(dcv - tv);
      acc[0] += log(D);
      acc[1] += By * u;
      acc[2] += uk_var * u - 0.5 * u * u * dD_var;
      acc[3] += uk_rng * u - 0.5 * u * u * dD_rng;
      acc[4] += Dinv * dD_var;
      acc[5] += Dinv * dD_rng;
    }
  }
  if (!want_like) return;
  __syncthreads();
  const double* red = smem + 4 * PD;   // 4 x kVecchiaSums
  if (lane < kVecchiaSums) {
    const double v = ((red[lane] + red[kVecchiaSums + lane]) + red[2 * kVecchiaSums + lane]) + red[3 * kVecchiaSums + lane];
    a.block_sums[(size_t)blockIdx.x * kVecchiaSums + lane] = v;
  }
}

constexpr int kMaxGrid = 2048;   // vecchia_rows_blocks' bound (kernels.h)

template <int COV, int DIM>
int launch16(const VecchiaRowsArgs& a, hipStream_t s) {
  constexpr int CS = DIM > 0 ? DIM : kD3;
  const size_t lds = (size_t)(4 * problem_doubles<CS>() + 4 * kVecchiaSums) * sizeof(double);
  auto kern = vecchia_rows16_kernel<COV, DIM>;
  static int cap = 0;
  if (cap == 0) {
    int dev = 0, cus = 0, per_cu = 0;
    HIP_CHECK(hipGetDevice(&dev));
    HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, 64, lds));
    cap = std::max(1, std::min(per_cu * cus, kMaxGrid));
  }
  const int need = (a.r1 - a.r0 + 3) / 4;
  int blocks = std::min(need, cap);
  if (a.sched == 2) {   // the same number of sets per wave
    const int rounds = (need + blocks - 1) / blocks;
    blocks = (need + rounds - 1) / rounds;
  }
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(64), lds, s, a);
  HIP_CHECK(hipGetLastError());
  return blocks;
}

}  // namespace

int launch_vecchia_rows16(int cov_type, const VecchiaRowsArgs& a, hipStream_t s) {
  if (a.m > kMK) Fatal("16-lane row kernel: num_neighbors %d > %d", a.m, kMK);
  if (a.r1 <= a.r0) return 0;
  const bool planar = a.d == 2;
  switch (cov_type) {
    case kMatern05: return planar ? launch16<kMatern05, 2>(a, s) : launch16<kMatern05, 0>(a, s);
    case kMatern15: return planar ? launch16<kMatern15, 2>(a, s) : launch16<kMatern15, 0>(a, s);
    case kMatern25: return planar ? launch16<kMatern25, 2>(a, s) : launch16<kMatern25, 0>(a, s);
    case kGaussian: return planar ? launch16<kGaussian, 2>(a, s) : launch16<kGaussian, 0>(a, s);
    default: Fatal("unsupported covariance type %d", cov_type);
  }
  return 0;
}

}  // namespace gpb_amd
