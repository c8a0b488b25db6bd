// VaduPrecond: the VADU preconditioner of the latent-Vecchia PCG, Z = P^-1 R with
// P = B^T (D^-1 + W) B, i.e. Z = B^-1 diag(1/dw) B^-T R (dw = D^-1 + W), for t columns.
//
// Reference replaced: CGVecchiaLaplaceVec / CGTridiagVecchiaLaplace (CG_utils.cpp:56-60,
// 131-136) and the P^-1 Z products of likelihoods.h:12321-12336 — two sparse unit-triangular
// solves per application, sequential over rows in the reference.
//
// The dependency DAG of a random Vecchia ordering is deep and thin at its early end (row i
// depends on its m nearest EARLIER points) and wide afterwards. The rows are split by Vecchia
// index into three parts, each solved the way its shape allows:
//   head 0 = [0, K0)  dense: G = B_00^-1 per factor, two triangular MFMA block products per
//                     application (vadu_dense.hip);
//   head 1 = [K0, K)  one workgroup per column with the segment in LDS, a workgroup barrier per
//                     level (vadu_head.hip);
//   tail   = [K, n)   one launch per merged group of g dependency levels over the whole GPU
//                     (vadu_level.hip; in-group dependencies substituted, coefficients per factor).
// Dependencies that cross parts are folded in by partial-sum launches (vadu_head.hip). One
// application, in launch order:
//   B^T solve:  tail levels: Xt_T = R_T - B_TT^T Xt_T
//               Xt_H = R_H - B_TH^T Xt_T                     (partial, rows of both heads)
//               head 1 (LDS): Xt_1 = Xt_1 - B_11^T Xt_1
//               Xt_0 -= B_10^T Xt_1                          (partial)
//   both heads: Z_0 = G diag(1/dw_0) G^T Xt_0                (dense, G = B_00^-1)
//   lower:      Z_1 = Xt_1 / dw_1 - B_10 Z_0                 (partial)
//               head 1 (LDS): Z_1 = Z_1 - B_11 Z_1
//               tail levels: Z_T = Xt_T / dw_T - B_T* Z
// The whole sequence is captured once per buffer set into a hipGraph.
// Storage labels: any symmetric permutation of the Vecchia order (the dense block gathers its
// rows through an index list).
#pragma once

#include <hip/hip_runtime.h>

#include <vector>

#include "common.h"
#include "latent_kernels.h"

namespace gpb_amd {

class VaduPrecond {
 public:
  VaduPrecond(int n, int m, hipStream_t s) : n_(n), m_(m), s_(s) {}
  ~VaduPrecond();
  VaduPrecond(const VaduPrecond&) = delete;
  VaduPrecond& operator=(const VaduPrecond&) = delete;

  // nbr: storage-labelled n x m neighbour table (row p holds min(vo[p], m) entries); vo: storage
  // row -> Vecchia index, lab = inverse; (tptr, trow, tslot): B^T lists in storage labels (column
  // j -> rows trow[e] ascending, value slot tslot[e] = row * m + r).
  void Build(const int* nbr, const std::vector<int>& vo, const std::vector<int>& lab, const std::vector<int>& tptr,
             const std::vector<int>& trow, const std::vector<int>& tslot, int K0, int K);
  // Per factor (B values in the n x m slot layout of `nbr`).
  void Refresh(const double* Bv);
  // Per system: dw = D^-1 + W (device, n), after its values are written (stream order). Must
  // precede Apply; the pointer is captured and the lower solve's coefficients are rescaled.
  void SetDiag(const double* dw);
  // Z = P^-1 R for t columns (row-major n x t); Xt: n x t scratch (holds B^-T R afterwards).
  // stream: null = the model's; applications that may run concurrently (on different streams)
  // use different scratch slots (< kSlots).
  static constexpr int kSlots = 2;
  void Apply(const double* R, double* Z, double* Xt, int t, hipStream_t stream = nullptr, int slot = 0);
  // Diagnostics: device time of each step (reps repetitions), printed to stderr.
  void TimeParts(const double* R, double* Z, double* Xt, int t, int reps);
  void DropGraphs();

  int K0() const { return K0_; }
  int K() const { return K_; }
  int tail_levels_bt() const { return (int)mt_bt_.lptr.size() - 1; }
  int tail_levels_lower() const { return (int)mt_low_.lptr.size() - 1; }
  int segment_passes() const { return seg_bt_.npass + seg_low_.npass; }
  int launches() const;   // dependent launches per application

 private:
  void Record(const double* R, double* Z, double* Xt, int t, hipStream_t st, double* S, int slot);
  void TailSolve(bool lower, const double* R, double* Xt, double* Z, int t, hipStream_t st, int slot);
  void DenseApply(const double* X0, double* Z, int t, hipStream_t st, double* S);
  double* Scratch(int slot, int t);

  int n_, m_;
  hipStream_t s_;
  int K0_ = 0, K_ = 0, ld0_ = 0;
  DenseHead dh_{};
  const double* dw_ = nullptr;
  MergedSolve mt_bt_{}, mt_low_{};   // merged tail levels of the two solves
  DevBuf<int> d_mint_;
  DevBuf<double> d_mval_;
  DevBuf<double> d_mcoef_;   // lower-solve coefficients with 1/dw folded in (SetDiag)
  int merge_g_ = 1;
  // persistent tail solves (GPBOOST_AMD_TAIL_FORM=persist; TailPersist, latent_kernels.h)
  bool tail_persist_ = false;
  TailPersist tp_bt_{}, tp_low_{};
  DevBuf<int> d_pint_;                 // both solves' level boundaries and tagged entry rows
  DevBuf<double> Tp_[2];               // padded tail values per scratch slot (n x kTailPad)
  DevBuf<unsigned> ctr_[2];            // barrier counters per scratch slot
  bool TailPersistOn(int t) const { return tail_persist_ && t >= 2 && t <= kTailPad; }
  long tail_entries_ = 0;
  HeadSolve seg_bt_{}, seg_low_{};
  SegWave segw_bt_{}, segw_low_{};   // the one-wave form of the same segment solves (default)
  bool seg_wave_ = false;            // GPBOOST_AMD_SEG_FORM = block (default, vadu_head_kernel) | wave
  void SegSolve(bool lower, const double* in, const double* dw, double* X, int t, hipStream_t st);
  PartialList p_th_{}, p_10_{}, p_01_{};
  DevBuf<int> d_int_, d_slot_;
  DevBuf<double> d_val_;
  int nslot_ = 0;
  DevBuf<double> Bd_, G_, GT_, T_;
  DevBuf<double> S_[kSlots];   // dense-head scratch per concurrent application
  struct GraphEntry {
    const void* key[3];
    int t, slot;
    hipGraphExec_t exec;
  };
  std::vector<GraphEntry> graphs_;
  bool use_graph_ = true;
};

}  // namespace gpb_amd
