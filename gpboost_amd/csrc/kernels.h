// Host-callable launchers for the HIP kernels (implemented in *.hip).
#pragma once

#include <hip/hip_runtime.h>

namespace gpb_amd {

// Number of partial sums per Vecchia row reduction:
// [logdet, q, s1_var, s1_range, s2_var, s2_range] (DESIGN.md "reduction contract").
constexpr int kVecchiaSums = 6;

struct VecchiaRowsArgs {
  const double* X;       // coords, Vecchia order, row-major n x d
  const double* Y;       // response, Vecchia order (may be null when only factor outputs are needed)
  const int* nbr;        // n x m neighbour indices (row i holds min(i, m) valid entries)
  int n, d, m;
  int r0, r1;            // row range of this launch
  double var, phi;       // transformed-scale marginal variance and range
  double diag_mult;      // between-neighbour diagonal: var * diag_mult + diag_add
  double diag_add;       //   gaussian: (1, 1)  [nugget, Vecchia_utils.cpp:1540]
                         //   latent:   (1 + 1e-10, 0) [JITTER_MULT_VECCHIA, :1547]
  double d_nugget;       // D_ii initial nugget term: 1 gaussian, 0 latent (:1351-1357)
  double* block_sums;    // [num_blocks x kVecchiaSums] (nullable if Y is null)
  double* Dinv_out;      // optional [n]  (indexed by global row)
  double* B_out;         // optional [n x m], B(i, nbr) = -A_i, 0-padded
  int row_base;          // nbr, B_out and Dinv_out hold rows from row_base on (0: all rows;
                         // predictions: the rows after the observed ones)
  int sched;             // 16-lane kernel, grid grid G < problem sets: 0 = wave w takes sets w, w + G, ...;
                         // 1 = the last, partial round's sets spread evenly over the waves;
                         // 2 = as 0 with G = ceil(sets / rounds) (every wave the same count)
};

int vecchia_rows_blocks(int rows, int m);   // upper bound of the grid (block-partial buffer size)
int launch_vecchia_rows(int cov_type, const VecchiaRowsArgs& a, hipStream_t s);   // returns the grid size
// 16-lane form for m <= 30 (vecchia_rows16.hip; DPP broadcasts, four rows per wave), same contract
int launch_vecchia_rows16(int cov_type, const VecchiaRowsArgs& a, hipStream_t s);
// Predictions from the prediction rows' factor: out[p] = -sum_r B[p, r] y[nbr[p, r]] (mean),
// out[n_pred + p] = (1 / Dinv[p] - nugget_sub) * sigma2 (variance). B, nbr: n_pred x m.
void launch_predict_mean_var(int n_pred, int m, const int* nbr, const double* B, const double* Dinv, const double* y,
                             double sigma2, double nugget_sub, double* out, hipStream_t s);
// Deterministic fixed-order sum of block partials -> out[kVecchiaSums].
// flag (nullable; host-coherent memory): after the sums are visible system-wide, *flag = seq (the
// host spins on it instead of synchronising the stream)
void launch_sum_blocks(const double* block_sums, int nblocks, int width, double* out, hipStream_t s,
                       unsigned long long* flag = nullptr, unsigned long long seq = 0);

// ---------------------------------------------------------------- dense path
struct DenseArgs {
  const double* X;   // coords row-major n x d (original order)
  int n, d, ld;      // ld = leading dimension of the n x n matrices (column-major)
  double var, phi;
};
// Sigma (+ I nugget on the diagonal) and dSigma/dlog(phi) as full n x n column-major matrices.
void launch_dense_build(int cov_type, const DenseArgs& a, double* Psi, double* dPsi, hipStream_t s);

}  // namespace gpb_amd
