// Launchers of the grouped-random-effects kernels (grouped_kernels.hip); the engine is grouped.h.
#pragma once

#include <hip/hip_runtime.h>

#include <vector>

namespace gpb_amd {

// Entry chunks of one entry range of every row (rows ascending, chunks of a row contiguous):
// chunk q covers entries [e0[q], e1[q]) of row row[q]; the chunks of row r are [ptr[r], ptr[r+1]).
struct GreChunks {
  int n = 0;
  const int* row = nullptr;
  const int* e0 = nullptr;
  const int* e1 = nullptr;
  const int* ptr = nullptr;
};

// Off-diagonal part of Z^T Z in CSR over the M RE rows (columns ascending; entries [rowptr[r],
// split[r]) belong to lower effects, [split[r], rowptr[r+1]) to higher ones), values = counts, and
// its chunk plans for a t-column pass: tc = min(64, next_pow2(t)) lanes span columns, 256 / tc
// lanes of a workgroup span the entries of one chunk (chunk length = 8 entries per lane).
struct GroupedOp {
  int M = 0;
  const int* rowptr = nullptr;
  const int* split = nullptr;
  const int* col = nullptr;
  const double* val = nullptr;
  int tc = 64;
  GreChunks full, lower, upper;
  double* P = nullptr;   // chunk partials (>= max(full.n, lower.n, upper.n) x t doubles)
};
int gre_tc(int t);
int gre_chunk_len(int tc);

void launch_gre_zty(int M, const int* obs_ptr, const int* obs, const double* y, double* zty, hipStream_t s);
// D = 1/tau_k + cnt, dis = sqrt(1/D); out[k] = sum_{effect k} log D, out[K + k] = sum 1/D
void launch_gre_diag(int K, const int* cum, const double* cnt, const double* tau, double* D, double* dis, double* out,
                     hipStream_t s);
// Y = (diag(dg) + offdiag(Z^T Z)) X, t columns
void launch_gre_apply(const GroupedOp& op, const double* dg, const double* X, double* Y, int t, hipStream_t s);
// Y = (L D^-1/2) R
void launch_gre_lds_mult(const GroupedOp& op, const double* D, const double* dis, const double* R, double* Y, int t,
                         hipStream_t s);
// SSOR: X = (L D^-1/2)^-1 R (effects ascending), then Z = (L D^-1/2)^-T X (effects descending);
// lower_q / upper_q (K + 1): the chunk ranges of each effect's rows in op.lower / op.upper
void launch_gre_ssor(const GroupedOp& op, const std::vector<int>& cum, const std::vector<int>& lower_q,
                     const std::vector<int>& upper_q, const double* D, const double* dis, const double* R, double* X,
                     double* Z, int t, hipStream_t s);
// Y = D^-1 (upper triangle of A incl. the diagonal) X
void launch_gre_upper(const GroupedOp& op, const double* D, const double* X, double* Y, int t, hipStream_t s);
// One grouping variable: u = zty / D, out[0] = sum cnt, out[1] = sum cnt^2 / D
void launch_gre_single(int M, const double* zty, const double* cnt, const double* D, double* u, double* out,
                       hipStream_t s);
// R = rhs - V (elementwise)
void launch_gre_residual(size_t count, const double* rhs, const double* V, double* R, hipStream_t s);
// Dense Cholesky form (K >= 2, matrix_inversion_method = "cholesky"): A = diag(D) + the off-diagonal
// Z^T Z counts into the column-major M x M matrix (ld; zero-filled beforehand), and diag(A^-1)_i =
// sum_{r >= i} Li[r, i]^2 from the lower inverse Cholesky factor Li.
void launch_gre_dense_build(int M, int ld, const int* rowptr, const int* col, const double* val, const double* D,
                            double* A, hipStream_t s);
void launch_gre_inv_diag(int M, int ld, const double* Li, double* out, hipStream_t s);
// E[:, p] = sum_k Li[:, idx[p K + k]] (lower part only; idx < 0 skipped) into E (M x np, ld), or (E null)
// var[p] = ||that column||^2
void launch_gre_pred_cols(int M, int ld, int K, int np, const int* idx, const double* Li, double* E, double* var,
                          hipStream_t s);
// Fisher information pieces (cholesky): B = S^1/2 A^-1 S^1/2 (sc[r] = 1 / sqrt(tau_k(r))) from the dense
// A^-1 (Ainv, ld); part[c K + k] = sum_{r in effect k} B[r, c]^2, diag[c] = B[c, c]. One wave per column.
void launch_gre_fisher_cols(int M, int ld, int K, const int* cum, const double* sc, const double* Ainv, double* part,
                            double* diag, hipStream_t s);

}  // namespace gpb_amd
