// Launchers of the grouped-random-effects kernels (grouped_kernels.hip); the engine is grouped.h.
#pragma once

#include <hip/hip_runtime.h>

#include <vector>

namespace gpb_amd {

// Off-diagonal part of Z^T Z in CSR over the M RE rows (columns ascending; entries [rowptr[r],
// split[r]) belong to lower effects, [split[r], rowptr[r+1]) to higher ones), values = counts.
struct GroupedOp {
  int M;
  const int* rowptr;
  const int* split;
  const int* col;
  const double* val;
};

void launch_gre_zty(int M, const int* obs_ptr, const int* obs, const double* y, double* zty, hipStream_t s);
// D = 1/tau_k + cnt, dis = sqrt(1/D); out[k] = sum_{effect k} log D, out[K + k] = sum 1/D
void launch_gre_diag(int K, const int* cum, const double* cnt, const double* tau, double* D, double* dis, double* out,
                     hipStream_t s);
// Y = (diag(dg) + offdiag(Z^T Z)) X, t columns
void launch_gre_apply(const GroupedOp& op, const double* dg, const double* X, double* Y, int t, hipStream_t s);
// Y = (L D^-1/2) R
void launch_gre_lds_mult(const GroupedOp& op, const double* D, const double* dis, const double* R, double* Y, int t,
                         hipStream_t s);
// SSOR: X = (L D^-1/2)^-1 R (effects ascending), then Z = (L D^-1/2)^-T X (effects descending)
void launch_gre_ssor(const GroupedOp& op, const std::vector<int>& cum, const double* D, const double* dis,
                     const double* R, double* X, double* Z, int t, hipStream_t s);
// Y = D^-1 (upper triangle of A incl. diagonal) X
void launch_gre_upper(const GroupedOp& op, const double* D, const double* X, double* Y, int t, hipStream_t s);
// One grouping variable: u = zty / D, out[0] = sum cnt, out[1] = sum cnt^2 / D
void launch_gre_single(int M, const double* zty, const double* cnt, const double* D, double* u, double* out,
                       hipStream_t s);
// R = rhs - V (elementwise)
void launch_gre_residual(size_t count, const double* rhs, const double* V, double* R, hipStream_t s);

}  // namespace gpb_amd
