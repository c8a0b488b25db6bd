// Host-side pieces of the stochastic Lanczos quadrature (SLQ) path that are O(n t) once or
// O(k^2) per probe: probe generation and the small tridiagonal eigenproblems.
#pragma once

#include <cstdint>
#include <vector>

namespace gpb_amd {

// Probe vectors r ~ N(0, I), identical to the reference's GenRandVecNormalParallel
// (CG_utils.cpp:930-947): column c is drawn from std::mt19937 seeded with
// std::seed_seq{seed, run_id_lo, run_id_hi, c} through std::normal_distribution<double>.
// Output layout: row-major n x t (probe-interleaved, R[i * t + c]) — the layout every
// multi-column device kernel uses. Columns are generated in parallel (OpenMP).
void gen_probes_normal(int n, int t, int seed, uint64_t run_id, double* R);
// Columns [c0, c1) of the same draw into R[i * ld + (c - c0)] (a probe-sharded rank's share).
void gen_probes_normal_cols(int n, int c0, int c1, int ld, int seed, uint64_t run_id, double* R);

// log-determinant estimate from the Lanczos tridiagonals of t probes
// (CG_utils.cpp:988-1004): n/t * sum_c e1^T log(T_c) e1.
// diag[c] has k_c entries, offdiag[c] has k_c - 1.
double slq_logdet(const std::vector<std::vector<double>>& diag, const std::vector<std::vector<double>>& offdiag,
                  int n);
// The per-probe terms e1^T log(T_c) e1 (slq_logdet = n/t * their sum in column order).
std::vector<double> slq_terms(const std::vector<std::vector<double>>& diag,
                              const std::vector<std::vector<double>>& offdiag);

// Control-variate coefficient (CG_utils.cpp:1006-1024).
double optimal_c(const double* zA, const double* zB, int t, double trA, double trB);

}  // namespace gpb_amd
