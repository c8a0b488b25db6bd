#pragma once

#include <hip/hip_runtime.h>

#include <vector>

namespace gpb_amd {

// perm[i] = original index of the i-th point in the Vecchia order.
std::vector<int> vecchia_order(int n, int seed, bool random);

// Neighbour lists for rows [row_begin, row_end) of the Vecchia-ordered coordinates x
// (row-major n x d). nbr has (row_end - row_begin) x m entries; row i holds min(i, m)
// indices in ascending distance, the rest -1. Requires m <= n - 1.
// end_search_at: candidates are the points j < i with j <= end_search_at (-1: n - 2, the
// likelihood's setting; prediction rows after n_obs observed points use n_obs - 1,
// Vecchia_utils.cpp:1716-1718, 751-753).
void vecchia_neighbors(const double* x, int n, int d, int m, int row_begin, int row_end, int* nbr,
                       int end_search_at = -1);
// Same lists, searched on the GPU (vecchia_knn.hip): one thread per row runs the identical
// sweep; bit-identical output. Synchronous on stream s.
void vecchia_neighbors_gpu(const double* x, int n, int d, int m, int row_begin, int row_end, int* nbr,
                           hipStream_t s, int end_search_at = -1);

}  // namespace gpb_amd
