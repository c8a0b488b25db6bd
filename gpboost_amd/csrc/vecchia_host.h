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

// Unique locations among the rows of x (row-major n x d), the reference's
// DetermineUniqueDuplicateCoordsFast (GP_utils.cpp:451-536): candidates grouped by their coordinate
// sum (ascending; a group extends while the next sum is not larger by more than 1e-10 relative,
// NumberIsSmallerThan utils.h:129-131), duplicates = squared distance < 1e-20 to a unique point of
// the group, a unique point represented by its first appearance; uniques are returned in order of
// first appearance (idx[i] = the unique index of row i).
void unique_locations(const double* x, int n, int d, std::vector<int>& uniques, std::vector<int>& idx);

}  // namespace gpb_amd
