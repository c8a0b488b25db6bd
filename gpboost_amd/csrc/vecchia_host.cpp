// Vecchia structure on the host: ordering and exact nearest-neighbour sets.
// These are one-off construction steps (excluded from the per-evaluation unit)
// whose integer outputs must be bit-identical to the reference:
//   ordering  : Vecchia_utils.cpp:1094-1095 (std::shuffle with std::mt19937(seed))
//   neighbours: Vecchia_utils.cpp:732-1058 (find_nearest_neighbors_Vecchia_fast, "nearest")
// The neighbour search is the reference's sum-of-coordinates sweep with the
// (sum_j - sum_i)^2 > d * r_k^2 cut-off, run row-parallel with OpenMP; each row's
// candidate order, comparisons and insertion sort (utils.h:245-257) are identical,
// so ties resolve identically.
#include "vecchia_host.h"

#include <algorithm>
#include <cmath>
#include <limits>
#include <numeric>
#include <random>

namespace gpb_amd {

std::vector<int> vecchia_order(int n, int seed, bool random) {
  std::vector<int> idx(n);
  std::iota(idx.begin(), idx.end(), 0);
  if (random) {
    std::mt19937 rng(seed);
    std::shuffle(idx.begin(), idx.end(), rng);
  }
  return idx;
}

void vecchia_neighbors(const double* x, int n, int d, int m, int row_begin, int row_end, int* nbr,
                       int end_search_at) {
  const int last_cand = end_search_at < 0 ? n - 2 : end_search_at;
  // coordinate sums and the sweep order (utils.h:228-236 SortIndeces = std::sort on iota)
  std::vector<double> csum(n);
  for (int i = 0; i < n; ++i) {
    double s = 0.;
    for (int q = 0; q < d; ++q) s += x[(size_t)i * d + q];
    csum[i] = s;
  }
  std::vector<int> order(n);
  std::iota(order.begin(), order.end(), 0);
  std::sort(order.begin(), order.end(), [&](int a, int b) { return csum[a] < csum[b]; });
  std::vector<int> pos(n);
  for (int i = 0; i < n; ++i) pos[order[i]] = i;

#pragma omp parallel
  {
    std::vector<double> best_d(m);
    std::vector<int> best_i(m);
#pragma omp for schedule(dynamic, 256)
    for (int i = row_begin; i < row_end; ++i) {
      int* out = nbr + (size_t)(i - row_begin) * m;
      std::fill(out, out + m, -1);
      if (i == 0) continue;
      if (i <= m) {  // conditioning set smaller than m: all earlier points, index order
        for (int j = 0; j < i; ++j) out[j] = j;
        continue;
      }
      std::fill(best_d.begin(), best_d.end(), std::numeric_limits<double>::infinity());
      std::fill(best_i.begin(), best_i.end(), 0);
      const double* xi = x + (size_t)i * d;
      bool go_down = true, go_up = true;
      int lo = pos[i], hi = pos[i];
      auto visit = [&](int cand, bool& alive) {
        if (cand >= i || cand > last_cand) return;
        const double ds = csum[cand] - csum[i];
        if (ds * ds > d * best_d[m - 1]) { alive = false; return; }
        double sq = 0.;
        const double* xc = x + (size_t)cand * d;
        for (int q = 0; q < d; ++q) { const double t = xc[q] - xi[q]; sq += t * t; }
        if (sq < best_d[m - 1]) {
          best_d[m - 1] = sq;
          best_i[m - 1] = cand;
          for (int j = m - 1; j > 0 && best_d[j] < best_d[j - 1]; --j) {
            std::swap(best_d[j], best_d[j - 1]);
            std::swap(best_i[j], best_i[j - 1]);
          }
        }
      };
      while (go_up || go_down) {
        if (lo == 0) go_down = false;
        if (hi == n - 1) go_up = false;
        if (go_down) visit(order[--lo], go_down);
        if (go_up) visit(order[++hi], go_up);
      }
      std::copy(best_i.begin(), best_i.end(), out);
    }
  }
}

void unique_locations(const double* x, int n, int d, std::vector<int>& uniques, std::vector<int>& idx) {
  constexpr double kEps = 1e-10;   // EPSILON_NUMBERS (utils.h)
  idx.assign(n, 0);
  std::vector<double> sum(n);
  for (int i = 0; i < n; ++i) {
    double s = 0.;
    for (int q = 0; q < d; ++q) s += x[(size_t)i * d + q];
    sum[i] = s;
  }
  std::vector<int> ord(n);
  for (int i = 0; i < n; ++i) ord[i] = i;
  std::sort(ord.begin(), ord.end(), [&](int a, int b) { return sum[a] < sum[b]; });
  auto smaller = [&](double a, double b) { return (b - a) > kEps * std::max(1.0, std::fabs(b)); };
  auto close = [&](int a, int b) {
    double s = 0.;
    for (int q = 0; q < d; ++q) {
      const double t = x[(size_t)a * d + q] - x[(size_t)b * d + q];
      s += t * t;
    }
    return s < kEps * kEps;
  };
  std::vector<int> rep;   // representative (first appearance) of every unique found, in discovery order
  for (int s0 = 0; s0 < n; ++s0) {
    const int i = ord[s0];
    int s1 = s0 + 1;
    while (s1 < n && !smaller(sum[i], sum[ord[s1]])) ++s1;   // [s0, s1): potential duplicates of i
    std::vector<int> local{(int)rep.size()};                  // unique indices found in this group
    rep.push_back(i);
    idx[i] = local[0];
    for (int s = s0 + 1; s < s1; ++s) {
      const int j = ord[s];
      int hit = -1;
      for (int u : local)
        if (close(rep[u], j)) { hit = u; break; }
      if (hit >= 0) {
        if (j < rep[hit]) rep[hit] = j;   // the first appearance represents the location
        idx[j] = hit;
      } else {
        local.push_back((int)rep.size());
        idx[j] = (int)rep.size();
        rep.push_back(j);
      }
    }
    s0 = s1 - 1;
  }
  // renumber by first appearance
  std::vector<int> order(rep.size());
  for (size_t u = 0; u < rep.size(); ++u) order[u] = (int)u;
  std::sort(order.begin(), order.end(), [&](int a, int b) { return rep[a] < rep[b]; });
  std::vector<int> newid(rep.size());
  uniques.resize(rep.size());
  for (size_t k = 0; k < order.size(); ++k) {
    newid[order[k]] = (int)k;
    uniques[k] = rep[order[k]];
  }
  for (int i = 0; i < n; ++i) idx[i] = newid[idx[i]];
}

}  // namespace gpb_amd
