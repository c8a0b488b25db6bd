#include "slq_host.h"

#include <cmath>
#include <limits>
#include <random>

namespace gpb_amd {

void gen_probes_normal_cols(int n, int c0, int c1, int ld, int seed, uint64_t run_id, double* R) {
  const uint32_t s32 = static_cast<uint32_t>(seed);
#pragma omp parallel for schedule(dynamic, 1)
  for (int c = c0; c < c1; ++c) {
    std::seed_seq seq{s32, static_cast<uint32_t>(run_id), static_cast<uint32_t>(run_id >> 32), static_cast<uint32_t>(c)};
    std::mt19937 gen(seq);
    std::normal_distribution<double> nd(0., 1.);
    for (int i = 0; i < n; ++i) R[(size_t)i * ld + (c - c0)] = nd(gen);
  }
}

void gen_probes_normal(int n, int t, int seed, uint64_t run_id, double* R) {
  gen_probes_normal_cols(n, 0, t, t, seed, run_id, R);
}

namespace {

// e1^T log(T) e1 for a symmetric tridiagonal T: implicit QL with Wilkinson shifts that
// tracks only the first row of the eigenvector matrix (O(k^2) instead of O(k^3)).
double e1_log_e1(std::vector<double> d, std::vector<double> e) {
  const int k = (int)d.size();
  std::vector<double> z(k, 0.);  // z[j] = first component of eigenvector j
  z[0] = 1.;
  e.resize(k, 0.);
  for (int l = 0; l < k; ++l) {
    for (int sweep = 0; sweep < 300; ++sweep) {
      int mm = l;
      for (; mm < k - 1; ++mm) {
        const double dd = std::fabs(d[mm]) + std::fabs(d[mm + 1]);
        if (std::fabs(e[mm]) <= std::numeric_limits<double>::epsilon() * dd) break;
      }
      if (mm == l) break;
      double g = (d[l + 1] - d[l]) / (2. * e[l]);
      double r = std::hypot(g, 1.);
      g = d[mm] - d[l] + e[l] / (g + std::copysign(r, g));
      double s = 1., c = 1., p = 0.;
      bool underflow = false;
      for (int i = mm - 1; i >= l; --i) {
        const double f = s * e[i], b = c * e[i];
        r = std::hypot(f, g);
        e[i + 1] = r;
        if (r == 0.) {
          d[i + 1] -= p;
          e[mm] = 0.;
          underflow = true;
          break;
        }
        s = f / r;
        c = g / r;
        g = d[i + 1] - p;
        r = (d[i] - g) * s + 2. * c * b;
        p = s * r;
        d[i + 1] = g + p;
        g = c * r - b;
        const double zi1 = z[i + 1];
        z[i + 1] = s * z[i] + c * zi1;
        z[i] = c * z[i] - s * zi1;
      }
      if (underflow) continue;
      d[l] -= p;
      e[l] = g;
      e[mm] = 0.;
    }
  }
  double acc = 0.;
  for (int j = 0; j < k; ++j) acc += z[j] * std::log(d[j]) * z[j];
  return acc;
}

}  // namespace

std::vector<double> slq_terms(const std::vector<std::vector<double>>& diag,
                              const std::vector<std::vector<double>>& offdiag) {
  const int t = (int)diag.size();
  std::vector<double> per(t);
#pragma omp parallel for schedule(dynamic, 1)
  for (int c = 0; c < t; ++c) per[c] = e1_log_e1(diag[c], offdiag[c]);
  return per;
}

double slq_logdet(const std::vector<std::vector<double>>& diag, const std::vector<std::vector<double>>& offdiag,
                  int n) {
  const int t = (int)diag.size();
  const std::vector<double> per = slq_terms(diag, offdiag);
  double ld = 0.;
  for (int c = 0; c < t; ++c) ld += per[c];
  return ld * n / t;
}

double optimal_c(const double* zA, const double* zB, int t, double trA, double trB) {
  double den = 0.;
  for (int c = 0; c < t; ++c) den += (zB[c] - trB) * (zB[c] - trB);
  den /= t;
  if (den == 0.) return 1.;
  double num = 0.;
  for (int c = 0; c < t; ++c) num += (zA[c] - trA) * (zB[c] - trB);
  num /= t;
  return num / den;
}

}  // namespace gpb_amd
