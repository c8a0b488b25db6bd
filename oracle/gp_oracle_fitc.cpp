// ORACLE TEST INFRASTRUCTURE — NOT PART OF THE PRODUCT.
//
// CPU restatement of the reference's FITC approximation for the Gaussian likelihood
// (gp_approx = "fitc"), used only as the checker by tests/. Plain O(n m^2) loops that follow
// the reference's matrix expressions term by term:
//   inducing points : re_model_template.h:6931-7073 -> GP_utils.cpp:203-223 (random_plusplus),
//                     :225-267 (calculate_means), :269-295 (kmeans_plusplus), utils.h:323-337
//                     (SampleIntNoReplaceSort); std::mt19937(seed) (re_model_template.h:154)
//   Sigma components: re_model_template.h:7341-7378 (jitter utils.h:39)
//   Woodbury factor : re_model_template.h:8823-8863
//   y_aux           : re_model_template.h:8898-8908
//   log det         : re_model_template.h:2698-2714
//   gradient        : re_model_template.h:1985-2232 (FITC branch), nugget :1992-1995
// Parity is pinned by tests/golden/golden_fitc.json (the reference itself, oracle/_ref/ref_harness
// gp_approx=fitc; tests/golden/make_golden_fitc.py).
#include <algorithm>
#include <cmath>
#include <random>
#include <vector>

#include "orc_math.h"

namespace {

const double kJitter = 1. + 1e-6;   // JITTER_MULT_IP_FITC_FSA (utils.h:39)

// GP_utils.cpp:196 / 234: (x - mu).lpNorm<2>() = sqrt of the in-order sum of squares
double km_dist(const double* x, const double* mu, int d) {
  double s = 0.;
  for (int q = 0; q < d; ++q) {
    const double t = x[q] - mu[q];
    const double sq = t * t;
    s = s + sq;
  }
  return std::sqrt(s);
}

// forward substitution L x = b (row-major lower L, k x k)
void fwd(const std::vector<double>& L, int k, double* b) {
  for (int i = 0; i < k; ++i) {
    double s = b[i];
    for (int p = 0; p < i; ++p) s -= L[(size_t)i * k + p] * b[p];
    b[i] = s / L[(size_t)i * k + i];
  }
}

}  // namespace

extern "C" {

}  // extern "C"

namespace {

// the selection with the caller's generator (CreateREComponentsFITC_FSA continues the model's rng_)
int inducing_points(const double* x, int n, int d, int m, int method, std::mt19937& gen, double* Z) {
  if (m > n || m < 1) return -1;
  if (method == 1) {
    std::vector<int> idx;
    for (int r = n - m; r < n; ++r) {
      int v = std::uniform_int_distribution<>(0, r)(gen);
      if (std::find(idx.begin(), idx.end(), v) == idx.end()) idx.push_back(v);
      else idx.push_back(r);
    }
    std::sort(idx.begin(), idx.end());
    for (int j = 0; j < m; ++j)
      for (int q = 0; q < d; ++q) Z[(size_t)j * d + q] = x[(size_t)idx[j] * d + q];
    return 0;
  }
  // random_plusplus
  std::vector<double> dist(n, 1.);
  for (int i = 0; i < m; ++i) {
    if (i == 1)
      for (double& v : dist) v *= -1;
    if (i > 0) {
      for (int p = 0; p < n; ++p) {
        double dd = km_dist(x + (size_t)p * d, Z + (size_t)(i - 1) * d, d);
        if (dist[p] > dd || dist[p] < 0) dist[p] = dd;
      }
    }
    int v = std::discrete_distribution<>(dist.data(), dist.data() + n)(gen);
    for (int q = 0; q < d; ++q) Z[(size_t)i * d + q] = x[(size_t)v * d + q];
  }
  // Lloyd iterations until the means repeat the previous or the one-before-previous iterate
  const size_t cnt = (size_t)m * d;
  std::vector<double> mu(Z, Z + cnt), old(cnt, 0.), old_old(cnt, 0.), sum(cnt);
  std::vector<int> cl(n);
  int it = 0;
  const int max_it = 1000;   // re_model_template.h:6995
  do {
    old_old = old;
    old = mu;
    for (int p = 0; p < n; ++p) {
      int best = 0;
      double bd = km_dist(x + (size_t)p * d, mu.data(), d);
      for (int j = 1; j < m; ++j) {
        double dj = km_dist(x + (size_t)p * d, mu.data() + (size_t)j * d, d);
        if (dj < bd) { bd = dj; best = j; }
      }
      cl[p] = best;
    }
    for (int j = 0; j < m; ++j) {
      double s[3] = {0., 0., 0.};
      int c = 0;
      for (int p = 0; p < n; ++p)
        if (cl[p] == j) {
          for (int q = 0; q < d; ++q) s[q] = s[q] + x[(size_t)p * d + q];
          ++c;
        }
      if (c > 0)
        for (int q = 0; q < d; ++q) mu[(size_t)j * d + q] = s[q] / c;
    }
    ++it;
  } while (mu != old && mu != old_old && it != max_it);
  std::copy(mu.begin(), mu.end(), Z);
  return it;
}

}  // namespace

extern "C" {

// method 0 = kmeans++, 1 = random. coords row-major n x d; Z row-major m x d.
int orc_fitc_inducing_points(const double* x, int n, int d, int m, int method, int seed, double* Z) {
  std::mt19937 gen((std::mt19937::result_type)seed);
  return inducing_points(x, n, d, m, method, gen, Z);
}

// full_scale_vecchia (re_model_template.h:348-357): the model's rng_ = mt19937(seed) first shuffles the
// data order (random ordering), then CreateREComponentsFITC_FSA selects the inducing points on the
// coordinates in that order with the same generator. perm (n) receives the order.
int orc_vif_inducing_points(const double* x, int n, int d, int m, int method, int seed, int shuffle, double* Z,
                            int* perm) {
  std::mt19937 gen((std::mt19937::result_type)seed);
  std::vector<int> idx(n);
  for (int i = 0; i < n; ++i) idx[i] = i;
  if (shuffle) std::shuffle(idx.begin(), idx.end(), gen);
  std::vector<double> xv((size_t)n * d);
  for (int i = 0; i < n; ++i)
    for (int q = 0; q < d; ++q) xv[(size_t)i * d + q] = x[(size_t)idx[i] * d + q];
  std::copy(idx.begin(), idx.end(), perm);
  return inducing_points(xv.data(), n, d, m, method, gen, Z);
}

// FITC nll + gradient on the transformed scale pars = (sigma2, sigma1^2 / sigma2, phi); mode 0:
// gradient [nugget, var, range] at sigma2 = pars[0]; mode 1: sigma2 profiled (q / n), gradient
// [var, range]. Returns 0, or -1 when a Cholesky factorization fails.
int orc_fitc_nll_grad(const double* x, const double* y, int n, int d, const double* Z, int m, int t,
                      const double* pars, int mode, double* nll, double* grad, double* sigma2_out) {
  const double var = pars[1], phi = pars[2];
  // K_nm (row-major n x m), K_mm, dK (log-scale derivatives, un-jittered)
  std::vector<double> Knm((size_t)n * m), dKnm((size_t)n * m), Kmm((size_t)m * m), dKmm((size_t)m * m);
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < m; ++j) {
      const double r = dist(x + (size_t)i * d, Z + (size_t)j * d, d);
      Knm[(size_t)i * m + j] = cov(t, r, var, phi);
      dKnm[(size_t)i * m + j] = dcov_dlogphi(t, r, var, phi);
    }
  for (int j = 0; j < m; ++j)
    for (int k = 0; k < m; ++k) {
      if (j == k) { Kmm[(size_t)j * m + k] = var; dKmm[(size_t)j * m + k] = 0.; continue; }
      const double r = dist(Z + (size_t)j * d, Z + (size_t)k * d, d);
      Kmm[(size_t)j * m + k] = cov(t, r, var, phi);
      dKmm[(size_t)j * m + k] = dcov_dlogphi(t, r, var, phi);
    }
  std::vector<double> Ks = Kmm;
  for (int j = 0; j < m; ++j) Ks[(size_t)j * m + j] *= kJitter;
  std::vector<double> L = Ks;
  if (!chol(L, m)) return -1;
  // V = L^-1 K_mn; d = 1 + Ks_00 - colsum V^2
  std::vector<double> V((size_t)n * m), dd(n);
  for (int i = 0; i < n; ++i) {
    double* v = V.data() + (size_t)i * m;
    for (int j = 0; j < m; ++j) v[j] = Knm[(size_t)i * m + j];
    fwd(L, m, v);
    double s = 0.;
    for (int j = 0; j < m; ++j) s += v[j] * v[j];
    dd[i] = (1. + Ks[0]) - s;
  }
  // W = K_mn D^-1 K_nm + Ks
  std::vector<double> W = Ks;
  for (int j = 0; j < m; ++j)
    for (int k = 0; k <= j; ++k) {
      double s = 0.;
      for (int i = 0; i < n; ++i) s += Knm[(size_t)i * m + j] * Knm[(size_t)i * m + k] / dd[i];
      W[(size_t)j * m + k] += s;
      if (k != j) W[(size_t)k * m + j] += s;
    }
  std::vector<double> Lw = W;
  if (!chol(Lw, m)) return -1;
  // y_aux
  std::vector<double> u(m, 0.), yaux(n);
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < m; ++j) u[j] += Knm[(size_t)i * m + j] * (y[i] / dd[i]);
  chol_solve(Lw, m, u.data());
  double q = 0., logdet = 0.;
  for (int i = 0; i < n; ++i) {
    double s = 0.;
    for (int j = 0; j < m; ++j) s += Knm[(size_t)i * m + j] * u[j];
    yaux[i] = y[i] / dd[i] - s / dd[i];
    q += y[i] * yaux[i];
    logdet += std::log(dd[i]);
  }
  for (int j = 0; j < m; ++j) logdet += -2. * std::log(L[(size_t)j * m + j]) + 2. * std::log(Lw[(size_t)j * m + j]);
  double sigma2 = pars[0];
  if (mode == 1) sigma2 = q / n;
  *sigma2_out = sigma2;
  *nll = q / 2. / sigma2 + logdet / 2. + n / 2. * (std::log(sigma2) + std::log(2 * M_PI));
  int off = 0;
  if (mode == 0) { grad[0] = -q / sigma2 / 2. + n / 2.; off = 1; }
  // P = Ks^-1 K_mn (column i = Ks^-1 K_nm[i, :]^T), a = P y_aux
  std::vector<double> P((size_t)n * m), a(m, 0.);
  for (int i = 0; i < n; ++i) {
    double* p = P.data() + (size_t)i * m;
    for (int j = 0; j < m; ++j) p[j] = Knm[(size_t)i * m + j];
    chol_solve(L, m, p);
    for (int j = 0; j < m; ++j) a[j] += p[j] * yaux[i];
  }
  for (int par = 0; par < 2; ++par) {
    const std::vector<double>& G = par == 0 ? Knm : dKnm;   // cross_cov_grad
    const std::vector<double>& Gm = par == 0 ? Kmm : dKmm;  // sigma_ip_stable_grad
    double g = 0.;
    // -1/2 tr(Ks^-1 dKmm)
    std::vector<double> col(m);
    double tr1 = 0.;
    for (int k = 0; k < m; ++k) {
      for (int j = 0; j < m; ++j) col[j] = Gm[(size_t)j * m + k];
      chol_solve(L, m, col.data());
      tr1 += col[k];
    }
    g -= 0.5 * tr1;
    // (1/2 a^T dKmm a - (dK_mn y_aux) . a) / sigma2
    double aga = 0., gya = 0.;
    for (int j = 0; j < m; ++j)
      for (int k = 0; k < m; ++k) aga += a[j] * Gm[(size_t)j * m + k] * a[k];
    for (int i = 0; i < n; ++i)
      for (int j = 0; j < m; ++j) gya += G[(size_t)i * m + j] * yaux[i] * a[j];
    g += (0.5 * aga - gya) / sigma2;
    // FITC_Diag_grad
    std::vector<double> FD(n, Gm[0]);
    for (int i = 0; i < n; ++i) {
      const double* p = P.data() + (size_t)i * m;
      double s1 = 0., s2 = 0.;
      for (int j = 0; j < m; ++j) {
        s1 += p[j] * G[(size_t)i * m + j];
        double gp = 0.;
        for (int k = 0; k < m; ++k) gp += Gm[(size_t)j * m + k] * p[k];
        s2 += p[j] * gp;
      }
      FD[i] -= 2 * s1 - s2;
    }
    double q3 = 0., t3 = 0.;
    for (int i = 0; i < n; ++i) { q3 += yaux[i] * FD[i] * yaux[i]; t3 += FD[i] / dd[i]; }
    g += -0.5 * q3 / sigma2 + 0.5 * t3;
    // Woodbury derivative: K_mn D^-1 dK_nm + (.)^T - K_mn diag(FD / d^2) K_nm + dKmm; 1/2 tr(W^-1 .)
    std::vector<double> Wg((size_t)m * m);
    for (int j = 0; j < m; ++j)
      for (int k = 0; k < m; ++k) {
        double s = 0.;
        for (int i = 0; i < n; ++i) {
          const double inv = 1. / dd[i];
          s += Knm[(size_t)i * m + j] * inv * G[(size_t)i * m + k] + G[(size_t)i * m + j] * inv * Knm[(size_t)i * m + k] -
               Knm[(size_t)i * m + j] * (inv * inv * FD[i]) * Knm[(size_t)i * m + k];
        }
        Wg[(size_t)j * m + k] = s + Gm[(size_t)j * m + k];
      }
    double tr4 = 0.;
    for (int k = 0; k < m; ++k) {
      for (int j = 0; j < m; ++j) col[j] = Wg[(size_t)j * m + k];
      chol_solve(Lw, m, col.data());
      tr4 += col[k];
    }
    g += 0.5 * tr4;
    grad[off + par] = g;
  }
  return 0;
}

}  // extern "C"
