// ORACLE TEST INFRASTRUCTURE — NOT PART OF THE PRODUCT.
// CPU restatement of the reference GP-likelihood hot path (see gp_oracle.h for the
// contract and how it is pinned). Written from the reference's math, citing the
// reference file:line each function follows. Plain loops, no Eigen, no GPU.
#include "gp_oracle.h"
#include "orc_math.h"

#include <algorithm>
#include <cmath>
#include <limits>
#include <numeric>
#include <random>
#include <vector>

namespace {

constexpr double kNugget = 1.0;  // transformed scale: Psi = Sigma/sigma2 + I

// Per-row Vecchia factor + derivatives for one row (Vecchia_utils.cpp:1405-1617,
// Gaussian likelihood, single GP component, transf_scale = true).
struct RowFactor {
  int k;
  std::vector<double> A;            // A_i (B(i,nbr) = -A_i)
  double D;                         // D_ii (not inverted)
  std::vector<double> dA[2];        // dA_i / dlog(par), par = var, range
  double dD[2];
};

void row_factor(const double* coords, const int* nbr_row, int i, int d, int m, int t,
                double var, double phi, RowFactor& f) {
  int k = std::min(i, m);
  f.k = k;
  f.A.assign(k, 0.);
  f.dA[0].assign(k, 0.);
  f.dA[1].assign(k, 0.);
  f.D = kNugget + var;        // :1351 identity nugget, :1507 += marginal variance
  f.dD[0] = var;              // :1512 derivative wrt the variance (transformed scale)
  f.dD[1] = 0.;
  if (k == 0) return;
  const double* xi = coords + (size_t)i * d;
  std::vector<double> c(k), dc(k), C(k * k), dC(k * k);
  for (int a = 0; a < k; ++a) {
    const double* xa = coords + (size_t)nbr_row[a] * d;
    double r = dist(xi, xa, d);
    c[a] = cov(t, r, var, phi);
    dc[a] = dcov_dlogphi(t, r, var, phi);
    for (int b = 0; b < k; ++b) {
      if (a == b) { C[a * k + b] = var; dC[a * k + b] = 0.; continue; }  // variance on diag, grad 0
      const double* xb = coords + (size_t)nbr_row[b] * d;
      double rab = dist(xa, xb, d);
      C[a * k + b] = cov(t, rab, var, phi);
      dC[a * k + b] = dcov_dlogphi(t, rab, var, phi);
    }
  }
  std::vector<double> L = C;
  for (int a = 0; a < k; ++a) L[a * k + a] += kNugget;   // :1540 nugget on between-neighbour cov
  if (!chol(L, k)) { f.D = std::numeric_limits<double>::quiet_NaN(); return; }
  // A_i = (C^-1 c)^T  (:1557)
  f.A = c;
  chol_solve(L, k, f.A.data());
  double Ac = 0.;
  for (int a = 0; a < k; ++a) Ac += f.A[a] * c[a];
  f.D -= Ac;                                              // :1562
  // gradients (:1573-1585): dA = (C^-1 dc)^T - A (C^-1 dC)^T ;
  // dD = d(marg var) - (dA c + A dc)
  for (int p = 0; p < 2; ++p) {
    const std::vector<double>& dcp = (p == 0) ? c : dc;      // d/dlog var: dc = c, dC = C
    const std::vector<double>& dCp = (p == 0) ? C : dC;
    std::vector<double> s = dcp;
    chol_solve(L, k, s.data());
    // A (C^-1 dC)^T = A dC C^-1  -> row vector: w^T = A dC, then solve
    std::vector<double> w(k, 0.);
    for (int b = 0; b < k; ++b) {
      double acc = 0.;
      for (int a = 0; a < k; ++a) acc += f.A[a] * dCp[a * k + b];
      w[b] = acc;
    }
    chol_solve(L, k, w.data());
    double dAc = 0., Adc = 0.;
    for (int a = 0; a < k; ++a) {
      f.dA[p][a] = s[a] - w[a];
      dAc += f.dA[p][a] * c[a];
      Adc += f.A[a] * dcp[a];
    }
    if (p == 0) f.dD[0] -= (dAc + Adc);   // :1579 ipar == 0 -> subtract from existing
    else f.dD[1] = -(dAc + Adc);          // :1583 range -> overwrite
  }
}

int num_pars_grad() { return 2; }

}  // namespace

extern "C" {

void orc_transform_cov_pars(int t, const double* orig, double* trafo) {
  // cov_fcts.h:438-460
  trafo[0] = orig[0];
  trafo[1] = orig[1] / orig[0];
  switch (t) {
    case ORC_MATERN05: trafo[2] = 1. / orig[2]; break;
    case ORC_MATERN15: trafo[2] = std::sqrt(3.) / orig[2]; break;
    case ORC_MATERN25: trafo[2] = std::sqrt(5.) / orig[2]; break;
    case ORC_GAUSSIAN: trafo[2] = 1. / (orig[2] * orig[2]); break;
  }
}

void orc_vecchia_order(int n, int seed, int random_ordering, int* perm) {
  std::vector<int> idx(n);
  std::iota(idx.begin(), idx.end(), 0);
  if (random_ordering) {
    std::mt19937 rng(seed);  // re_model_template.h:154, type_defs.h RNG_t
    std::shuffle(idx.begin(), idx.end(), rng);
  }
  std::copy(idx.begin(), idx.end(), perm);
}

// FindInitCovPar's range (re_model_template.h:4452-4458 -> cov_fcts.h:1275-1450): median of the
// pairwise distances of at most 1000 points, for n > 1000 drawn by std::uniform_int_distribution
// from the model's mt19937(seed) after the Vecchia ordering shuffle (Vecchia_utils.cpp:1094-1095);
// phi such that the correlation is 0.05 at half the median. x: the component's coordinates
// (Vecchia order for the Vecchia approximation), row-major n x d.
double orc_init_range_trafo(const double* x, int n, int d, int seed, int shuffled, int t) {
  const int nf = std::min(n, 1000);
  std::vector<int> idx(nf);
  if (nf < n) {
    std::mt19937 rng(seed);
    if (shuffled) {
      std::vector<int> dummy(n);
      std::iota(dummy.begin(), dummy.end(), 0);
      std::shuffle(dummy.begin(), dummy.end(), rng);
    }
    std::uniform_int_distribution<> dis(0, n - 1);
    for (int i = 0; i < nf; ++i) idx[i] = dis(rng);
  } else {
    std::iota(idx.begin(), idx.end(), 0);
  }
  std::vector<double> dist;
  dist.reserve((size_t)nf * (nf - 1) / 2);
  for (int i = 0; i < nf - 1; ++i)
    for (int j = i + 1; j < nf; ++j) {
      double s = 0.;
      for (int q = 0; q < d; ++q) {
        const double u = x[(size_t)idx[i] * d + q] - x[(size_t)idx[j] * d + q];
        s += u * u;
      }
      dist.push_back(std::sqrt(s));
    }
  const size_t pos = dist.size() / 2;   // utils.h:189-202
  std::nth_element(dist.begin(), dist.begin() + pos, dist.end());
  double med = dist[pos];
  if (dist.size() % 2 == 0) {
    std::nth_element(dist.begin(), dist.begin() + pos - 1, dist.end());
    med = (med + dist[pos - 1]) / 2.;
  }
  if (med < 1e-10) med = std::accumulate(dist.begin(), dist.end(), 0.) / (double)dist.size();
  switch (t) {
    case 0: return 2. * 3. / med;
    case 1: return 2. * 4.7 / med;
    case 2: return 2. * 5.9 / med;
    default: return 3. / std::pow(med / 2., 2.);
  }
}

void orc_find_neighbors(const double* x, int n, int d, int m, int* nbr) {
  std::fill(nbr, nbr + (size_t)n * m, -1);
  const int end_search_at = n - 2;                 // :751-753
  if (m > end_search_at + 1) m = end_search_at + 1;  // :754-757 (caller passes stride m)
  std::vector<double> csum(n);
  for (int i = 0; i < n; ++i) {
    double s = 0.;
    for (int k = 0; k < d; ++k) s += x[(size_t)i * d + k];
    csum[i] = s;
  }
  std::vector<int> sort_sum(n);                    // utils.h:228-236
  std::iota(sort_sum.begin(), sort_sum.end(), 0);
  std::sort(sort_sum.begin(), sort_sum.end(), [&](int a, int b) { return csum[a] < csum[b]; });
  std::vector<int> inv(n);
  for (int i = 0; i < n; ++i) inv[sort_sum[i]] = i;
  for (int i = 1; i <= std::min(m, n - 1); ++i)    // :786-807 first rows: all earlier points
    for (int j = 0; j < i; ++j) nbr[(size_t)i * m + j] = j;
  std::vector<double> nd(m);
  std::vector<int> ni(m);
  for (int i = m + 1; i < n; ++i) {                 // :883-898, :994-1058
    std::fill(nd.begin(), nd.end(), std::numeric_limits<double>::infinity());
    std::fill(ni.begin(), ni.end(), 0);
    bool up = true, down = true;
    int up_i = inv[i], down_i = inv[i];
    auto consider = [&](int cand, bool& dir) {
      if (cand < i && cand <= end_search_at) {
        double smd = (csum[cand] - csum[i]) * (csum[cand] - csum[i]);
        if (smd > d * nd[m - 1]) { dir = false; return; }
        double sed = 0.;
        for (int k = 0; k < d; ++k) {
          double t = x[(size_t)cand * d + k] - x[(size_t)i * d + k];
          sed += t * t;
        }
        if (sed < nd[m - 1]) {
          nd[m - 1] = sed;
          ni[m - 1] = cand;
          for (int j = m - 1; j > 0 && nd[j] < nd[j - 1]; --j) {  // utils.h:245-257
            std::swap(nd[j], nd[j - 1]);
            std::swap(ni[j], ni[j - 1]);
          }
        }
      }
    };
    while (up || down) {
      if (down_i == 0) down = false;
      if (up_i == n - 1) up = false;
      if (down) { --down_i; consider(sort_sum[down_i], down); }
      if (up) { ++up_i; consider(sort_sum[up_i], up); }
    }
    for (int j = 0; j < m; ++j) nbr[(size_t)i * m + j] = ni[j];
  }
}

// Prediction neighbours, vecchia_pred_type = "order_obs_first_cond_obs_only"
// (Vecchia_utils.cpp:1672-1674, 1715-1718 -> :732-1058 with start_at = n_obs,
// end_search_at = n_obs - 1): x_all = observed points (model order) then prediction points; row
// i >= n_obs takes its m nearest among the observed points by the same coordinate-sum sweep.
// nbr: n_pred x m; m must be <= n_obs (the reference caps it at end_search_at + 1, :754-757).
void orc_find_neighbors_pred(const double* x, int n_obs, int n_all, int d, int m, int* nbr) {
  const int end_search_at = n_obs - 1;
  std::vector<double> csum(n_all);
  for (int i = 0; i < n_all; ++i) {
    double s = 0.;
    for (int k = 0; k < d; ++k) s += x[(size_t)i * d + k];
    csum[i] = s;
  }
  std::vector<int> sort_sum(n_all);
  std::iota(sort_sum.begin(), sort_sum.end(), 0);
  std::sort(sort_sum.begin(), sort_sum.end(), [&](int a, int b) { return csum[a] < csum[b]; });
  std::vector<int> inv(n_all);
  for (int i = 0; i < n_all; ++i) inv[sort_sum[i]] = i;
  std::vector<double> nd(m);
  std::vector<int> ni(m);
  for (int i = n_obs; i < n_all; ++i) {
    std::fill(nd.begin(), nd.end(), std::numeric_limits<double>::infinity());
    std::fill(ni.begin(), ni.end(), 0);
    bool up = true, down = true;
    int up_i = inv[i], down_i = inv[i];
    auto consider = [&](int cand, bool& dir) {
      if (cand < i && cand <= end_search_at) {
        double smd = (csum[cand] - csum[i]) * (csum[cand] - csum[i]);
        if (smd > d * nd[m - 1]) { dir = false; return; }
        double sed = 0.;
        for (int k = 0; k < d; ++k) {
          double t = x[(size_t)cand * d + k] - x[(size_t)i * d + k];
          sed += t * t;
        }
        if (sed < nd[m - 1]) {
          nd[m - 1] = sed;
          ni[m - 1] = cand;
          for (int j = m - 1; j > 0 && nd[j] < nd[j - 1]; --j) {
            std::swap(nd[j], nd[j - 1]);
            std::swap(ni[j], ni[j - 1]);
          }
        }
      }
    };
    while (up || down) {
      if (down_i == 0) down = false;
      if (up_i == n_all - 1) up = false;
      if (down) { --down_i; consider(sort_sum[down_i], down); }
      if (up) { ++up_i; consider(sort_sum[up_i], up); }
    }
    for (int j = 0; j < m; ++j) nbr[(size_t)(i - n_obs) * m + j] = ni[j];
  }
}

// Predictive mean and variance, exact Gaussian Vecchia, "order_obs_first_cond_obs_only"
// (Vecchia_utils.cpp:1779-1895, 1900-1931; re_model_template.h:3787-3803, :4066-4071): per
// prediction point the row of (Bpo, Dp) from its observed neighbours — A = (C + I)^-1 c,
// Dp = 1 + marginal variance - A c on the transformed scale — then mean = -Bpo y = A . y_nbr,
// var = (Dp - [latent: 1]) * sigma2. pars = transformed (sigma2, sigma1^2 / sigma2, phi).
int orc_vecchia_predict(const double* x_all, const double* y_obs, const int* nbr, int n_obs, int n_pred, int d,
                        int m, int t, const double* pars, int predict_response, double* mean, double* var) {
  RowFactor f;
  std::vector<int> row(m);
  for (int p = 0; p < n_pred; ++p) {
    const int i = n_obs + p;
    for (int r = 0; r < m; ++r) row[r] = nbr[(size_t)p * m + r];
    // row_factor with k = min(i, m) = m: the same per-row algebra as the likelihood rows
    row_factor(x_all, row.data(), i, d, m, t, pars[1], pars[2], f);
    if (!(f.D > 0.)) return -1;
    double mu = 0.;
    for (int r = 0; r < f.k; ++r) mu += f.A[r] * y_obs[row[r]];
    mean[p] = mu;
    if (var) var[p] = (f.D - (predict_response ? 0. : kNugget)) * pars[0];
  }
  return 0;
}

int orc_vecchia_partials(const double* coords, const double* y, const int* nbr,
                         int n, int d, int m, int t, const double* pars,
                         int r0, int r1, double* sums) {
  const double var = pars[1], phi = pars[2];
  const int P = num_pars_grad();
  std::fill(sums, sums + 2 + 2 * P, 0.);
  RowFactor f;
  for (int i = r0; i < r1; ++i) {
    const int* nb = nbr + (size_t)i * m;
    row_factor(coords, nb, i, d, m, t, var, phi, f);
    if (!(f.D > 0.)) return -1;
    // By (re_model_template.h:9073-9080): (B y)_i = y_i - A_i . y_nbr
    double By = y[i];
    for (int a = 0; a < f.k; ++a) By -= f.A[a] * y[nb[a]];
    const double Dinv = 1. / f.D;
    const double u = Dinv * By;                 // u = D^-1 B y (:1779)
    sums[0] += -std::log(Dinv);                 // logdet = -sum log D^-1 (:2694-2695)
    sums[1] += By * By * Dinv;                  // q = (By)^T D^-1 (By)
    for (int p = 0; p < P; ++p) {
      double uk = 0.;                           // uk = dB_p y ; dB = -dA (:1576)
      for (int a = 0; a < f.k; ++a) uk -= f.dA[p][a] * y[nb[a]];
      sums[2 + p] += uk * u - 0.5 * u * f.dD[p] * u;     // :1786
      sums[2 + P + p] += Dinv * f.dD[p];                  // :1787
    }
  }
  return 0;
}

int orc_vecchia_nll_grad(const double* coords, const double* y, const int* nbr,
                         int n, int d, int m, int t, const double* pars, int mode,
                         double* nll, double* grad, double* sigma2_out,
                         double* Dinv, double* Bvals) {
  const int P = num_pars_grad();
  std::vector<double> s(2 + 2 * P);
  if (orc_vecchia_partials(coords, y, nbr, n, d, m, t, pars, 0, n, s.data())) return -1;
  if (Dinv || Bvals) {
    RowFactor f;
    for (int i = 0; i < n; ++i) {
      row_factor(coords, nbr + (size_t)i * m, i, d, m, t, pars[1], pars[2], f);
      if (Dinv) Dinv[i] = 1. / f.D;
      if (Bvals) for (int a = 0; a < m; ++a) Bvals[(size_t)i * m + a] = a < f.k ? -f.A[a] : 0.;
    }
  }
  const double logdet = s[0], q = s[1];
  double sigma2 = pars[0];
  if (mode == 1) sigma2 = q / n;               // ProfileOutSigma2 (re_model_template.h:2407)
  *sigma2_out = sigma2;
  *nll = q / 2. / sigma2 + logdet / 2. + n / 2. * (std::log(sigma2) + std::log(2 * M_PI));  // :2880
  int off = 0;
  if (mode == 0) {
    grad[0] = -q / sigma2 / 2. + n / 2.;        // :1774
    off = 1;
  }
  for (int p = 0; p < P; ++p) grad[off + p] = s[2 + p] / sigma2 + 0.5 * s[2 + P + p];
  return 0;
}

int orc_dense_nll_grad(const double* x, const double* y, int n, int d, int t,
                       const double* pars, int mode, double* nll, double* grad, double* sigma2_out) {
  const double var = pars[1], phi = pars[2];
  std::vector<double> S((size_t)n * n), dS((size_t)n * n);
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) {
      if (i == j) { S[(size_t)i * n + j] = var; dS[(size_t)i * n + j] = 0.; continue; }
      double r = dist(x + (size_t)i * d, x + (size_t)j * d, d);
      S[(size_t)i * n + j] = cov(t, r, var, phi);           // cov_fcts.h:564-679
      dS[(size_t)i * n + j] = dcov_dlogphi(t, r, var, phi);  // cov_fcts.h:1000-1102
    }
  std::vector<double> L = S;
  for (int i = 0; i < n; ++i) L[(size_t)i * n + i] += kNugget;  // CalcZSigmaZt + I (:8430-8441)
  if (!chol(L, n)) return -1;                                   // CalcChol (:5902)
  std::vector<double> yaux(y, y + n);
  chol_solve(L, n, yaux.data());                                 // CalcYAux (:9007)
  double q = 0., logdet = 0.;
  for (int i = 0; i < n; ++i) { q += y[i] * yaux[i]; logdet += 2. * std::log(L[(size_t)i * n + i]); }
  double sigma2 = pars[0];
  if (mode == 1) sigma2 = q / n;
  *sigma2_out = sigma2;
  *nll = q / 2. / sigma2 + logdet / 2. + n / 2. * (std::log(sigma2) + std::log(2 * M_PI));
  // Psi^-1 explicitly, column by column (CalcPsiInv :5987-6007)
  std::vector<double> Pinv((size_t)n * n);
  std::vector<double> e(n);
  for (int j = 0; j < n; ++j) {
    std::fill(e.begin(), e.end(), 0.);
    e[j] = 1.;
    chol_solve(L, n, e.data());
    for (int i = 0; i < n; ++i) Pinv[(size_t)i * n + j] = e[i];
  }
  int off = 0;
  if (mode == 0) { grad[0] = -q / sigma2 / 2. + n / 2.; off = 1; }   // :1806
  for (int p = 0; p < 2; ++p) {
    const std::vector<double>& G = (p == 0) ? S : dS;               // GetZSigmaZtGrad (re_comp.h:1389)
    double quad = 0., tr = 0.;
    for (int i = 0; i < n; ++i) {
      double gi = 0.;
      for (int j = 0; j < n; ++j) {
        gi += G[(size_t)i * n + j] * yaux[j];
        tr += G[(size_t)i * n + j] * Pinv[(size_t)j * n + i];
      }
      quad += yaux[i] * gi;
    }
    grad[off + p] = -0.5 * quad / sigma2 + 0.5 * tr;              // :1813-1814
  }
  return 0;
}

}  // extern "C"
