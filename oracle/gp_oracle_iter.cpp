// ORACLE TEST INFRASTRUCTURE — NOT PART OF THE PRODUCT.
//
// CPU restatement of the reference's LATENT Vecchia path with iterative methods
// (matrix_inversion_method = "iterative", cg_preconditioner_type = "vadu"):
//   * latent Vecchia factor B, D^-1 and range derivatives   Vecchia_utils.cpp:1307-1632
//     (gauss_likelihood = false: no nugget, diagonal jitter, D starts at 0)
//   * Laplace mode finding (Newton + PCG + Armijo)           likelihoods.h:2765-3076
//   * PCG with the VADU preconditioner                       CG_utils.cpp:21-108
//   * probe vectors                                          CG_utils.cpp:930-947
//   * block PCG + Lanczos tridiagonals (SLQ)                  CG_utils.cpp:110-217
//   * stochastic log-determinant                             CG_utils.cpp:988-1004,
//                                                            likelihoods.h:12069-12212
//   * gradient with control variates                         likelihoods.h:4951-5206,
//     12225-12378 (mode), 12393-12465 (cov pars), 12477-12546 (aux pars),
//     CG_utils.cpp:1006-1041 (optimal c)
// Likelihoods: "gaussian" under gp_approx = "vecchia_latent" (aux par = error variance)
// and "bernoulli_logit". Plain sequential loops (no Eigen, no OpenMP in the math) so that
// it is an independent statement of the algorithm; the random probes use the same
// std::seed_seq / std::mt19937 / std::normal_distribution<double> as the reference.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <limits>
#include <random>
#include <vector>

#include "gp_oracle.h"
#include "orc_math.h"

namespace {

constexpr double kJitterMultVecchia = 1. + 1e-10;  // JITTER_MULT_VECCHIA (utils.h)
constexpr double kZeroRhsThreshold = 1e-100;       // ZERO_RHS_CG_THRESHOLD (utils.h:45)
constexpr double kCArmijo = 1e-4;                  // c_armijo_ (likelihoods.h:12737)

using Vec = std::vector<double>;

// Latent Vecchia factor: B(i, nbr) = Bv[i*m + r], D^-1, dB/dlog(phi), dD/dlog(phi).
struct Factor {
  int n = 0, m = 0;
  std::vector<int> k;      // neighbours per row
  const int* nbr = nullptr;
  Vec Bv, dBv, Dinv, dD;
};

// Vecchia_utils.cpp:1496-1617 with gauss_likelihood = false (single GP, transf_scale):
// D_ii = sigma1^2 - A_i c_i, between-neighbour diagonal *= JITTER_MULT_VECCHIA (:1547),
// the marginal-variance derivative is excluded (exclude_marg_var_grad), range derivative
// dA = C^-1 dc - A dC C^-1, dD = -(dA c + A dc) (:1573-1585).
bool latent_factor(const double* x, const int* nbr, int n, int d, int m, int ct, double var, double phi,
                   Factor& F) {
  F.n = n; F.m = m; F.nbr = nbr;
  F.k.assign(n, 0);
  F.Bv.assign((size_t)n * m, 0.);
  F.dBv.assign((size_t)n * m, 0.);
  F.Dinv.assign(n, 0.);
  F.dD.assign(n, 0.);
  for (int i = 0; i < n; ++i) {
    const int k = std::min(i, m);
    F.k[i] = k;
    double D = var;
    double dD = 0.;
    if (k > 0) {
      const int* nb = nbr + (size_t)i * m;
      const double* xi = x + (size_t)i * d;
      Vec c(k), dc(k), C((size_t)k * k), dC((size_t)k * k);
      for (int a = 0; a < k; ++a) {
        const double* xa = x + (size_t)nb[a] * d;
        const double r = dist(xi, xa, d);
        c[a] = cov(ct, r, var, phi);
        dc[a] = dcov_dlogphi(ct, r, var, phi);
        for (int b = 0; b < k; ++b) {
          if (a == b) { C[a * k + a] = var * kJitterMultVecchia; dC[a * k + a] = 0.; continue; }
          const double rab = dist(xa, x + (size_t)nb[b] * d, d);
          C[a * k + b] = cov(ct, rab, var, phi);
          dC[a * k + b] = dcov_dlogphi(ct, rab, var, phi);
        }
      }
      Vec L = C;
      if (!chol(L, k)) return false;
      Vec A = c;
      chol_solve(L, k, A.data());
      Vec w(k, 0.);
      for (int b = 0; b < k; ++b) {
        double s = 0.;
        for (int a = 0; a < k; ++a) s += A[a] * dC[a * k + b];
        w[b] = s;
      }
      chol_solve(L, k, w.data());
      Vec s = dc;
      chol_solve(L, k, s.data());
      double Ac = 0., dAc = 0., Adc = 0.;
      for (int a = 0; a < k; ++a) {
        const double dA = s[a] - w[a];
        F.Bv[(size_t)i * m + a] = -A[a];
        F.dBv[(size_t)i * m + a] = -dA;
        Ac += A[a] * c[a];
        dAc += dA * c[a];
        Adc += A[a] * dc[a];
      }
      D -= Ac;
      dD = -(dAc + Adc);
    }
    if (!(D > 0.)) return false;
    F.Dinv[i] = 1. / D;
    F.dD[i] = dD;
  }
  return true;
}

// ---- sparse operators (Vecchia order; B unit lower triangular)
void B_apply(const Factor& F, const Vec& vals, bool unit, const double* x, double* y) {
  for (int i = 0; i < F.n; ++i) {
    double s = unit ? x[i] : 0.;
    for (int r = 0; r < F.k[i]; ++r) s += vals[(size_t)i * F.m + r] * x[F.nbr[(size_t)i * F.m + r]];
    y[i] = s;
  }
}
void Bt_apply(const Factor& F, const Vec& vals, bool unit, const double* x, double* y) {
  for (int j = 0; j < F.n; ++j) y[j] = unit ? x[j] : 0.;
  for (int i = 0; i < F.n; ++i)
    for (int r = 0; r < F.k[i]; ++r) y[F.nbr[(size_t)i * F.m + r]] += vals[(size_t)i * F.m + r] * x[i];
}
// (B^T D^-1 B + diag(W)) x   (CG_utils.cpp:75)
void A_apply(const Factor& F, const Vec& W, const double* x, double* y) {
  Vec t(F.n), g(F.n);
  B_apply(F, F.Bv, true, x, t.data());
  for (int i = 0; i < F.n; ++i) g[i] = F.Dinv[i] * t[i];
  Bt_apply(F, F.Bv, true, g.data(), y);
  for (int i = 0; i < F.n; ++i) y[i] += W[i] * x[i];
}
// VADU: z = ((D^-1 + W) B)^-1 B^-T r   (CG_utils.cpp:56-60)
void vadu_solve(const Factor& F, const Vec& dw, const double* r, double* z) {
  Vec y(r, r + F.n);
  for (int i = F.n - 1; i >= 0; --i)          // B^T unit upper: back substitution by columns
    for (int a = 0; a < F.k[i]; ++a) y[F.nbr[(size_t)i * F.m + a]] -= F.Bv[(size_t)i * F.m + a] * y[i];
  for (int i = 0; i < F.n; ++i) {              // (dw B) lower: forward substitution
    double s = y[i] / dw[i];
    for (int a = 0; a < F.k[i]; ++a) s -= F.Bv[(size_t)i * F.m + a] * z[F.nbr[(size_t)i * F.m + a]];
    z[i] = s;
  }
}
double dot(const double* a, const double* b, int n) {
  double s = 0.;
  for (int i = 0; i < n; ++i) s += a[i] * b[i];
  return s;
}

// CG_utils.cpp:21-108 (single right-hand side). Returns false on NaN/Inf.
bool pcg(const Factor& F, const Vec& W, const Vec& dw, const Vec& rhs, Vec& u, int p, bool init_zero,
         double delta, int* iters) {
  const int n = F.n;
  p = std::min(p, n);
  double l1 = 0.;
  for (double v : rhs) l1 += std::fabs(v);
  *iters = 0;
  if (l1 < kZeroRhsThreshold) { u.assign(n, 0.); return true; }
  Vec r(n), z(n), h(n), v(n), r_old, z_old;
  bool u_zero = true;
  for (double x : u) if (x != 0.) { u_zero = false; break; }
  if (init_zero || u_zero) {
    u.assign(n, 0.);
    r = rhs;
  } else {
    A_apply(F, W, u.data(), v.data());
    for (int i = 0; i < n; ++i) r[i] = rhs[i] - v[i];
  }
  vadu_solve(F, dw, r.data(), z.data());
  h = z;
  for (int j = 0; j < p; ++j) {
    A_apply(F, W, h.data(), v.data());
    const double a = dot(r.data(), z.data(), n) / dot(h.data(), v.data(), n);
    for (int i = 0; i < n; ++i) u[i] += a * h[i];
    r_old = r;
    for (int i = 0; i < n; ++i) r[i] -= a * v[i];
    const double rn = std::sqrt(dot(r.data(), r.data(), n));
    *iters = j + 1;
    if (std::isnan(rn) || std::isinf(rn)) return false;
    if (rn < delta) return true;
    z_old = z;
    vadu_solve(F, dw, r.data(), z.data());
    const double b = dot(r.data(), z.data(), n) / dot(r_old.data(), z_old.data(), n);
    for (int i = 0; i < n; ++i) h[i] = z[i] + b * h[i];
  }
  return true;
}

// CG_utils.cpp:110-217: block PCG on t columns (column-major n x t), Lanczos coefficients.
bool pcg_tridiag(const Factor& F, const Vec& W, const Vec& dw, const Vec& RHS, int t, int p, double delta,
                 Vec& U, std::vector<Vec>& Td, std::vector<Vec>& Ts) {
  const int n = F.n;
  p = std::min(p, n);
  Vec R = RHS, Z((size_t)n * t), H, V((size_t)n * t), R_old, Z_old;
  U.assign((size_t)n * t, 0.);
  Vec a(t, 1.), a_old(t), b(t, 0.), b_old(t);
  Td.assign(t, Vec());
  Ts.assign(t, Vec());
  for (int c = 0; c < t; ++c) vadu_solve(F, dw, &R[(size_t)c * n], &Z[(size_t)c * n]);
  H = Z;
  for (int j = 0; j < p; ++j) {
    for (int c = 0; c < t; ++c) A_apply(F, W, &H[(size_t)c * n], &V[(size_t)c * n]);
    a_old = a;
    for (int c = 0; c < t; ++c)
      a[c] = dot(&R[(size_t)c * n], &Z[(size_t)c * n], n) / dot(&H[(size_t)c * n], &V[(size_t)c * n], n);
    for (int c = 0; c < t; ++c)
      for (int i = 0; i < n; ++i) U[(size_t)c * n + i] += H[(size_t)c * n + i] * a[c];
    R_old = R;
    for (int c = 0; c < t; ++c)
      for (int i = 0; i < n; ++i) R[(size_t)c * n + i] -= V[(size_t)c * n + i] * a[c];
    double mean_norm = 0.;
    for (int c = 0; c < t; ++c) mean_norm += std::sqrt(dot(&R[(size_t)c * n], &R[(size_t)c * n], n));
    mean_norm /= t;
    if (std::isnan(mean_norm) || std::isinf(mean_norm)) return false;
    const bool stop = mean_norm < delta;
    Z_old = Z;
    for (int c = 0; c < t; ++c) vadu_solve(F, dw, &R[(size_t)c * n], &Z[(size_t)c * n]);
    b_old = b;
    for (int c = 0; c < t; ++c)
      b[c] = dot(&R[(size_t)c * n], &Z[(size_t)c * n], n) / dot(&R_old[(size_t)c * n], &Z_old[(size_t)c * n], n);
    for (int c = 0; c < t; ++c)
      for (int i = 0; i < n; ++i) H[(size_t)c * n + i] = Z[(size_t)c * n + i] + H[(size_t)c * n + i] * b[c];
    for (int c = 0; c < t; ++c) {
      Td[c].push_back(1. / a[c] + b_old[c] / a_old[c]);
      if (j > 0) Ts[c].push_back(std::sqrt(b_old[c]) / a_old[c]);
    }
    if (stop) return true;
  }
  return true;
}

// Symmetric tridiagonal eigen-decomposition by implicit QL with Wilkinson shifts,
// accumulating the full eigenvector matrix (columns = eigenvectors). diag d (k), off e (k-1).
void tridiag_eigen(Vec d, Vec e, Vec& lam, Vec& Q) {
  const int k = (int)d.size();
  Q.assign((size_t)k * k, 0.);
  for (int i = 0; i < k; ++i) Q[(size_t)i * k + i] = 1.;
  e.push_back(0.);
  for (int l = 0; l < k; ++l) {
    for (int iter = 0; iter < 200; ++iter) {
      int mm = l;
      for (; mm < k - 1; ++mm) {
        const double dd = std::fabs(d[mm]) + std::fabs(d[mm + 1]);
        if (std::fabs(e[mm]) <= std::numeric_limits<double>::epsilon() * dd) break;
      }
      if (mm == l) break;
      double g = (d[l + 1] - d[l]) / (2. * e[l]);
      double r = std::hypot(g, 1.);
      g = d[mm] - d[l] + e[l] / (g + (g >= 0 ? r : -r));
      double s = 1., c = 1., pp = 0.;
      int i = mm - 1;
      for (; i >= l; --i) {
        double f = s * e[i], b = c * e[i];
        r = std::hypot(f, g);
        e[i + 1] = r;
        if (r == 0.) { d[i + 1] -= pp; e[mm] = 0.; break; }
        s = f / r; c = g / r;
        g = d[i + 1] - pp;
        r = (d[i] - g) * s + 2. * c * b;
        pp = s * r;
        d[i + 1] = g + pp;
        g = c * r - b;
        for (int q = 0; q < k; ++q) {   // rotate columns i, i+1 of Q
          f = Q[(size_t)q * k + i + 1];
          Q[(size_t)q * k + i + 1] = s * Q[(size_t)q * k + i] + c * f;
          Q[(size_t)q * k + i] = c * Q[(size_t)q * k + i] - s * f;
        }
      }
      if (r == 0. && i >= l) continue;
      d[l] -= pp; e[l] = g; e[mm] = 0.;
    }
  }
  lam = d;
}

// CG_utils.cpp:988-1004
double logdet_stoch_tridiag(const std::vector<Vec>& Td, const std::vector<Vec>& Ts, int n, int t) {
  double ld = 0.;
  for (int c = 0; c < t; ++c) {
    Vec lam, Q;
    tridiag_eigen(Td[c], Ts[c], lam, Q);
    const int k = (int)lam.size();
    for (int j = 0; j < k; ++j) ld += Q[j] * std::log(lam[j]) * Q[j];   // row 0 of Q
  }
  return ld * n / t;
}

// CG_utils.cpp:1006-1024
double optimal_c(const Vec& zA, const Vec& zB, double trA, double trB) {
  double den = 0., num = 0.;
  for (size_t c = 0; c < zB.size(); ++c) den += (zB[c] - trB) * (zB[c] - trB);
  den /= zB.size();
  if (den == 0.) return 1.;
  for (size_t c = 0; c < zB.size(); ++c) num += (zA[c] - trA) * (zB[c] - trB);
  num /= zB.size();
  return num / den;
}
double mean(const Vec& v) {
  double s = 0.;
  for (double x : v) s += x;
  return s / v.size();
}

// ---- likelihoods (likelihoods.h: gaussian :8795, 9263, 9937, 10586, 10967;
//      bernoulli_logit :8724, 9226, 9896, 10187; DF_utils.h:37-60)
double sigmoid_stable(double x) {
  if (x >= 0.) { const double t = std::exp(-x); return 1. / (1. + t); }
  const double t = std::exp(x);
  return t / (1. + t);
}
double softplus(double x) { return std::log1p(std::exp(-std::fabs(x))) + std::max(x, 0.); }

struct Lik {
  int type;       // ORC_LIK_GAUSSIAN | ORC_LIK_BERNOULLI_LOGIT
  double s2;      // gaussian error variance (aux par)
  double loglik(const double* y, const Vec& loc) const {
    double ll = 0.;
    for (size_t i = 0; i < loc.size(); ++i) {
      if (type == ORC_LIK_GAUSSIAN) {
        const double r = y[i] - loc[i];
        ll += -r * r / 2. / s2 - 0.91893853320467274178 - 0.5 * std::log(s2);
      } else {
        ll += y[i] * loc[i] - softplus(loc[i]);
      }
    }
    return ll;
  }
  double d1(double y, double l) const { return type == ORC_LIK_GAUSSIAN ? (y - l) / s2 : y - sigmoid_stable(l); }
  double info(double l) const {
    if (type == ORC_LIK_GAUSSIAN) return 1. / s2;
    const double p = sigmoid_stable(l);
    return p * (1. - p);
  }
  double dinfo(double l) const {    // derivative of the information wrt the location
    if (type == ORC_LIK_GAUSSIAN) return 0.;
    const double p = sigmoid_stable(l);
    return -p * (1. - p) * (2. * p - 1.);
  }
  bool info_changes() const { return type != ORC_LIK_GAUSSIAN; }
  int maxit() const { return type == ORC_LIK_GAUSSIAN ? 1 : 1000; }
  int max_shrink() const { return type == ORC_LIK_GAUSSIAN ? 1 : 20; }
};

double quad_SigmaI(const Factor& F, const Vec& x) {   // x^T B^T D^-1 B x
  Vec bx(F.n);
  B_apply(F, F.Bv, true, x.data(), bx.data());
  double s = 0.;
  for (int i = 0; i < F.n; ++i) s += bx[i] * F.Dinv[i] * bx[i];
  return s;
}

// SigmaI_deriv * x for parameter p (0: variance -> -Sigma^-1, 1: range), likelihoods.h:5036-5063
void SigmaI_deriv_apply(const Factor& F, int p, const Vec& x, Vec& y) {
  const int n = F.n;
  Vec bx(n), dbx(n), g(n), tmp(n);
  B_apply(F, F.Bv, true, x.data(), bx.data());
  if (p == 0) {
    for (int i = 0; i < n; ++i) g[i] = -F.Dinv[i] * bx[i];
    Bt_apply(F, F.Bv, true, g.data(), y.data());
    return;
  }
  B_apply(F, F.dBv, false, x.data(), dbx.data());
  // dB^T D^-1 B x + B^T D^-1 dB x - B^T D^-1 dD D^-1 B x
  for (int i = 0; i < n; ++i) g[i] = F.Dinv[i] * bx[i];
  Bt_apply(F, F.dBv, false, g.data(), y.data());
  for (int i = 0; i < n; ++i) g[i] = F.Dinv[i] * dbx[i] - F.Dinv[i] * F.dD[i] * F.Dinv[i] * bx[i];
  Bt_apply(F, F.Bv, true, g.data(), tmp.data());
  for (int i = 0; i < n; ++i) y[i] += tmp[i];
}

}  // namespace

extern "C" {

int orc_latent_vecchia_factor(const double* coords_vo, const int* nbr, int n, int d, int m, int cov_type,
                              const double* trafo, double* Bv, double* dBv, double* Dinv, double* dD) {
  Factor F;
  if (!latent_factor(coords_vo, nbr, n, d, m, cov_type, trafo[0], trafo[1], F)) return -1;
  std::copy(F.Bv.begin(), F.Bv.end(), Bv);
  std::copy(F.dBv.begin(), F.dBv.end(), dBv);
  std::copy(F.Dinv.begin(), F.Dinv.end(), Dinv);
  std::copy(F.dD.begin(), F.dD.end(), dD);
  return 0;
}

void orc_gen_probes(int n, int t, int seed, unsigned long long run_id, double* R) {
  // CG_utils.cpp:930-947; R column-major n x t
  const uint32_t b32 = static_cast<uint32_t>(seed);
  for (int c = 0; c < t; ++c) {
    std::normal_distribution<double> nd(0., 1.);
    std::seed_seq seq{b32, static_cast<uint32_t>(run_id), static_cast<uint32_t>(run_id >> 32), static_cast<uint32_t>(c)};
    std::mt19937 gen(seq);
    for (int i = 0; i < n; ++i) R[(size_t)c * n + i] = nd(gen);
  }
}

int orc_latent_vecchia_iterative(const double* coords_vo, const double* y_vo, const int* nbr, int n, int d, int m,
                                 int cov_type, const double* trafo, int likelihood, double aux, int t, int seed,
                                 double cg_delta_conv, int cg_max_num_it, int cg_max_num_it_tridiag, int want_grad,
                                 double* nll, double* grad, double* info) {
  Factor F;
  if (!latent_factor(coords_vo, nbr, n, d, m, cov_type, trafo[0], trafo[1], F)) return -1;
  const Lik L{likelihood, aux};
  // ---- mode finding, likelihoods.h:2765-2995 (mode initialised to 0 per call)
  Vec mode(n, 0.), loc(n, 0.), W(n), d1(n), rhs(n), mode_update(n, 0.), mode_new(n), dw(n), bx(n), tmp(n);
  double mll = L.loglik(y_vo, loc) - 0.5 * quad_SigmaI(F, mode);
  double mll_new = mll;
  int newton_its = 0, cg_its_total = 0;
  for (int it = 0; it < L.maxit(); ++it) {
    for (int i = 0; i < n; ++i) d1[i] = L.d1(y_vo[i], loc[i]);
    if (it == 0 || L.info_changes())
      for (int i = 0; i < n; ++i) W[i] = L.info(loc[i]);
    for (int i = 0; i < n; ++i) rhs[i] = W[i] * mode[i] + d1[i];
    if (it == 0 || L.info_changes())
      for (int i = 0; i < n; ++i) dw[i] = F.Dinv[i] + W[i];
    int its = 0;
    if (!pcg(F, W, dw, rhs, mode_update, cg_max_num_it, it == 0, cg_delta_conv, &its)) return -2;
    cg_its_total += its;
    // Armijo, likelihoods.h:2957-2994
    Vec dir(n), gvec(n);
    for (int i = 0; i < n; ++i) dir[i] = mode_update[i] - mode[i];
    A_apply(F, W, dir.data(), gvec.data());
    const double gdd = dot(dir.data(), gvec.data(), n);
    double lr = 1.;
    for (int ih = 0; ih < L.max_shrink(); ++ih) {
      for (int i = 0; i < n; ++i) mode_new[i] = (ih == 0) ? mode_update[i] : (1 - lr) * mode[i] + lr * mode_update[i];
      loc = mode_new;
      mll_new = L.loglik(y_vo, loc) - 0.5 * quad_SigmaI(F, mode_new);
      if (mll_new < mll + kCArmijo * lr * gdd || std::isnan(mll_new) || std::isinf(mll_new)) lr *= 0.5;
      else break;
    }
    mode = mode_new;
    newton_its = it + 1;
    // CheckConvergenceModeFinding, likelihoods.h:11820-11870
    if (std::isnan(mll_new) || std::isinf(mll_new)) return -3;
    bool term = (it == 0) ? std::fabs(mll_new - mll) < 1e-8 * std::fabs(mll) : (mll_new - mll) < 1e-8 * std::fabs(mll);
    mll = mll_new;
    if (term) break;
  }
  for (int i = 0; i < n; ++i) d1[i] = L.d1(y_vo[i], loc[i]);
  if (L.info_changes()) for (int i = 0; i < n; ++i) W[i] = L.info(loc[i]);
  // ---- SLQ log-determinant, likelihoods.h:3018-3045, 12155-12212
  Vec Rn((size_t)n * t);
  orc_gen_probes(n, t, seed, 0ull, Rn.data());
  for (int i = 0; i < n; ++i) dw[i] = F.Dinv[i] + W[i];
  Vec Zp((size_t)n * t), sc(n);
  for (int c = 0; c < t; ++c) {
    for (int i = 0; i < n; ++i) sc[i] = std::sqrt(dw[i]) * Rn[(size_t)c * n + i];
    Bt_apply(F, F.Bv, true, sc.data(), &Zp[(size_t)c * n]);
  }
  Vec U;
  std::vector<Vec> Td, Ts;
  if (!pcg_tridiag(F, W, dw, Zp, t, cg_max_num_it_tridiag, cg_delta_conv, U, Td, Ts)) return -4;
  double ldet = logdet_stoch_tridiag(Td, Ts, n, t);
  for (int i = 0; i < n; ++i) ldet += -std::log(F.Dinv[i]) + std::log(dw[i]);
  mll -= 0.5 * ldet;
  *nll = -mll;
  if (info) {
    info[0] = newton_its;
    info[1] = cg_its_total;
    info[2] = (double)Td[0].size();
    info[3] = ldet;
  }
  if (!want_grad) return 0;

  // ---- gradient, likelihoods.h:4951-5206
  const bool gi_nonzero = L.info_changes();   // grad_information_wrt_mode_non_zero_
  Vec PI_Z((size_t)n * t), BPZ((size_t)n * t), dBPZ((size_t)n * t), BU((size_t)n * t), dBU((size_t)n * t);
  for (int c = 0; c < t; ++c) {
    vadu_solve(F, dw, &Zp[(size_t)c * n], &PI_Z[(size_t)c * n]);
    B_apply(F, F.Bv, true, &PI_Z[(size_t)c * n], &BPZ[(size_t)c * n]);
    B_apply(F, F.dBv, false, &PI_Z[(size_t)c * n], &dBPZ[(size_t)c * n]);
    B_apply(F, F.Bv, true, &U[(size_t)c * n], &BU[(size_t)c * n]);
    B_apply(F, F.dBv, false, &U[(size_t)c * n], &dBU[(size_t)c * n]);
  }
  Vec dwinv(n);
  for (int i = 0; i < n; ++i) dwinv[i] = 1. / dw[i];
  Vec vS(n, 0.);   // (Sigma^-1 + W)^-1 d_mll_d_mode
  if (gi_nonzero) {
    // CalcLogDetStochDerivModeVecchia, likelihoods.h:12320-12341 (vadu)
    Vec dW(n);
    for (int i = 0; i < n; ++i) dW[i] = L.dinfo(loc[i]);
    Vec dmode(n);
    for (int i = 0; i < n; ++i) {
      double tr1 = 0., trP = 0.;
      Vec z1(t), zP(t);
      for (int c = 0; c < t; ++c) {
        z1[c] = U[(size_t)c * n + i] * dW[i] * PI_Z[(size_t)c * n + i];
        zP[c] = BPZ[(size_t)c * n + i] * dW[i] * BPZ[(size_t)c * n + i];
        tr1 += z1[c]; trP += zP[c];
      }
      tr1 /= t; trP /= t;
      double cv = 0., vv = 0.;
      for (int c = 0; c < t; ++c) { cv += (z1[c] - tr1) * (zP[c] - trP); vv += (zP[c] - trP) * (zP[c] - trP); }
      cv /= t; vv /= t;
      const double copt = (vv == 0.) ? 1. : cv / vv;
      dmode[i] = tr1 + copt * (dwinv[i] * dW[i]) - copt * trP;
    }
    Vec dmll(n);
    for (int i = 0; i < n; ++i) dmll[i] = 0.5 * dmode[i];
    int its = 0;
    pcg(F, W, dw, dmll, vS, cg_max_num_it, true, cg_delta_conv, &its);
  }
  // covariance parameters, likelihoods.h:5028-5103, 12440-12465
  for (int p = 0; p < 2; ++p) {
    Vec z1(t), zP(t);
    double trD = 0., ddiag = 0.;
    for (int c = 0; c < t; ++c) {
      double s1 = 0., sP = 0.;
      for (int i = 0; i < n; ++i) {
        const size_t q = (size_t)c * n + i;
        if (p == 0) {
          s1 += -F.Dinv[i] * BU[q] * BPZ[q];
          sP += -F.Dinv[i] * BPZ[q] * BPZ[q];
        } else {
          const double Di = F.Dinv[i];
          s1 += Di * (dBU[q] * BPZ[q] + BU[q] * dBPZ[q] - Di * F.dD[i] * BU[q] * BPZ[q]);
          sP += Di * (2. * dBPZ[q] * BPZ[q] - Di * F.dD[i] * BPZ[q] * BPZ[q]) + 2. * W[i] * BPZ[q] * dBPZ[q];
        }
      }
      z1[c] = s1; zP[c] = sP;
    }
    for (int i = 0; i < n; ++i) {
      if (p == 0) { trD += -dwinv[i] * F.Dinv[i]; }
      else { trD += -dwinv[i] * F.Dinv[i] * F.dD[i] * F.Dinv[i]; ddiag += F.Dinv[i] * F.dD[i]; }
    }
    const double tr1 = mean(z1), trP = mean(zP);
    double dld = tr1 + (p == 0 ? (double)n : ddiag);
    const double copt = optimal_c(z1, zP, tr1, trP);
    dld += copt * trD - copt * trP;
    Vec Sm(n);
    SigmaI_deriv_apply(F, p, mode, Sm);
    grad[p] = 0.5 * (dot(mode.data(), Sm.data(), n) + dld);
    if (gi_nonzero) grad[p] -= dot(vS.data(), Sm.data(), n);
  }
  // auxiliary parameter (gaussian error variance, log scale), likelihoods.h:5166-5200, 12520-12546
  if (likelihood == ORC_LIK_GAUSSIAN) {
    double rss = 0.;
    for (int i = 0; i < n; ++i) { const double r = y_vo[i] - loc[i]; rss += r * r; }
    const double neg_ll_deriv = rss * (-0.5 / aux) + 0.5 * n;
    const double dWa = -1. / aux;
    Vec z1(t), zP(t);
    for (int c = 0; c < t; ++c) {
      double s1 = 0., sP = 0.;
      for (int i = 0; i < n; ++i) {
        const size_t q = (size_t)c * n + i;
        s1 += U[q] * dWa * PI_Z[q];
        sP += BPZ[q] * dWa * BPZ[q];
      }
      z1[c] = s1; zP[c] = sP;
    }
    double trD = 0.;
    for (int i = 0; i < n; ++i) trD += dwinv[i] * dWa;
    const double tr1 = mean(z1), trP = mean(zP);
    const double copt = optimal_c(z1, zP, tr1, trP);
    const double dd = tr1 + copt * trD - copt * trP;
    grad[2] = neg_ll_deriv + 0.5 * dd;
  }
  return 0;
}

}  // extern "C"
