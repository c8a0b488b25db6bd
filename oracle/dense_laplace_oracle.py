"""ORACLE TEST INFRASTRUCTURE — NOT PART OF THE PRODUCT.

CPU restatement (numpy, dense algebra) of the reference's Laplace approximation for a GP without an
approximation (gp_approx = "none"), the checker of gpboost_amd's DenseLaplace (csrc/dense_laplace.h).
Importable only from tests/. Follows
  FindModePostRandEffCalcMLLStable               likelihoods.h:1843-1960 (Newton on a = Sigma^-1 mode with
      B = I + W^1/2 Sigma W^1/2 = L L^T, Armijo c = 1e-4 with up to 20 halvings, CheckConvergenceModeFinding
      :11820-11870, mll = -1/2 a^T mode + log p(y | mode + F) - sum log L_ii)
  CalcGradNegMargLikelihoodLaplaceApproxStable   likelihoods.h:3261-3413 (explicit -1/2 a^T dSigma a
      + 1/2 tr((W^-1 + Sigma)^-1 dSigma), implicit d_mll_d_mode^T (dSigma d1 - Sigma (W^-1 + Sigma)^-1 dSigma d1)
      with d_mll_d_mode = 1/2 diag((Sigma^-1 + W)^-1) o dW/dmode; fixed-effect gradient)
  PredictLaplaceApproxStable                     likelihoods.h:5610-5676
The likelihood terms and covariance functions are oracle/fitc_laplace_oracle.py's. Pinned to the reference by
tests/test_oracle_dense_laplace.py.
"""
from __future__ import annotations

import numpy as np
from scipy.special import gammaln

from oracle.fitc_laplace_oracle import _dist, _lik, cov_dcov


def _lik_any(lik, y, l, aux):
    """_lik plus likelihood 'gamma' with shape aux (likelihoods.h:8740, 9234, 9908, 10228)."""
    if lik != "gamma":
        return _lik(lik, y, l)
    e = y * np.exp(-l)
    return float(np.sum(-aux * (l + e))), aux * (e - 1.), aux * e, -aux * e


def _digamma(x):
    """AS 103 (the reference's GPBoost::digamma, DF_utils.cpp:82-123)."""
    if x <= 1e-6:
        return -0.57721566490153286060 - 1. / x + 1.6449340668482264365 * x
    v, x2 = 0., x
    while x2 < 8.5:
        v -= 1. / x2
        x2 += 1.
    r = 1. / x2
    v += np.log(x2) - 0.5 * r
    r *= r
    return v - r * (1. / 12 - r * (1. / 120 - r * (1. / 252 - r * (1. / 240 - r * (1. / 132)))))


class DenseLaplaceOracle:
    def __init__(self, X, y, cov_type, var, phi, likelihood, fixed_effects=None, delta=1e-8, aux=1.):
        self.X, self.y = np.asarray(X, float), np.asarray(y, float)
        self.lik, self.ct, self.var, self.phi, self.delta, self.aux = likelihood, cov_type, var, phi, delta, aux
        self.const = -float(gammaln(self.y + 1.).sum()) if likelihood == "poisson" else 0.
        if likelihood == "gamma" and abs(aux - 1.) >= 1e-10 * max(1., aux):   # :8431-8449
            n = len(self.y)
            self.const = (aux - 1.) * float(np.log(self.y).sum()) + n * (aux * np.log(aux) - gammaln(aux))
        self.F = np.zeros(len(self.y)) if fixed_effects is None else np.asarray(fixed_effects, float)
        D = _dist(self.X, self.X)
        self.S, self.dS = cov_dcov(D, var, phi, cov_type)
        np.fill_diagonal(self.S, var)
        np.fill_diagonal(self.dS, 0.)
        self._mode()

    def _obj(self, mode, a):
        return -0.5 * float(a @ mode) + _lik_any(self.lik, self.y, mode + self.F, self.aux)[0] + self.const

    def _mode(self):
        n = len(self.y)
        mode, a = np.zeros(n), np.zeros(n)
        obj = self._obj(mode, a)
        for it in range(1000):
            _, d1, w, _ = _lik_any(self.lik, self.y, mode + self.F, self.aux)
            ws = np.sqrt(w)
            B = np.eye(n) + ws[:, None] * self.S * ws[None, :]
            L = np.linalg.cholesky(B)
            rhs = w * mode + d1
            rhs2 = ws * (self.S @ rhs)
            t = np.linalg.solve(L.T, np.linalg.solve(L, rhs2))
            a_upd = rhs - ws * t
            m_upd = self.S @ a_upd
            direc = m_upd - mode
            gdd = float(direc @ (a_upd - a + w * direc))
            lam = 1.
            for _ in range(20):
                a_new = a_upd if lam == 1. else (1 - lam) * a + lam * a_upd
                m_new = m_upd if lam == 1. else (1 - lam) * mode + lam * m_upd
                obj_new = self._obj(m_new, a_new)
                if obj_new < obj + 1e-4 * lam * gdd or not np.isfinite(obj_new):
                    lam *= 0.5
                else:
                    break
            mode, a = m_new, a_new
            conv = abs(obj_new - obj) < self.delta * abs(obj) if it == 0 else (obj_new - obj) < self.delta * abs(obj)
            obj = obj_new
            if conv:
                break
        self.mode, self.a, self.obj = mode, a, obj
        _, self.d1, self.w, self.dw = _lik_any(self.lik, self.y, mode + self.F, self.aux)
        self.ws = np.sqrt(self.w)
        B = np.eye(n) + self.ws[:, None] * self.S * self.ws[None, :]
        self.L = np.linalg.cholesky(B)
        self.nll = -(obj - float(np.sum(np.log(np.diag(self.L)))))

    def grad(self):
        Q = np.linalg.solve(self.L, np.diag(self.ws))          # L^-1 W^1/2
        R = Q.T @ Q                                           # (W^-1 + Sigma)^-1
        C = Q @ self.S
        diag = np.diag(self.S) - (C * C).sum(0)
        dmll = 0.5 * diag * self.dw
        g = []
        for dS in (self.S, self.dS):
            u = dS @ self.d1
            g.append(-0.5 * float(self.a @ dS @ self.a) + 0.5 * float(np.sum(R * dS)) + float(dmll @ (u - self.S @ (R @ u))))
        v = self.S @ dmll - C.T @ (C @ dmll)
        gf = -self.d1 + dmll - self.w * v
        if self.lik == "gamma":   # shape on the log scale (:3379-3411, 10508-10524, 10856-10869)
            a, l, n = self.aux, self.mode + self.F, len(self.y)
            neg = a * (float(np.sum(l + self.y * np.exp(-l))) - n * (np.log(a) + 1. - _digamma(a))
                       - float(np.log(self.y).sum()))
            g.append(neg + 0.5 * float(self.w @ diag) + float(self.d1 @ v))
        return np.array(g), gf

    def predict(self, Xp, want_cov=False):
        Xp = np.asarray(Xp, float)
        Cp, _ = cov_dcov(_dist(self.X, Xp), self.var, self.phi, self.ct)
        Cp[_dist(self.X, Xp) == 0.] = self.var
        mean = Cp.T @ self.d1
        M = np.linalg.solve(self.L, self.ws[:, None] * Cp)
        if want_cov:
            Spp, _ = cov_dcov(_dist(Xp, Xp), self.var, self.phi, self.ct)
            np.fill_diagonal(Spp, self.var)
            return mean, Spp - M.T @ M
        return mean, self.var - (M * M).sum(0)
