"""ORACLE TEST INFRASTRUCTURE — NOT PART OF THE PRODUCT.

CPU restatement (numpy, dense algebra) of the reference's Laplace approximation for a latent Vecchia GP with
matrix_inversion_method = "cholesky", the checker of gpboost_amd's sparse-Cholesky path (csrc/latent_chol.cpp,
csrc/sparse_chol.{h,hip}). Importable only from tests/. Follows
  FindModePostRandEffCalcMLLVecchia, Cholesky branch   likelihoods.h:2780-3070
      (mode from 0; per Newton step SigmaI_plus_W = B^T D^-1 B + diag(W), mode_update = (SigmaI + W)^-1 (W mode + d1),
      Armijo with grad_dot_direction = dir^T (SigmaI + W) dir, c = 1e-4, up to 20 halvings (:2957-2995), the
      trial mode's change capped at log(100) for poisson / gamma (CapChangeModeUpdateNewton :11800-11810),
      CheckConvergenceModeFinding :11820-11870; approx_marginal_ll = log p(y | mode + F) - 1/2 (Bm)^T D^-1 (Bm)
      - sum log L_ii + 1/2 sum log D^-1_ii (:3067-3070))
  CalcGradNegMargLikelihoodLaplaceApproxVecchia, Cholesky branch   likelihoods.h:5207-5336
      (SigmaI_deriv = -SigmaI for the variance, dB^T D^-1 B + B^T D^-1 dB - B^T D^-1 dD D^-1 B for the range;
      explicit 1/2 (m^T SigmaI_deriv m + tr(SigmaI_deriv (SigmaI + W)^-1)) + n / 2 | 1/2 sum D^-1 dD; implicit
      - ((SigmaI + W)^-1 d_mll_d_mode)^T SigmaI_deriv m with d_mll_d_mode = 1/2 diag((SigmaI + W)^-1) o dW;
      gaussian error variance and gamma shape (:5304-5335); the gradient wrt F (:5337-5369))
with B, D^-1 and their range derivatives from the pinned C restatement of the latent Vecchia factor
(oracle.latent_factor, Vecchia_utils.cpp:1307-1632). Pinned to the reference by tests/test_oracle_latent_chol.py.
"""
from __future__ import annotations

import numpy as np
from scipy.special import gammaln

from oracle import oracle
from oracle.dense_laplace_oracle import _digamma, _lik_any


def _lik_all(lik, y, loc, aux):
    """(sum log p, d1, W, dW) including the Gaussian likelihood of "vecchia_latent" (aux = error variance)."""
    if lik == "gaussian":
        r = y - loc
        n = len(y)
        ll = float(np.sum(-r * r / 2. / aux)) - n * (0.91893853320467274178 + 0.5 * np.log(aux))
        return ll, r / aux, np.full(n, 1. / aux), np.zeros(n)
    return _lik_any(lik, y, loc, aux)


class LatentCholOracle:
    """Exact Laplace-Vecchia nll / gradient at (sigma1^2, phi) on the transformed scale (latent form, no nugget)."""

    def __init__(self, coords_vo, y_vo, nbr, cov_type, trafo2, likelihood, aux=1., fixed_effects=None, delta=1e-8):
        self.y = np.asarray(y_vo, float)
        n = len(self.y)
        f = oracle.latent_factor(coords_vo, nbr, cov_type, trafo2)
        m = nbr.shape[1]
        B = np.eye(n)
        dB = np.zeros((n, n))
        for i in range(1, n):
            k = min(i, m)
            B[i, nbr[i, :k]] = f["B"][i, :k]
            dB[i, nbr[i, :k]] = f["dB"][i, :k]
        self.B, self.dB, self.Dinv, self.dD = B, dB, f["Dinv"], f["dD"]
        self.lik, self.aux = likelihood, aux
        self.F = np.zeros(n) if fixed_effects is None else np.asarray(fixed_effects, float)
        self.const = -float(gammaln(self.y + 1.).sum()) if likelihood == "poisson" else 0.
        if likelihood == "gamma" and abs(aux - 1.) >= 1e-10 * max(1., aux):   # :8431-8449
            self.const = (aux - 1.) * float(np.log(self.y).sum()) + n * (aux * np.log(aux) - gammaln(aux))
        self.SigmaI = B.T @ (self.Dinv[:, None] * B)
        self._mode(delta)

    def _obj(self, mode):
        bm = self.B @ mode
        return _lik_all(self.lik, self.y, mode + self.F, self.aux)[0] + self.const - 0.5 * float(bm @ (self.Dinv * bm))

    def _mode(self, delta):
        n = len(self.y)
        mode = np.zeros(n)
        obj = self._obj(mode)
        gauss = self.lik == "gaussian"
        for it in range(1 if gauss else 1000):
            _, d1, w, _ = _lik_all(self.lik, self.y, mode + self.F, self.aux)
            A = self.SigmaI + np.diag(w)
            L = np.linalg.cholesky(A)
            upd = np.linalg.solve(L.T, np.linalg.solve(L, w * mode + d1))
            direc = upd - mode
            gdd = 0. if gauss else float(direc @ (A @ direc))
            lam = 1.
            for ih in range(1 if gauss else 20):
                new = upd if ih == 0 else (1 - lam) * mode + lam * upd
                if self.lik in ("poisson", "gamma"):   # CapChangeModeUpdateNewton (:11800-11810, log(100))
                    c = np.abs(new - mode)
                    big = c > np.log(100.)
                    new = np.where(big, mode + (new - mode) / np.where(big, c, 1.) * np.log(100.), new)
                obj_new = self._obj(new)
                if obj_new < obj + 1e-4 * lam * gdd or not np.isfinite(obj_new):
                    lam *= 0.5
                else:
                    break
            mode = new
            conv = abs(obj_new - obj) < delta * abs(obj) if it == 0 else (obj_new - obj) < delta * abs(obj)
            obj = obj_new
            if conv:
                break
        self.mode, self.obj = mode, obj
        _, self.d1, self.w, self.dw = _lik_all(self.lik, self.y, mode + self.F, self.aux)
        self.A = self.SigmaI + np.diag(self.w)
        self.L = np.linalg.cholesky(self.A)
        self.nll = -(obj - float(np.log(np.diag(self.L)).sum()) + 0.5 * float(np.log(self.Dinv).sum()))

    def grad(self):
        n = len(self.y)
        S = np.linalg.inv(self.A)
        S = 0.5 * (S + S.T)
        dmll = 0.5 * np.diag(S) * self.dw
        v = S @ dmll
        DB = self.Dinv[:, None] * self.B
        g = []
        for k in range(2):
            if k == 0:
                SId = -self.SigmaI
                expl = 0.5 * n
            else:
                SId = self.dB.T @ DB + DB.T @ self.dB - DB.T @ ((self.dD)[:, None] * DB)
                expl = 0.5 * float(np.sum(self.Dinv * self.dD))
            sm = SId @ self.mode
            gk = 0.5 * (float(self.mode @ sm) + float(np.sum(SId * S))) + expl
            if self.lik != "gaussian":
                gk -= float(v @ sm)
            g.append(gk)
        gf = -self.d1 + dmll - self.w * v
        if self.lik == "gamma":   # shape on the log scale
            a, loc = self.aux, self.mode + self.F
            neg = a * (float(np.sum(loc + self.y * np.exp(-loc))) - n * (np.log(a) + 1. - _digamma(a))
                       - float(np.log(self.y).sum()))
            g.append(neg + 0.5 * float(self.w @ np.diag(S)) + float(self.d1 @ v))
        if self.lik == "gaussian":   # error variance on the log scale: dW = -W
            r = self.y - self.mode - self.F
            g.append(-0.5 * float(r @ r) / self.aux + 0.5 * n + 0.5 * float(-np.diag(S).sum() / self.aux))
        return np.array(g), gf
