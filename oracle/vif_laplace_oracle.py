"""ORACLE TEST INFRASTRUCTURE — NOT PART OF THE PRODUCT.

CPU restatement (numpy, dense algebra) of the reference's full-scale Vecchia approximation ("VIF") with a
non-Gaussian likelihood and matrix_inversion_method = "cholesky" (the FSVA Laplace approximation), the checker
of gpboost_amd's VIF Laplace path (csrc/vif_laplace.cpp). Importable only from tests/. Follows
  residual factor (latent form)   Vecchia_utils.cpp:1355-1356, 1405-1617 (no nugget; the neighbours' residual
                                  matrix times JITTER_MULT_VECCHIA on its diagonal; oracle.vif_oracle.vif_factor)
  Sigma^-1 (Woodbury)             R - R K M^-1 K^T R, R = B^T D^-1 B, M = K_mm,s + K^T R K (re_model_template.h
                                  :8832-8863 CalcCovFactorFITC_FSA; likelihoods.h:2365-2372)
  mode finding                    FindModePostRandEffCalcMLLFSVA, Cholesky branch (likelihoods.h:2316-2742:
                                  Newton from 0, update (Sigma^-1 + W)^-1 (W mode + d1) (:2585-2601), Armijo with
                                  direction^T (Sigma^-1 + W) direction (:2603-2635), the objective -1/2 m^T Sigma^-1 m
                                  + log p(y | m + F); log det (:2724-2736): -sum log L_A + 1/2 sum log D^-1 + sum log
                                  L_{K_mm,s} - sum log L_{M2}, M2 = M - (R K)^T A^-1 (R K), A = R + W)
  gradient                        CalcGradNegMargLikelihoodLaplaceApproxFSVA, Cholesky branch (:4716-4925), restated
                                  literally: SigmaI_deriv = -R (variance) | dB^T D^-1 B + B^T D^-1 dB - B^T D^-1 dD
                                  D^-1 B (range); sigma_woodbury_grad = dK_mm (un-jittered) + K^T S' K + (RK)^T dK +
                                  dK^T (RK); explicit 1/2 (m^T dSigma^-1 m + tr(S' A^-1)) + 1/2 sum D^-1 dD - 1/2
                                  tr(K_mm,s^-1 dK_mm) + 1/2 tr(M2^-1 dM2); implicit - ((Sigma^-1 + W)^-1 d_mll)^T
                                  dSigma^-1 m with d_mll = 1/2 diag((Sigma^-1 + W)^-1) dW; the gradient wrt F and the
                                  gamma shape (:4843-4923)
Pinned to the reference by tests/test_oracle_vif_laplace.py (fixtures of oracle/_ref/ref_harness).
"""
from __future__ import annotations

import numpy as np
from scipy.linalg import cho_factor, cho_solve

from oracle.latent_chol_oracle import LatentCholOracle, _lik_all
from oracle.dense_laplace_oracle import _digamma
from oracle.vif_oracle import vif_factor


def _logdet(A):
    s, v = np.linalg.slogdet(A)
    return float(v) if s > 0 else float("nan")


class VifLaplaceOracle(LatentCholOracle):
    """Laplace-approximated nll / gradient of a VIF model at (sigma1^2, phi) on the transformed scale."""

    def __init__(self, xv, y_vo, nb, Z, cov_type, var, phi, likelihood, aux=1., fixed_effects=None, delta=1e-8):
        from scipy.special import gammaln
        self.y = np.asarray(y_vo, float)
        n = len(self.y)
        f = vif_factor(xv, nb, Z, cov_type, var, phi, nugget=0.)
        self.f = f
        self.B, self.D = f["B"], f["D"]
        self.Dinv = 1. / self.D
        self.lik, self.aux = likelihood, aux
        self.F = np.zeros(n) if fixed_effects is None else np.asarray(fixed_effects, float)
        self.const = -float(gammaln(self.y + 1.).sum()) if likelihood == "poisson" else 0.
        if likelihood == "gamma" and abs(aux - 1.) >= 1e-10 * max(1., aux):
            self.const = (aux - 1.) * float(np.log(self.y).sum()) + n * (aux * np.log(aux) - gammaln(aux))
        B, Dinv, K = self.B, self.Dinv, f["K"]
        self.R = B.T @ (Dinv[:, None] * B)
        self.RK = self.R @ K
        self.M = f["Ks"] + K.T @ self.RK
        SI = self.R - self.RK @ np.linalg.solve(self.M, self.RK.T)
        self.SigmaI = 0.5 * (SI + SI.T)
        self._mode(delta)
        A = self.R + np.diag(self.w)
        self.Ai = np.linalg.inv(A)
        self.AiC = self.Ai @ self.RK
        self.M2 = self.M - self.RK.T @ self.AiC
        ld = (_logdet(A) - float(np.log(Dinv).sum()) - _logdet(f["Ks"]) + _logdet(self.M2))
        self.logdet = ld
        self.nll = -(self.obj - 0.5 * ld)

    def _obj(self, mode):
        return (_lik_all(self.lik, self.y, mode + self.F, self.aux)[0] + self.const
                - 0.5 * float(mode @ (self.SigmaI @ mode)))

    def grad(self, grad_offset=None):
        """grad_offset: the offsets at which the location-dependent gradient terms are evaluated (the reference's
        CalcGradPars passes FSVA the fixed effects in data order, re_model_template.h:1859; None: the model-order
        offsets of the mode finding)."""
        n = len(self.y)
        f, K, R, RK, M, M2, Ai, AiC = self.f, self.f["K"], self.R, self.RK, self.M, self.M2, self.Ai, self.AiC
        S = np.linalg.inv(self.SigmaI + np.diag(self.w))
        S = 0.5 * (S + S.T)
        d1g, wg, dwg = self.d1, self.w, self.dw
        locg = self.mode + self.F
        if grad_offset is not None:
            locg = self.mode + np.asarray(grad_offset, float)
            _, d1g, wg, dwg = _lik_all(self.lik, self.y, locg, self.aux)
        dmll = 0.5 * np.diag(S) * dwg
        v = S @ dmll
        DB = self.Dinv[:, None] * self.B
        Ks = cho_factor(f["Ks"], lower=True)
        m = self.mode
        MiKR = np.linalg.solve(M, RK.T)
        g = []
        for k in range(2):
            if k == 0:
                Sp = -R
                dK = K
            else:
                dB, dD = f["dB"][1], f["dD"][1]
                Sp = dB.T @ DB + DB.T @ dB - DB.T @ (dD[:, None] * DB)
                dK = f["dK"][1]
            dKmm = f["dKmm"][k]
            SpK = Sp @ K
            dM = dKmm + K.T @ SpK + RK.T @ dK + dK.T @ RK
            X = SpK + R @ dK
            dSI = Sp - X @ MiKR - RK @ np.linalg.solve(M, X.T) + RK @ np.linalg.solve(M, dM @ MiKR)
            expl = 0.5 * (float(m @ (dSI @ m)) + float(np.sum(Sp * Ai)))
            expl += 0.5 * float(np.sum(self.Dinv * f["dD"][k]))
            expl -= 0.5 * float(np.trace(cho_solve(Ks, dKmm)))
            T1 = RK.T @ Ai @ (R @ dK)
            T2 = RK.T @ Ai @ SpK
            dM2 = dM - (T1 + T1.T) - (T2 + T2.T) + AiC.T @ Sp @ AiC
            expl += 0.5 * float(np.trace(np.linalg.solve(M2, dM2)))
            gk = expl
            if self.lik != "gaussian":
                gk -= float(v @ (dSI @ m))
            g.append(gk)
        gf = -self.d1 + dmll - self.w * v
        if self.lik == "gamma":   # shape on the log scale
            a, loc = self.aux, locg
            neg = a * (float(np.sum(loc + self.y * np.exp(-loc))) - n * (np.log(a) + 1. - _digamma(a))
                       - float(np.log(self.y).sum()))
            # with the covariance gradient the reference adds diag(A^-1) to SigmaI_plus_W_inv_diag a second time
            # before this sum (likelihoods.h:4866-4868 after :4771), so diag(A^-1) enters twice
            dg = np.diag(S) + np.diag(Ai)
            g.append(neg + 0.5 * float(wg @ dg) + float(d1g @ v))
        return np.array(g), gf
