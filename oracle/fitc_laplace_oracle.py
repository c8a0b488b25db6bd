"""ORACLE TEST INFRASTRUCTURE — NOT PART OF THE PRODUCT.

CPU restatement (numpy) of the reference's FITC approximation with a Laplace likelihood
(gp_approx = "fitc", likelihood = "bernoulli_logit" | "bernoulli_probit" | "poisson",
matrix_inversion_method = "cholesky"), the checker
of gpboost_amd's FitcLaplace (csrc/fitc_laplace.hip). Importable only from tests/. Follows, step for
step and with the reference's own factorizations (Cholesky solves, not explicit inverses):
  CalcSigmaComps                          re_model_template.h:7341-7378 (fitc_resid_diag, no nugget)
  FindModePostRandEffCalcMLLFITC          likelihoods.h:3090-3235
  CheckConvergenceModeFinding             likelihoods.h:11820-11870
  CalcGradNegMargLikelihoodLaplaceApproxFITC  likelihoods.h:5397-5593 (cov_grad, fixed_effect_grad)
  CalcPredFITC_FSA + PredictLaplaceApproxFITC re_model_template.h:10600-10760, likelihoods.h:7157-7232
  bernoulli_logit log-likelihood / derivatives likelihoods.h:8724, 9226, 9896, 10187 (DF_utils.h:37-60)
  bernoulli_probit :8708, 9208, 9871, 10171 (here through scipy's log_ndtr);  poisson :8730, 9230, 9904,
  10200 with the normalizing constant -sum log y! (CalculateAuxQuantLogNormalizingConstant)
  covariance functions and log-range derivatives cov_fcts.h:1681-1786, 2116-2143 (transformed scale)
The inducing points are an input (the reference's own, from the fixtures; their selection is pinned by
test_oracle_fitc.py / test_gpu_fitc.py).
"""
from __future__ import annotations

import numpy as np
from scipy.linalg import cho_factor, cho_solve, solve_triangular
from scipy.special import gammaln, log_ndtr

JITTER = 1.0 + 1e-6   # JITTER_MULT_IP_FITC_FSA (utils.h:39)


def cov_dcov(r, var, phi, cov_type):
    """C(r) and dC/dlog(phi) (cov.h's cov_dcov; cov_type 0 Matern 0.5, 1: 1.5, 2: 2.5, 3 Gaussian)."""
    if cov_type == 0:
        e = np.exp(-phi * r)
        c = var * e
        return c, -phi * r * c
    if cov_type == 1:
        x = phi * r
        e = np.exp(-x)
        return var * (1. + x) * e, -var * x * x * e
    if cov_type == 2:
        x = phi * r
        e = np.exp(-x)
        return var * (1. + x + x * x / 3.) * e, -var * x * x / 3. * (1. + x) * e
    e = np.exp(-phi * r * r)
    c = var * e
    return c, -phi * r * r * c


def _dist(A, B):
    return np.sqrt(np.maximum(((A[:, None, :] - B[None, :, :]) ** 2).sum(-1), 0.))


def _sigmoid(x):
    out = np.empty_like(x)
    pos = x >= 0
    out[pos] = 1. / (1. + np.exp(-x[pos]))
    e = np.exp(x[~pos])
    out[~pos] = e / (1. + e)
    return out


def _lik(lik, y, l):
    """(sum of log-likelihoods, first derivative, information, d information / d l) per sample."""
    if lik == "bernoulli_logit":
        p = _sigmoid(l)
        ll = float(np.sum(y * l - (np.log1p(np.exp(-np.abs(l))) + np.maximum(l, 0.))))
        return ll, y - p, p * (1. - p), -p * (1. - p) * (2. * p - 1.)
    if lik == "poisson":
        e = np.exp(l)
        return float(np.sum(y * l - e)), y - e, e, e
    if lik != "bernoulli_probit":
        raise ValueError(lik)
    s = 2. * y - 1.                       # log Phi(s l); d/dl = s r, r = phi(s l) / Phi(s l)
    x = s * l
    lc = log_ndtr(x)
    r = np.exp(-0.5 * x * x - 0.5 * np.log(2. * np.pi) - lc)
    d1 = s * r
    w = r * (x + r)                       # -d2/dl2 log Phi(s l)
    dinfo = -s * r * (x * x - 1. + r * (3. * x + 2. * r))
    return float(lc.sum()), d1, w, dinfo


class FitcLaplaceOracle:
    def __init__(self, X, y, Z, cov_type, var, phi, fixed_effects=None, likelihood="bernoulli_logit"):
        self.X, self.y, self.Z = np.asarray(X, float), np.asarray(y, float), np.asarray(Z, float)
        self.lik = likelihood
        self.const = -float(gammaln(self.y + 1.).sum()) if likelihood == "poisson" else 0.
        self.ct, self.var, self.phi = cov_type, var, phi
        self.F = np.zeros(len(y)) if fixed_effects is None else np.asarray(fixed_effects, float)
        K, dK = cov_dcov(_dist(self.X, self.Z), var, phi, cov_type)          # n x m (cross_cov)
        r = _dist(self.Z, self.Z)
        Kmm, dKmm = cov_dcov(r, var, phi, cov_type)
        np.fill_diagonal(Kmm, var)
        np.fill_diagonal(dKmm, 0.)
        self.K, self.dK, self.Kmm, self.dKmm = K, dK, Kmm, dKmm
        Ks = Kmm.copy()
        Ks[np.diag_indices_from(Ks)] *= JITTER                                # sigma_ip_stable
        self.Ks = Ks
        self.cKs = cho_factor(Ks, lower=True)
        V = solve_triangular(self.cKs[0], K.T, lower=True)                    # L^-1 K^T
        self.d = var * JITTER - (V * V).sum(0)                                 # fitc_resid_diag (no nugget)
        self.logdet_Ks_half = float(np.log(np.diag(self.cKs[0])).sum())

    def _ll(self, mode):
        return _lik(self.lik, self.y, mode + self.F)[0] + self.const

    def sigma(self, x):   # K (K_mm,s^-1 (K^T x)) + d o x (likelihoods.h:3153-3154)
        return self.K @ cho_solve(self.cKs, self.K.T @ x) + self.d * x

    def find_mode(self, delta=1e-8, mode=None, a=None, maxit=1000):
        n = len(self.y)
        K, d, y = self.K, self.d, self.y
        mode = np.zeros(n) if mode is None else mode.copy()
        a = np.zeros(n) if a is None else a.copy()
        obj = -0.5 * a.dot(mode) + self._ll(mode)
        for it in range(maxit):
            _, g, w, _ = _lik(self.lik, y, mode + self.F)
            ws = np.sqrt(w)
            DW = 1. / (w * d + 1.)
            wdw = ws * ws * DW
            M = self.Ks + K.T @ (wdw[:, None] * K)
            cM = cho_factor(M, lower=True)
            rhs = w * mode + g
            srhs = self.sigma(rhs)
            vaux2 = cho_solve(cM, K.T @ (wdw * srhs))
            upd = DW * (ws * srhs - ws * (K @ vaux2))
            a_upd = rhs - upd * ws
            m_upd = self.sigma(a_upd)
            direc = m_upd - mode
            gdd = direc.dot(a_upd - a + w * direc)
            lr = 1.
            for ih in range(20):
                if ih == 0:
                    a_new, m_new = a_upd, m_upd
                else:
                    a_new = (1 - lr) * a + lr * a_upd
                    m_new = (1 - lr) * mode + lr * m_upd
                obj_new = -0.5 * a_new.dot(m_new) + self._ll(m_new)
                if obj_new < obj + 1e-4 * lr * gdd or not np.isfinite(obj_new):
                    lr *= 0.5
                else:
                    break
            mode, a = m_new, a_new
            if not np.isfinite(obj_new):
                raise FloatingPointError("NaN in the mode finding")
            conv = abs(obj_new - obj) < delta * abs(obj) if it == 0 else (obj_new - obj) < delta * abs(obj)
            obj = obj_new
            if conv:
                break
        self.mode, self.a, self.obj, self.newton_its = mode, a, obj, it + 1
        # after the mode finding (:3200-3232)
        _, self.g, self.w, self.dinfo = _lik(self.lik, y, mode + self.F)
        self.dpwi = 1. / (d + 1. / self.w)
        self.cM = cho_factor(self.Ks + K.T @ (self.dpwi[:, None] * K), lower=True)
        mll = obj - np.log(np.diag(self.cM[0])).sum() + self.logdet_Ks_half + 0.5 * np.log(self.dpwi).sum() \
            - 0.5 * np.log(self.w).sum()
        self.nll = -float(mll)
        return self.nll

    def gradient(self, want_f=False):
        """[d/dlog sigma1^2, d/dlog phi] of the negative approximate marginal log-likelihood (and the
        gradient wrt F) at the mode (likelihoods.h:5397-5593)."""
        K, d, w, g, a = self.K, self.d, self.w, self.g, self.a
        dinfo = self.dinfo
        WI = 1. / w
        DW = 1. / (w * d + 1.)
        Linv_KT_DW = solve_triangular(self.cM[0], K.T * DW[None, :], lower=True)
        sw = (Linv_KT_DW * Linv_KT_DW).sum(0) + WI - DW * WI
        dmll = 0.5 * sw * dinfo
        A = cho_solve(self.cKs, K.T)                                         # sigma_ip_inv_cross_cov_T
        b = cho_solve(self.cKs, K.T @ a)
        Dp = 1. / (d + WI)
        grads = []
        for dK, dKmm, dvar in ((K, self.Kmm, self.var), (self.dK, self.dKmm, 0.)):
            fdg = dvar - 2. * (A * dK.T).sum(0) + (A * (dKmm @ A)).sum(0)
            Wg = dKmm + K.T @ (Dp[:, None] * dK)
            Wg = Wg + (K.T @ (Dp[:, None] * dK)).T - K.T @ ((Dp * Dp * fdg)[:, None] * K)
            tr_M = np.trace(cho_solve(self.cM, Wg))
            tr_Ks = np.trace(cho_solve(self.cKs, dKmm))
            expl = -(dK.T @ a).dot(b) + 0.5 * b.dot(dKmm @ b) - 0.5 * a.dot(fdg * a)
            expl += 0.5 * tr_M - 0.5 * tr_Ks + 0.5 * fdg.dot(Dp)
            sd = dK @ (A @ g) + A.T @ (dK.T @ g) - A.T @ ((dKmm @ A) @ g) + fdg * g
            vaux = cho_solve(self.cM, K.T @ (Dp * sd))
            dmode = WI * (Dp * sd - Dp * (K @ vaux))
            grads.append(expl + dmll.dot(dmode))
        out = {"grad": np.array(grads)}
        if want_f:
            s = WI * dmll - (1. / DW) * (WI * dmll) + Linv_KT_DW.T @ (Linv_KT_DW @ dmll)
            out["grad_f"] = -g + dmll - s * w
        return out

    def predict(self, Xp, match=None, want_var=True, want_cov=False):
        """Latent predictive mean / variance / covariance (CalcPredFITC_FSA + PredictLaplaceApproxFITC)."""
        Xp = np.asarray(Xp, float)
        Kp, _ = cov_dcov(_dist(Xp, self.Z), self.var, self.phi, self.ct)          # np x m
        mean = Kp @ cho_solve(self.cKs, self.K.T @ self.g)
        npred = Xp.shape[0]
        corr = np.zeros((npred, len(self.y)))
        if match is not None:
            A = cho_solve(self.cKs, self.K.T)
            for p_, o in enumerate(match):
                if o >= 0:
                    corr[p_, o] = self.var - Kp[p_].dot(A[:, o])
        mean = mean + corr @ self.g
        Vp = solve_triangular(self.cKs[0], Kp.T, lower=True)
        resid = self.var - (Vp * Vp).sum(0)
        wps = Kp.T - self.K.T @ (self.dpwi[:, None] * corr.T)
        U = solve_triangular(self.cM[0], wps, lower=True)
        out = {"mean": mean}
        if want_var:
            out["var"] = resid + (U * U).sum(0) - (corr * (self.dpwi[None, :] * corr)).sum(1)
        if want_cov:
            out["cov"] = U.T @ U + np.diag(resid) - corr @ (self.dpwi[:, None] * corr.T)
        return out
