"""ORACLE TEST INFRASTRUCTURE — NOT PART OF THE PRODUCT.

CPU restatement (numpy, dense algebra) of the reference's negative log-likelihood and gradient for combined
Gaussian process + grouped random effects models (gp_approx = "none", Gaussian likelihood), the checker of
gpboost_amd's GroupedModel with an attached GP (csrc/grouped_model.h). Importable only from tests/.
Transformed scale (re_comp.h TransformCovPars): pars = (sigma^2, tau_1 .. tau_K, v, phi),
  Psi = sum_k tau_k Z_k Z_k^T + v corr(phi) + I      (CalcZSigmaZt re_model_template.h:8430-8441)
  nll = y^T Psi^-1 y / (2 sigma^2) + log|Psi| / 2 + n / 2 (log sigma^2 + log 2 pi)      (:2880)
  d nll / dlog theta_k = -y_aux^T dPsi_k y_aux / (2 sigma^2) + tr(Psi^-1 dPsi_k) / 2   (:1798-1818)
  nugget (mode 0): -y^T Psi^-1 y / (2 sigma^2) + n / 2
Pinned to the reference by tests/test_oracle_combined.py.
"""
from __future__ import annotations

import numpy as np

from oracle.fitc_laplace_oracle import cov_dcov, _dist


def combined_nll_grad(X, groups, y, cov_type, pars, mode=0):
    X = np.asarray(X, float)
    g = np.asarray(groups)
    if g.ndim == 1:
        g = g.reshape(-1, 1)
    n, K = g.shape
    s2 = float(pars[0])
    tau = [float(t) for t in pars[1:1 + K]]
    v, phi = float(pars[1 + K]), float(pars[2 + K])
    C, dC = cov_dcov(_dist(X, X), v, phi, cov_type)
    np.fill_diagonal(C, v)
    np.fill_diagonal(dC, 0.)
    same = [(g[:, k][:, None] == g[:, k][None, :]).astype(float) for k in range(K)]
    Psi = C + np.eye(n)
    for k in range(K):
        Psi += tau[k] * same[k]
    L = np.linalg.cholesky(Psi)
    Pinv = np.linalg.inv(Psi)
    ya = Pinv @ y
    q = float(y @ ya)
    logdet = 2. * np.sum(np.log(np.diag(L)))
    if mode == 1:
        s2 = q / n
    nll = q / 2. / s2 + logdet / 2. + n / 2. * (np.log(s2) + np.log(2. * np.pi))
    derivs = [tau[k] * same[k] for k in range(K)] + [C, dC]
    grad = [] if mode == 1 else [-q / s2 / 2. + n / 2.]
    for D in derivs:
        grad.append(-float(ya @ D @ ya) / s2 / 2. + float(np.sum(Pinv * D)) / 2.)
    return dict(nll=float(nll), grad=np.array(grad), sigma2=s2)
