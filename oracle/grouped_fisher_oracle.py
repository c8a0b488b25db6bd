"""ORACLE TEST INFRASTRUCTURE — NOT PART OF THE PRODUCT.

CPU restatement (numpy, dense n x n algebra) of the reference's standard deviations of the covariance
parameters of grouped random effects models (CalcStdDevCovPar re_model_template.h:9775-9789 ->
CalcFisherInformation_Only_Grouped_REs_Woodbury :9559-9651, cholesky, original scale): with
Sigma = sigma^2 Psi, Psi = I + sum_k tau_k Z_k Z_k^T, dSigma / dsigma^2 = I, dSigma / dsigma_k^2 = Z_k Z_k^T,
  FI_ab = 1/2 tr(Sigma^-1 dSigma_a Sigma^-1 dSigma_b),  std = sqrt(diag(FI^-1)).
Formed directly from Psi^-1 (independent of the reference's Woodbury formulas and of the build's
B = S^1/2 A^-1 S^1/2 closed forms, csrc/grouped.h). Pinned to the reference by
tests/test_oracle_grouped_fisher.py. Small n only (n x n dense).
"""
from __future__ import annotations

import numpy as np


def grouped_fisher(groups, cov_pars):
    """groups: n x K integer labels; cov_pars original scale [sigma^2, sigma_1^2, ...]."""
    g = np.asarray(groups)
    n, K = g.shape
    s2 = float(cov_pars[0])
    Zs = []
    for k in range(K):
        _, inv = np.unique(g[:, k], return_inverse=True)
        Z = np.zeros((n, inv.max() + 1))
        Z[np.arange(n), inv] = 1.
        Zs.append(Z)
    Sigma = s2 * np.eye(n)
    for k in range(K):
        Sigma += float(cov_pars[k + 1]) * Zs[k] @ Zs[k].T
    Si = np.linalg.inv(Sigma)
    dS = [np.eye(n)] + [Z @ Z.T for Z in Zs]
    G = [Si @ d for d in dS]
    P = K + 1
    FI = np.array([[0.5 * np.sum(G[a] * G[b].T) for b in range(P)] for a in range(P)])
    return FI, np.sqrt(np.diag(np.linalg.inv(FI)))
