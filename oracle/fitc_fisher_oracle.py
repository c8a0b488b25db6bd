"""ORACLE TEST INFRASTRUCTURE — NOT PART OF THE PRODUCT.

CPU restatement (numpy, dense algebra) of the reference's standard deviations of the covariance parameters
for the Gaussian FITC model, the checker of gpboost_amd's FitcSolver::Fisher (csrc/fitc.h). Importable only
from tests/. Follows the reference:
  CalcStdDevCovPar              re_model_template.h:9775-9789 (std = sqrt(diag(FI^-1)))
  CalcFisherInformation_FITC_FSA re_model_template.h:9363-9548, gp_approx = "fitc", cholesky, original scale:
                                Psi on the transformed scale (nugget 1, fitc_resid_diag d with the jittered
                                variance, :7358-7377), the derivative G_k of the ORIGINAL covariance
                                (GetZSigmaZtGrad(k, false, sigma^2): dSigma / dsigma1^2 = the correlations,
                                dSigma / drho = sigma^2 dK / drho; diagonal part 1 resp. 0 minus
                                2 A_i . dK_i - A_i . (dK_mm A)_i, A = K_mm,s^-1 K_mn),
                                x0 = Psi^-1 z, S_k = Psi^-1 G_k z, R_k = G_k Psi^-1 z,
                                FI = 1/2 mean_c [x0.x0, x0.S_k; R_k.S_l (k <= l)] / sigma^4
The probes z are GenRandVecNormalParallel's (oracle.gen_probes). Pinned to the reference by
tests/test_oracle_stddev_fitc.py.
"""
from __future__ import annotations

import numpy as np

from oracle import oracle as O
from oracle.fitc_laplace_oracle import JITTER, cov_dcov, _dist


def fitc_fisher(X, Z, cov_type, orig, t=50, seed=1, run_id=0):
    """(FI 3 x 3, std devs) at the original-scale parameters orig = (sigma^2, sigma1^2, rho)."""
    X = np.asarray(X, float)
    n = X.shape[0]
    s2, v1, rho = (float(p) for p in orig)
    tr = O.transform(cov_type, orig)
    var, phi = tr[1], tr[2]
    g = (-2. if cov_type == 3 else -1.) / rho
    K, dKr = cov_dcov(_dist(X, Z), var, phi, cov_type)            # n x m
    Kmm, dKmmr = cov_dcov(_dist(Z, Z), var, phi, cov_type)
    np.fill_diagonal(Kmm, var)
    np.fill_diagonal(dKmmr, 0.)
    Ks = Kmm.copy()
    Ks[np.diag_indices_from(Ks)] *= JITTER
    A = np.linalg.solve(Ks, K.T)                                   # m x n
    Lk = np.linalg.cholesky(Ks)
    V = np.linalg.solve(Lk, K.T)
    d = 1. + var * JITTER - (V * V).sum(0)
    M = Ks + (K.T / d) @ K
    Minv = np.linalg.inv(M)

    def psi_inv(R):
        R1 = R / d[:, None]
        return R1 - (K @ (Minv @ (K.T @ R1))) / d[:, None]

    # original-scale derivatives (dK n x m, dK_mm, diagonal base)
    derivs = [(K / var, Kmm / var, 1.), (s2 * g * dKr, s2 * g * dKmmr, 0.)]
    Gs = []
    for dK, dKmm, base in derivs:
        dd = base - (2. * np.sum(A.T * dK, axis=1) - np.sum(A * (dKmm @ A), axis=0))

        def G(R, dK=dK, dKmm=dKmm, dd=dd):
            AR = A @ R
            return dd[:, None] * R + A.T @ (dK.T @ R) + dK @ AR - A.T @ (dKmm @ AR)
        Gs.append(G)
    z = O.gen_probes(n, t, seed, run_id)
    x0 = psi_inv(z)
    S = [psi_inv(G(z)) for G in Gs]
    R = [G(x0) for G in Gs]
    FI = np.zeros((3, 3))
    FI[0, 0] = 0.5 * np.mean(np.sum(x0 * x0, axis=0))
    for k in range(2):
        FI[0, k + 1] = 0.5 * np.mean(np.sum(x0 * S[k], axis=0))
        for l in range(k, 2):
            FI[k + 1, l + 1] = 0.5 * np.mean(np.sum(R[k] * S[l], axis=0))
    FI /= s2 * s2
    FI = np.triu(FI) + np.triu(FI, 1).T
    return FI, np.sqrt(np.diag(np.linalg.inv(FI)))
