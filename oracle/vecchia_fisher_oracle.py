"""ORACLE TEST INFRASTRUCTURE — NOT PART OF THE PRODUCT.

CPU restatement (numpy / scipy.sparse) of the reference's standard deviations of the covariance parameters
for the Gaussian Vecchia model, the checker of gpboost_amd's VecchiaFisher (csrc/vecchia_fisher.h).
Importable only from tests/. Follows the reference:
  CalcStdDevCovPar              re_model_template.h:9775-9789 (factor and derivatives on the ORIGINAL scale,
                                CalcCovFactor(false, sigma^2) + CalcGradientVecchia(false, sigma^2, true);
                                std = sqrt(diag(FI^-1)))
  row factor + derivatives      Vecchia_utils.cpp:1498-1600 (transf_scale = false: covariances times sigma^2,
                                dSigma / dsigma1^2 = correlation, dSigma / drho = sigma1^2 dcorr / drho, D_grad
                                of the variance 1 on the diagonal)
  Fisher information            re_model_template.h:9246-9298 (use_stochastic_trace_for_Fisher_information_Vecchia_,
                                the default): probes z (GenRandVecNormalParallel(seed_rand_vec_trace,
                                cg_generator_counter_), CG_utils.cpp:930-947; oracle.gen_probes),
                                g_0 = B^T D^-1 B z, g_k = B^T D^-1 (-dB_k Sigma z + dD_k B^-T z) - dB_k^T B^-T z,
                                FI_kl = 1/2 mean over the t columns of (g_k . g_l)
The row factor is restated directly on the original scale here (the GPU derives it from the transformed
scale); pinned to the reference by tests/test_oracle_stddev_vecchia.py.
"""
from __future__ import annotations

import numpy as np
import scipy.sparse as sp
from scipy.linalg import cho_factor, cho_solve
from scipy.sparse.linalg import spsolve_triangular

from oracle import oracle as O
from oracle.fitc_laplace_oracle import cov_dcov, _dist


def _dlogphi_drho(cov_type, rho):
    return (-2. if cov_type == 3 else -1.) / rho


def vecchia_factor_orig(xv, nb, cov_type, orig):
    """B (sparse unit lower), D, and per original-scale parameter (sigma1^2, rho) dB (sparse), dD."""
    xv = np.asarray(xv, float)
    n = xv.shape[0]
    s2, v1, rho = (float(p) for p in orig)
    phi = O.transform(cov_type, orig)[2]
    g = _dlogphi_drho(cov_type, rho)
    rows, cols, bv, dbv0, dbv1 = [], [], [], [], []
    D = np.zeros(n)
    dD = [np.zeros(n), np.zeros(n)]
    for i in range(n):
        k = min(i, nb.shape[1])
        D[i] = v1 + s2
        dD[0][i] = 1.
        if k == 0:
            continue
        N = nb[i, :k]
        xs = xv[N]
        cnn, dcnn = cov_dcov(_dist(xs, xs), v1, phi, cov_type)   # sigma1^2 corr, d / dlog phi
        np.fill_diagonal(cnn, v1)
        np.fill_diagonal(dcnn, 0.)
        cni, dcni = cov_dcov(_dist(xs, xv[i:i + 1])[:, 0], v1, phi, cov_type)
        C = cnn + s2 * np.eye(k)
        cC = cho_factor(C, lower=True)
        a = cho_solve(cC, cni)
        D[i] -= a @ cni
        # d / dsigma1^2: the correlations; d / drho: sigma1^2 dcorr / dlog phi * dlog phi / drho
        for p, (dC, dc) in enumerate(((cnn / v1, cni / v1), (dcnn * g, dcni * g))):
            da = cho_solve(cC, dc - dC @ a)
            (dbv0 if p == 0 else dbv1).extend(-da)
            dD[p][i] -= da @ cni + a @ dc
        rows.extend([i] * k)
        cols.extend(N)
        bv.extend(-a)
    eye = sp.identity(n, format="csr")
    B = (sp.csr_matrix((bv, (rows, cols)), shape=(n, n)) + eye).tocsr()
    dB = [sp.csr_matrix((v, (rows, cols)), shape=(n, n)) for v in (dbv0, dbv1)]
    return B, D, dB, dD


def vecchia_fisher(xv, nb, cov_type, orig, t=50, seed=1, run_id=0):
    """(FI 3 x 3, std devs) of the stochastic-trace Fisher information at the original-scale parameters."""
    n = xv.shape[0]
    B, D, dB, dD = vecchia_factor_orig(xv, nb, cov_type, orig)
    z = O.gen_probes(n, t, seed, run_id)                        # n x t
    BT = B.T.tocsr()
    W = spsolve_triangular(BT, z, lower=False)                 # B^-T z
    Sz = spsolve_triangular(B, D[:, None] * W, lower=True)     # B^-1 D B^-T z
    Dinv = 1. / D
    g = [BT @ (Dinv[:, None] * (B @ z))]
    for k in range(2):
        u = -(dB[k] @ Sz) + dD[k][:, None] * W
        g.append(BT @ (Dinv[:, None] * u) - dB[k].T @ W)
    FI = np.zeros((3, 3))
    for k in range(3):
        for l in range(k, 3):
            FI[k, l] = FI[l, k] = 0.5 * np.mean(np.sum(g[k] * g[l], axis=0))
    return FI, np.sqrt(np.diag(np.linalg.inv(FI)))
