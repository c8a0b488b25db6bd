"""ORACLE TEST INFRASTRUCTURE — NOT PART OF THE PRODUCT.

Dense numpy restatement of the reference's vecchia_pred_type = "order_pred_first" for the Gaussian
likelihood (CalcPredVecchiaPredictedFirstOrder, Vecchia_utils.cpp:2018-2239): the prediction points first
(given order), then the observed points in the model's Vecchia order; every point conditions on its
nearest earlier points (find_nearest_neighbors_Vecchia_fast over [pred; obs], num_neighbors_pred; the
oracle's kNN is bit-exact with it); rows A_i = (C_NN + I)^-1 c_Ni, D_i = 1 + var - A_i c_Ni (nugget 1 on
the transformed scale, prediction rows included); the conditional precision
Q = Bp^T Dp^-1 Bp + Bop^T Do^-1 Bop; mean = -Q^-1 Bop^T Do^-1 Bo y; covariance Q^-1 (transformed scale:
times sigma^2; latent predictions minus the nugget on the diagonal, re_model_template.h:3898-3913).

The reference reads variances / covariances off the inverse of its AMD-permuted sparse Cholesky factor
(Vecchia_utils.cpp:2220-2237), so they come out in its permuted order; this restatement returns them in
prediction-point order. tests/test_oracle_pred_first.py pins it to the reference: means elementwise, and
the reference's covariance equals this covariance under ONE permutation (recovered from the variances),
i.e. the reference's output is exactly the permuted natural-order result.
"""
from __future__ import annotations

import numpy as np
from scipy.linalg import cho_factor, cho_solve

from oracle import oracle as O
from oracle.fitc_laplace_oracle import _dist, cov_dcov


def pred_first(X, y, xp, cov_type, pars_trafo, m, mp=None, response=False):
    """(mean, covariance) of the prediction points in their own order (original scale)."""
    s2, var, phi = pars_trafo
    mp = mp or 2 * m
    perm, xv, _ = O.vecchia_setup(X, m, 0, True)
    yv = y[perm]
    npred = xp.shape[0]
    A = np.vstack([xp, xv])
    N = A.shape[0]
    nb = O.find_neighbors(A, min(mp, N - 1))
    B = np.eye(N)
    Dinv = np.zeros(N)
    for i in range(N):
        k = min(i, nb.shape[1])
        Ni = nb[i, :k]
        d = 1. + var
        if k > 0:
            C, _ = cov_dcov(_dist(A[Ni], A[Ni]), var, phi, cov_type)
            np.fill_diagonal(C, var)
            C += np.eye(k)
            c, _ = cov_dcov(_dist(A[Ni], A[i:i + 1])[:, 0], var, phi, cov_type)
            a = cho_solve(cho_factor(C, lower=True), c)
            B[i, Ni] -= a
            d -= a @ c
        Dinv[i] = 1. / d
    Bp, Bop, Bo = B[:npred, :npred], B[npred:, :npred], B[npred:, npred:]
    Q = Bp.T @ np.diag(Dinv[:npred]) @ Bp + Bop.T @ np.diag(Dinv[npred:]) @ Bop
    cQ = cho_factor(Q, lower=True)
    mean = -cho_solve(cQ, Bop.T @ (Dinv[npred:] * (Bo @ yv)))
    cov = cho_solve(cQ, np.eye(npred))
    if not response:
        cov = cov - np.eye(npred)
    return mean, s2 * cov
