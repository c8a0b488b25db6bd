"""ORACLE TEST INFRASTRUCTURE — NOT PART OF THE PRODUCT.

CPU restatement of GPB_OptimCovPar for the Gaussian likelihood (profiled nugget) on top of the
oracle's exact nll / gradient (oracle.py -> gp_oracle.cpp):

  initial values  re_model_template.h:4388-4504 (FindInitCovPar), cov_fcts.h:1275-1450
                  (median distance of <= 1000 points; gp_oracle.cpp orc_init_range_trafo)
  objective       optim_utils.h:243-364 (EvalLLforLBFGSpp, profile_out_error_variance)
  L-BFGS          external_libs/LBFGSpp/include/LBFGS.h:86-301 (past = 1, epsilon = 1e-20),
                  LineSearchBacktracking.h:45-143 (Armijo, GPBoost's 1/32 shrink), BFGSMat.h:89-186
                  (two-loop recursion), step cap optim_utils.h:497-534 / re_model_template.h:4937-4945

Pinned by tests/test_oracle_fit.py against golden_fit.json (the reference run here).
"""
from __future__ import annotations

import math

import numpy as np

from oracle import oracle as O


def init_trafo(coords: np.ndarray, y: np.ndarray, cov_type: int, seed: int = 0, shuffled: bool = False) -> np.ndarray:
    """coords in the component's order (Vecchia order for the Vecchia approximation); the range
    comes from gp_oracle.cpp (orc_init_range_trafo: the sampled case needs libstdc++'s mt19937,
    shuffle and uniform_int_distribution)."""
    n = coords.shape[0]
    mean = float(np.sum(y)) / n
    var = float(np.sum((y - mean) ** 2)) / (n - 1)
    return np.array([var / 2., 1., O.init_range_trafo(coords, cov_type, seed, shuffled)])


def range_back(cov_type: int, phi: float) -> float:
    return {0: 1. / phi, 1: math.sqrt(3.) / phi, 2: math.sqrt(5.) / phi}.get(cov_type, 1. / math.sqrt(phi))


def lbfgs(f, x, m=6, max_iter=1000, delta=1e-6, step_factor=1.0, max_ls=20, ftol=1e-4,
          max_log_change=math.log(100.)):
    """f(x) -> (fx, grad). Returns (x, fx, iterations)."""
    x = np.array(x, float)
    fx, g = f(x)
    S, Y, YS = [], [], []
    drt = -g
    step = step_factor / np.linalg.norm(drt)
    fx_lag = fx
    k = 1
    while True:
        xp, gp = x.copy(), g.copy()
        step = min(step, max_log_change / np.max(np.abs(drt)))
        fx_init, dg_init = fx, float(g @ drt)
        for it in range(max_ls):
            x = xp + step * drt
            fx, g_new = f(x)
            if fx > fx_init + step * ftol * dg_init or fx != fx:
                step *= 0.5 / 16. if (fx - fx_init) > 2. * max(abs(fx_init), 1.) else 0.5
            else:
                g = g_new
                break
        else:
            x, fx = xp, fx_init
            g = f(x)[1]
        if (fx_lag - fx) <= delta * max(abs(fx_lag), 1.) or k >= max_iter:
            return x, fx, k
        s, yv = x - xp, g - gp
        if float(s @ yv) > np.finfo(float).eps * float(yv @ yv):
            S.append(s); Y.append(yv); YS.append(float(s @ yv))
            if len(S) > m:
                S.pop(0); Y.pop(0); YS.pop(0)
        q = -g.copy()
        alpha = [0.] * len(S)
        for idx in range(len(S) - 1, -1, -1):
            alpha[idx] = float(S[idx] @ q) / YS[idx]
            q -= alpha[idx] * Y[idx]
        if S:
            q /= float(Y[-1] @ Y[-1]) / YS[-1]
        for idx in range(len(S)):
            beta = float(Y[idx] @ q) / YS[idx]
            q += (alpha[idx] - beta) * S[idx]
        drt = q
        step = 1.
        fx_lag = fx
        k += 1


def fit_gaussian(coords, y, cov_type, gp_approx="none", m=30, seed=0, random=True, init_orig=None):
    """Returns (cov_pars_orig, nll, num_it)."""
    if gp_approx == "vecchia":
        perm, xv, nbr = O.vecchia_setup(coords, m, seed, random)
        yv = np.ascontiguousarray(y[perm])

        def ev(trafo):
            return O.vecchia_nll_grad(xv, yv, nbr, cov_type, trafo, 1)
        cx = xv
    else:
        def ev(trafo):
            return O.dense_nll_grad(coords, y, cov_type, trafo, 1)
        cx = coords
    t0 = (O.transform(cov_type, init_orig) if init_orig is not None
          else init_trafo(cx, y, cov_type, seed, gp_approx == "vecchia" and random))
    state = {}

    def f(x):
        r = ev(np.array([1., math.exp(x[0]), math.exp(x[1])]))
        state["sigma2"] = r["sigma2"]
        return r["nll"], np.asarray(r["grad"], float)

    x, fx, k = lbfgs(f, [math.log(t0[1]), math.log(t0[2])])
    f(x)
    s2 = state["sigma2"]
    return np.array([s2, math.exp(x[0]) * s2, range_back(cov_type, math.exp(x[1]))]), fx, k
