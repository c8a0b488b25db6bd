"""ORACLE TEST INFRASTRUCTURE — NOT PART OF THE PRODUCT.

ctypes wrapper for oracle/build/libgp_oracle.so (the CPU restatement, gp_oracle.cpp).
Importable only from tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "libgp_oracle.so")
REF_HARNESS = os.path.join(HERE, "_ref", "ref_harness")

COV_CODES = {("exponential", 0.5): 0, ("matern", 0.5): 0, ("matern", 1.5): 1, ("matern", 2.5): 2,
             ("gaussian", 0.0): 3, ("gaussian", 0.5): 3}

_lib = None


def build():
    subprocess.run(["make", "-s", "-C", HERE, "oracle"], check=True)


def lib():
    global _lib
    if _lib is None:
        build()  # incremental: rebuilds only when a restatement source changed
        L = ctypes.CDLL(LIB_PATH)
        D = ctypes.POINTER(ctypes.c_double)
        I = ctypes.POINTER(ctypes.c_int)
        L.orc_transform_cov_pars.argtypes = [ctypes.c_int, D, D]
        L.orc_vecchia_order.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, I]
        L.orc_find_neighbors.argtypes = [D, ctypes.c_int, ctypes.c_int, ctypes.c_int, I]
        L.orc_find_neighbors_pred.argtypes = [D, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, I]
        L.orc_vecchia_predict.argtypes = [D, D, I, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                          ctypes.c_int, D, ctypes.c_int, D, D]
        L.orc_vecchia_nll_grad.argtypes = [D, D, I, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, D,
                                           ctypes.c_int, D, D, D, D, D]
        L.orc_vecchia_partials.argtypes = [D, D, I, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, D,
                                           ctypes.c_int, ctypes.c_int, D]
        L.orc_dense_nll_grad.argtypes = [D, D, ctypes.c_int, ctypes.c_int, ctypes.c_int, D, ctypes.c_int, D, D, D]
        L.orc_latent_vecchia_factor.argtypes = [D, I, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, D,
                                                D, D, D, D]
        L.orc_init_range_trafo.argtypes = [D, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int]
        L.orc_init_range_trafo.restype = ctypes.c_double
        L.orc_gen_probes.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_ulonglong, D]
        L.orc_latent_vecchia_iterative.argtypes = [D, D, I, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, D,
                                                   ctypes.c_int, ctypes.c_double, ctypes.c_int, ctypes.c_int,
                                                   ctypes.c_double, ctypes.c_int, ctypes.c_int, ctypes.c_int, D, D, D]
        L.orc_fitc_inducing_points.argtypes = [D, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, D]
        L.orc_vif_inducing_points.argtypes = [D, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                               ctypes.c_int, D, I]
        L.orc_fitc_nll_grad.argtypes = [D, D, ctypes.c_int, ctypes.c_int, D, ctypes.c_int, ctypes.c_int, D, ctypes.c_int,
                                        D, D, D]
        _lib = L
    return _lib


def _d(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))


def _i(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_int))


def cov_code(cov_fct: str, shape: float = 0.5) -> int:
    if cov_fct == "gaussian":
        return 3
    if cov_fct == "exponential":
        return 0
    return COV_CODES[(cov_fct, float(shape))]


def transform(cov_type: int, orig) -> np.ndarray:
    o = np.ascontiguousarray(orig, dtype=np.float64)
    t = np.zeros(3)
    lib().orc_transform_cov_pars(cov_type, _d(o), _d(t))
    return t


def vecchia_order(n: int, seed: int = 0, random: bool = True) -> np.ndarray:
    p = np.zeros(n, dtype=np.int32)
    lib().orc_vecchia_order(n, seed, int(random), _i(p))
    return p


def find_neighbors(coords_vo: np.ndarray, m: int) -> np.ndarray:
    x = np.ascontiguousarray(coords_vo, dtype=np.float64)
    n, d = x.shape
    nb = np.zeros((n, m), dtype=np.int32)
    lib().orc_find_neighbors(_d(x), n, d, m, _i(nb))
    return nb


def find_neighbors_pred(coords_vo: np.ndarray, coords_pred: np.ndarray, m: int) -> np.ndarray:
    """Prediction neighbours among the observed points (order_obs_first_cond_obs_only)."""
    x = np.ascontiguousarray(np.vstack([coords_vo, coords_pred]), dtype=np.float64)
    n_obs = coords_vo.shape[0]
    n_all, d = x.shape
    nb = np.zeros((n_all - n_obs, m), dtype=np.int32)
    lib().orc_find_neighbors_pred(_d(x), n_obs, n_all, d, m, _i(nb))
    return nb


def vecchia_predict(coords_vo, y_vo, coords_pred, m_pred, cov_type, pars_trafo, predict_response=True):
    """(mean, var, nbr) of the exact Gaussian Vecchia prediction (order_obs_first_cond_obs_only)."""
    xo = np.ascontiguousarray(coords_vo, dtype=np.float64)
    xp = np.ascontiguousarray(coords_pred, dtype=np.float64)
    m = min(m_pred, xo.shape[0])
    nb = find_neighbors_pred(xo, xp, m)
    x = np.ascontiguousarray(np.vstack([xo, xp]))
    yv = np.ascontiguousarray(y_vo, dtype=np.float64)
    p = np.ascontiguousarray(pars_trafo, dtype=np.float64)
    n_pred = xp.shape[0]
    mean = np.zeros(n_pred)
    var = np.zeros(n_pred)
    if lib().orc_vecchia_predict(_d(x), _d(yv), _i(nb), xo.shape[0], n_pred, x.shape[1], m, cov_type, _d(p),
                                 int(predict_response), _d(mean), _d(var)):
        raise RuntimeError("oracle prediction failed")
    return mean, var, nb


def init_range_trafo(coords_vo: np.ndarray, cov_type: int, seed: int = 0, shuffled: bool = True) -> float:
    """FindInitCovPar's initial phi (transformed range); coords in the component's order."""
    x = np.ascontiguousarray(coords_vo, dtype=np.float64)
    return float(lib().orc_init_range_trafo(_d(x), x.shape[0], x.shape[1], seed, int(shuffled), cov_type))


def vecchia_setup(coords: np.ndarray, m: int, seed: int = 0, random: bool = True):
    perm = vecchia_order(coords.shape[0], seed, random)
    xv = np.ascontiguousarray(coords[perm])
    return perm, xv, find_neighbors(xv, m)


def vecchia_nll_grad(coords_vo, y_vo, nbr, cov_type, pars_trafo, mode, want_factor=False):
    x = np.ascontiguousarray(coords_vo, dtype=np.float64)
    yv = np.ascontiguousarray(y_vo, dtype=np.float64)
    nb = np.ascontiguousarray(nbr, dtype=np.int32)
    n, d = x.shape
    m = nb.shape[1]
    p = np.ascontiguousarray(pars_trafo, dtype=np.float64)
    nll = np.zeros(1)
    grad = np.zeros(3)
    s2 = np.zeros(1)
    Dinv = np.zeros(n) if want_factor else None
    B = np.zeros((n, m)) if want_factor else None
    rc = lib().orc_vecchia_nll_grad(_d(x), _d(yv), _i(nb), n, d, m, cov_type, _d(p), mode, _d(nll), _d(grad), _d(s2),
                                    _d(Dinv) if want_factor else None, _d(B) if want_factor else None)
    if rc != 0:
        raise RuntimeError("oracle vecchia failed")
    g = grad[:3] if mode == 0 else grad[:2]
    out = dict(nll=float(nll[0]), grad=g.copy(), sigma2=float(s2[0]))
    if want_factor:
        out.update(Dinv=Dinv, B=B)
    return out


def vecchia_partials(coords_vo, y_vo, nbr, cov_type, pars_trafo, r0, r1):
    x = np.ascontiguousarray(coords_vo, dtype=np.float64)
    yv = np.ascontiguousarray(y_vo, dtype=np.float64)
    nb = np.ascontiguousarray(nbr, dtype=np.int32)
    n, d = x.shape
    p = np.ascontiguousarray(pars_trafo, dtype=np.float64)
    s = np.zeros(6)
    if lib().orc_vecchia_partials(_d(x), _d(yv), _i(nb), n, d, nb.shape[1], cov_type, _d(p), r0, r1, _d(s)):
        raise RuntimeError("oracle partials failed")
    return s


def dense_nll_grad(coords, y, cov_type, pars_trafo, mode):
    x = np.ascontiguousarray(coords, dtype=np.float64)
    yv = np.ascontiguousarray(y, dtype=np.float64)
    n, d = x.shape
    p = np.ascontiguousarray(pars_trafo, dtype=np.float64)
    nll = np.zeros(1)
    grad = np.zeros(3)
    s2 = np.zeros(1)
    if lib().orc_dense_nll_grad(_d(x), _d(yv), n, d, cov_type, _d(p), mode, _d(nll), _d(grad), _d(s2)):
        raise RuntimeError("oracle dense failed")
    return dict(nll=float(nll[0]), grad=(grad[:3] if mode == 0 else grad[:2]).copy(), sigma2=float(s2[0]))


LIKELIHOODS = {"gaussian": 0, "bernoulli_logit": 1}


def transform_latent(cov_type: int, orig) -> np.ndarray:
    """(sigma1^2, rho) -> (sigma1^2, phi): TransformCovPars without a nugget (non-Gaussian / latent)."""
    t = transform(cov_type, [1.0, orig[0], orig[1]])
    return t[1:].copy()


def latent_factor(coords_vo, nbr, cov_type, trafo2):
    x = np.ascontiguousarray(coords_vo, dtype=np.float64)
    nb = np.ascontiguousarray(nbr, dtype=np.int32)
    n, d = x.shape
    m = nb.shape[1]
    p = np.ascontiguousarray(trafo2, dtype=np.float64)
    B, dB = np.zeros((n, m)), np.zeros((n, m))
    Dinv, dD = np.zeros(n), np.zeros(n)
    if lib().orc_latent_vecchia_factor(_d(x), _i(nb), n, d, m, cov_type, _d(p), _d(B), _d(dB), _d(Dinv), _d(dD)):
        raise RuntimeError("oracle latent factor failed")
    return dict(B=B, dB=dB, Dinv=Dinv, dD=dD)


def gen_probes(n: int, t: int, seed: int = 1, run_id: int = 0) -> np.ndarray:
    R = np.zeros((t, n))   # column-major n x t == row-major t x n
    lib().orc_gen_probes(n, t, seed, run_id, _d(R))
    return R.T


def latent_iterative(coords_vo, y_vo, nbr, cov_type, trafo2, likelihood="gaussian", aux=1.0, t=50, seed=1,
                     cg_delta_conv=1e-2, cg_max_num_it=1000, cg_max_num_it_tridiag=1000, want_grad=True):
    x = np.ascontiguousarray(coords_vo, dtype=np.float64)
    yv = np.ascontiguousarray(y_vo, dtype=np.float64)
    nb = np.ascontiguousarray(nbr, dtype=np.int32)
    n, d = x.shape
    p = np.ascontiguousarray(trafo2, dtype=np.float64)
    nll = np.zeros(1)
    grad = np.zeros(3)
    info = np.zeros(4)
    lk = LIKELIHOODS[likelihood]
    rc = lib().orc_latent_vecchia_iterative(_d(x), _d(yv), _i(nb), n, d, nb.shape[1], cov_type, _d(p), lk,
                                            float(aux), t, seed, cg_delta_conv, cg_max_num_it, cg_max_num_it_tridiag,
                                            int(want_grad), _d(nll), _d(grad), _d(info))
    if rc != 0:
        raise RuntimeError(f"oracle latent iterative failed ({rc})")
    ng = 3 if lk == 0 else 2
    return dict(nll=float(nll[0]), grad=grad[:ng].copy(), newton_its=int(info[0]), cg_its=int(info[1]),
                lanczos_steps=int(info[2]), logdet=float(info[3]))


def fitc_inducing_points(coords, m: int, method: str = "kmeans++", seed: int = 0):
    """Inducing points of CreateREComponentsFITC_FSA (kmeans++ / random) and the Lloyd iteration count."""
    x = np.ascontiguousarray(coords, dtype=np.float64)
    n, d = x.shape
    Z = np.zeros((m, d))
    its = lib().orc_fitc_inducing_points(_d(x), n, d, m, 0 if method == "kmeans++" else 1, seed, _d(Z))
    if its < 0:
        raise ValueError("invalid number of inducing points")
    return Z, its


def vif_inducing_points(coords, m: int, method: str = "kmeans++", seed: int = 0, shuffle: bool = True):
    """full_scale_vecchia: the ordering shuffle, then the inducing points on the coordinates in that order
    with the same generator (re_model_template.h:348-357). Returns (perm, Z, Lloyd iterations)."""
    x = np.ascontiguousarray(coords, dtype=np.float64)
    n, d = x.shape
    Z = np.zeros((m, d))
    perm = np.zeros(n, dtype=np.int32)
    its = lib().orc_vif_inducing_points(_d(x), n, d, m, 0 if method == "kmeans++" else 1, seed, int(shuffle), _d(Z),
                                        _i(perm))
    if its < 0:
        raise ValueError("invalid number of inducing points")
    return perm, Z, its


def fitc_nll_grad(coords, y, Z, cov_type, pars_trafo, mode):
    """FITC Gaussian nll + gradient (transformed scale; mode 0: with the nugget, 1: profiled)."""
    x = np.ascontiguousarray(coords, dtype=np.float64)
    z = np.ascontiguousarray(Z, dtype=np.float64)
    yy = np.ascontiguousarray(y, dtype=np.float64)
    p = np.ascontiguousarray(pars_trafo, dtype=np.float64)
    nll, s2 = np.zeros(1), np.zeros(1)
    g = np.zeros(3 if mode == 0 else 2)
    rc = lib().orc_fitc_nll_grad(_d(x), _d(yy), x.shape[0], x.shape[1], _d(z), z.shape[0], cov_type, _d(p), mode,
                                 _d(nll), _d(g), _d(s2))
    if rc != 0:
        raise ValueError("FITC factorization failed")
    return {"nll": float(nll[0]), "grad": g, "sigma2": float(s2[0])}
