"""Portable synthetic inputs for tests and benchmarks.

The generator is the linear congruential generator the reference's own R tests
use (R-package/tests/testthat/test_GPModel_gaussian_process.R:29-35):

    sim[1] = floor(c * 2^32);  sim[k] = (22695477 * sim[k-1] + 1) %% 2^32;  u = sim / 2^32

evaluated in IEEE double arithmetic exactly as R does it (the product exceeds
2^53, so the rounding is part of the definition). Everything here is input
generation only: no likelihood arithmetic.
"""
from __future__ import annotations

import numpy as np

_MOD = 4294967296.0


def sim_rand_unif(n: int, init_c: float = 0.1) -> np.ndarray:
    """R-test LCG (test_GPModel_gaussian_process.R:29-35), double arithmetic."""
    out = np.empty(n, dtype=np.float64)
    s = float(np.floor(init_c * _MOD))
    out[0] = s
    for k in range(1, n):
        s = (22695477.0 * s + 1.0) % _MOD
        out[k] = s
    return out / _MOD


def rtest_coords(n: int = 100, d: int = 2) -> np.ndarray:
    """coords <- matrix(sim_rand_unif(n*d, 0.1), ncol=d)  (column-major fill)."""
    return sim_rand_unif(n * d, 0.1).reshape(d, n).T.copy()


def rtest_gaussian_y(n: int = 100) -> tuple[np.ndarray, np.ndarray]:
    """The R tests' GP data (test_GPModel_gaussian_process.R:38-61): y = eps + xi."""
    from scipy.stats import norm

    coords = rtest_coords(n)
    diff = coords[:, None, :] - coords[None, :, :]
    dist = np.sqrt((diff ** 2).sum(-1))
    sigma = np.exp(-dist / 0.1) + np.eye(n) * 1e-20
    chol = np.linalg.cholesky(sigma)
    b1 = norm.ppf(sim_rand_unif(n, 0.8))
    eps = chol @ b1
    xi = norm.ppf(sim_rand_unif(n, 0.1)) / 5.0
    return coords, eps + xi


def rtest_bernoulli_probit_y(n: int = 100, init_c: float = 0.19341) -> tuple[np.ndarray, np.ndarray]:
    """R non-Gaussian test data (test_GPModel_non_Gaussian_data.R:17-81 pattern); init_c = 0.2341 gives the data of
    the "Binary classification with Gaussian process model" test (:89-90)."""
    from scipy.stats import norm

    coords = rtest_coords(n)
    diff = coords[:, None, :] - coords[None, :, :]
    dist = np.sqrt((diff ** 2).sum(-1))
    sigma = np.exp(-dist / 0.1) + np.eye(n) * 1e-20
    chol = np.linalg.cholesky(sigma)
    b1 = norm.ppf(sim_rand_unif(n, 0.8))
    eps = chol @ b1
    probs = norm.cdf(eps)
    y = (sim_rand_unif(n, init_c) < probs).astype(np.float64)
    return coords, y


def _rtest_field(n: int = 100) -> tuple[np.ndarray, np.ndarray]:
    from scipy.stats import norm

    coords = rtest_coords(n)
    diff = coords[:, None, :] - coords[None, :, :]
    dist = np.sqrt((diff ** 2).sum(-1))
    chol = np.linalg.cholesky(np.exp(-dist / 0.1) + np.eye(n) * 1e-20)
    return coords, chol @ norm.ppf(sim_rand_unif(n, 0.8))


def rtest_combined_y(n: int = 100) -> tuple[np.ndarray, np.ndarray, np.ndarray]:
    """The R tests' combined GP + grouped random effects data (test_GPModel_combined_GP_random_effects.R:23-79):
    coords, group = rep(1:10, each = n/10), y = L b_1 + Z1 b_gr_1 + xi."""
    from scipy.stats import norm

    coords, field = _rtest_field(n)
    m = 10
    group = np.repeat(np.arange(1, m + 1), n // m)
    b_gr_1 = norm.ppf(sim_rand_unif(m, 0.56))
    xi = norm.ppf(sim_rand_unif(n, 0.1)) / 5.0
    return coords, group, field + b_gr_1[group - 1] + xi


def rtest_poisson_y(n: int = 100) -> tuple[np.ndarray, np.ndarray]:
    """R non-Gaussian test data, spatial Poisson case (test_GPModel_non_Gaussian_data.R:2386-2387):
    y = qpois(sim_rand_unif(n, 0.435), exp(L b_1))."""
    from scipy.stats import poisson

    coords, eps = _rtest_field(n)
    return coords, poisson.ppf(sim_rand_unif(n, 0.435), np.exp(eps)).astype(np.float64)


def rtest_multiple_y(n: int = 100) -> tuple[np.ndarray, np.ndarray]:
    """The R tests' GP data with multiple observations per location (test_GPModel_gaussian_process.R:63-70, 645):
    25 locations from sim_rand_unif(n*d/4, 0.1) repeated 4 times, Sigma = exp(-D / 0.1) + 1e-10 I,
    y = chol(Sigma) qnorm(sim_rand_unif(n, 0.8)) + qnorm(sim_rand_unif(n, 0.1)) / 5."""
    from scipy.stats import norm

    m = n // 4
    c = sim_rand_unif(m * 2, 0.1).reshape(2, m).T
    coords = np.vstack([c, c, c, c])
    dist = np.sqrt(((coords[:, None, :] - coords[None, :, :]) ** 2).sum(-1))
    chol = np.linalg.cholesky(np.exp(-dist / 0.1) + np.eye(n) * 1e-10)
    eps = chol @ norm.ppf(sim_rand_unif(n, 0.8))
    return coords, eps + norm.ppf(sim_rand_unif(n, 0.1)) / 5.


def rtest_gamma_y(n: int = 100, shape: float = 1.0) -> tuple[np.ndarray, np.ndarray]:
    """R non-Gaussian test data, spatial gamma case (test_GPModel_non_Gaussian_data.R:2603-2604):
    y = qgamma(sim_rand_unif(n, 0.435), scale = mu / shape, shape = shape), mu = exp(L b_1)."""
    from scipy.stats import gamma

    coords, eps = _rtest_field(n)
    mu = np.exp(eps)
    return coords, gamma.ppf(sim_rand_unif(n, 0.435), a=shape, scale=mu / shape)


def bench_gamma_y(coords: np.ndarray, shape: float = 2.0) -> np.ndarray:
    """Gamma responses with log-mean 0.3 + sin(2 pi x1) cos(2 pi x2) and the given shape, drawn by inversion of
    the gamma CDF at u from LCG c=0.31415 (exact arithmetic)."""
    from scipy.stats import gamma

    mu = np.exp(0.3 + np.sin(2 * np.pi * coords[:, 0]) * np.cos(2 * np.pi * coords[:, 1]))
    return gamma.ppf(lcg_unif(coords.shape[0], 0.31415), a=shape, scale=mu / shape)


def rtest_probit_X(n: int = 100) -> np.ndarray:
    """X <- cbind(rep(1,n), sin((1:n-n/2)^2*2*pi/n)) (test_GPModel_non_Gaussian_data.R:60)."""
    i = np.arange(1, n + 1, dtype=np.float64)
    return np.column_stack([np.ones(n), np.sin((i - n / 2) ** 2 * 2 * np.pi / n)])


def lcg_unif(n: int, init_c: float = 0.1) -> np.ndarray:
    """The same LCG in exact integer arithmetic, u_{k+1} = (22695477 u_k + 1) mod 2^32.
    The R tests' double-arithmetic version (sim_rand_unif) rounds 22695477 u_k once it exceeds 2^53
    and falls into a cycle of ~40.6k draws: 2n draws for n = 100k coordinates give only 20318
    distinct points. The benchmark generators use this exact form (period 2^32)."""
    out = np.empty(n, dtype=np.float64)
    s = int(np.floor(init_c * _MOD))
    for k in range(n):
        out[k] = s
        s = (22695477 * s + 1) & 0xFFFFFFFF
    return out / _MOD


def bench_coords(n: int, d: int = 2) -> np.ndarray:
    """Benchmark coordinates: 2n LCG draws (c=0.1, exact arithmetic) filled column-major."""
    return lcg_unif(n * d, 0.1).reshape(d, n).T.copy()


def repeated_coords(n: int, n_unique: int, d: int = 2) -> np.ndarray:
    """n observations at n_unique distinct locations (bench_coords(n_unique)), observation i at the
    location floor(u_i n_unique), u from the exact LCG with c = 0.37: locations repeat at random."""
    pts = bench_coords(n_unique, d)
    return pts[np.floor(lcg_unif(n, 0.37) * n_unique).astype(np.int64)].copy()


def cycled_coords(n: int, d: int = 2) -> np.ndarray:
    """The round-1/2 benchmark coordinates: the R tests' double-arithmetic LCG (sim_rand_unif) filled
    column-major; it cycles after ~40.6k draws, so n = 100k gives 20318 distinct locations."""
    return sim_rand_unif(n * d, 0.1).reshape(d, n).T.copy()


def bench_gaussian_y(n: int) -> np.ndarray:
    """iid N(0,1) by Box-Muller from LCG streams c=0.8 and c=0.42 (exact arithmetic)."""
    u1 = np.maximum(lcg_unif(n, 0.8), 1e-300)
    u2 = lcg_unif(n, 0.42)
    return np.sqrt(-2.0 * np.log(u1)) * np.cos(2.0 * np.pi * u2)


def bench_bernoulli_y(coords: np.ndarray) -> np.ndarray:
    """y = 1[u < (1 + sin(2 pi x1) cos(2 pi x2)) / 2], u from LCG c=0.19341 (exact arithmetic)."""
    n = coords.shape[0]
    p = 0.5 * (1.0 + np.sin(2 * np.pi * coords[:, 0]) * np.cos(2 * np.pi * coords[:, 1]))
    return (lcg_unif(n, 0.19341) < p).astype(np.float64)


def bench_poisson_y(coords: np.ndarray) -> np.ndarray:
    """Counts with log-rate 0.5 + sin(2 pi x1) cos(2 pi x2), drawn by inversion of the Poisson CDF
    at u from LCG c=0.27183 (exact arithmetic)."""
    n = coords.shape[0]
    lam = np.exp(0.5 + np.sin(2 * np.pi * coords[:, 0]) * np.cos(2 * np.pi * coords[:, 1]))
    u = lcg_unif(n, 0.27183)
    k = np.zeros(n)
    p = np.exp(-lam)
    cdf = p.copy()
    active = u > cdf
    while active.any():
        k[active] += 1.0
        p[active] *= lam[active] / k[active]
        cdf[active] += p[active]
        active &= u > cdf
    return k


def bench_spatial_gaussian_y(coords: np.ndarray) -> np.ndarray:
    """A Gaussian response with spatial structure: sin(2 pi x1) cos(2 pi x2) + 0.5 iid N(0,1)
    (bench_gaussian_y), for latent-Gaussian fits whose optimum is not at a zero GP variance."""
    f = np.sin(2 * np.pi * coords[:, 0]) * np.cos(2 * np.pi * coords[:, 1])
    return f + 0.5 * bench_gaussian_y(coords.shape[0])


def bench_covariates(n: int, p: int = 2) -> np.ndarray:
    """Linear regression covariates X (n x (p + 1), column-major-friendly): an intercept column and p
    LCG columns (c = 0.31, 0.57, ... exact arithmetic), shifted to mean ~0."""
    cols = [np.ones(n)]
    for k in range(p):
        cols.append(lcg_unif(n, 0.31 + 0.26 * k) - 0.5)
    return np.column_stack(cols)


def bench_gaussian_y_cov(coords: np.ndarray, X: np.ndarray, beta=None) -> np.ndarray:
    """Response with a linear predictor: X beta + iid N(0,1) (bench_gaussian_y) + a smooth spatial term."""
    n = coords.shape[0]
    if beta is None:
        beta = np.array([1.0, 2.0, -1.5, 0.5, -0.25][: X.shape[1]])
    f = np.sin(4 * coords[:, 0]) * np.cos(3 * coords[:, 1])
    return X @ beta + f + 0.5 * bench_gaussian_y(n)


def _normal(n: int, c1: float, c2: float) -> np.ndarray:
    u1 = np.maximum(lcg_unif(n, c1), 1e-300)
    return np.sqrt(-2.0 * np.log(u1)) * np.cos(2.0 * np.pi * lcg_unif(n, c2))


def bench_groups(n: int, levels=(5000, 500)) -> np.ndarray:
    """Crossed grouped random effects (BASELINE config 4 proxy): an n x K integer
    label matrix, effect k uniform over levels[k] from the LCG stream c = 0.23 + 0.17 k."""
    return np.column_stack([np.floor(lcg_unif(n, 0.23 + 0.17 * k) * m).astype(np.int32)
                            for k, m in enumerate(levels)])


def bench_grouped_y(groups: np.ndarray, sd=(1.0, 0.5), noise_sd: float = 1.0) -> np.ndarray:
    """y = sum_k b_k[g_k] + noise, b_k ~ N(0, sd_k^2) per level (LCG Box-Muller streams)."""
    n, K = groups.shape
    y = noise_sd * _normal(n, 0.8, 0.42)
    for k in range(K):
        m = int(groups[:, k].max()) + 1
        b = sd[k % len(sd)] * _normal(m, 0.31 + 0.1 * k, 0.57 + 0.1 * k)
        y = y + b[groups[:, k]]
    return y
