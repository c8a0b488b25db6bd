import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: test needs an MI355X (runs on the GPU box)")
    config.addinivalue_line("markers", "slow: long-running test")


@pytest.fixture(scope="session")
def golden():
    import json
    with open(os.path.join(ROOT, "tests", "golden", "golden_gaussian.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def golden_arrays():
    import numpy as np
    return dict(np.load(os.path.join(ROOT, "tests", "golden", "golden_vecchia_arrays.npz")))


@pytest.fixture(scope="session")
def rtest_data():
    from gpboost_amd import synthetic
    return synthetic.rtest_gaussian_y(100)


@pytest.fixture(scope="session")
def synth2000():
    from gpboost_amd import synthetic
    return synthetic.bench_coords(2000), synthetic.bench_gaussian_y(2000)


@pytest.fixture(scope="session")
def golden_latent():
    import json
    with open(os.path.join(ROOT, "tests", "golden", "golden_latent.json")) as f:
        return json.load(f)


def lik_case_data(case):
    """Inputs of a golden_latent_lik.json case (bernoulli_probit / poisson; make_golden_latent_lik.py)."""
    from gpboost_amd import synthetic
    if case["data"] == "rtest_probit":
        return synthetic.rtest_bernoulli_probit_y(case["n"])
    if case["data"] == "rtest_poisson":
        return synthetic.rtest_poisson_y(case["n"])
    if case["data"] == "rtest_gamma":
        return synthetic.rtest_gamma_y(case["n"])
    X = synthetic.bench_coords(case["n"])
    if case["data"] == "bench_gamma":
        return X, synthetic.bench_gamma_y(X)
    return X, (synthetic.bench_poisson_y(X) if case["data"] == "bench_pois" else synthetic.bench_bernoulli_y(X))


def latent_case_data(case):
    """Inputs of a golden_latent.json case (regenerated from the portable LCG generators)."""
    from gpboost_amd import synthetic
    if case["data"] == "rtest_bern":
        return synthetic.rtest_bernoulli_probit_y(100)
    X = synthetic.bench_coords(case["n"])
    if case["data"] == "bench":
        return X, synthetic.bench_gaussian_y(case["n"])
    return X, synthetic.bench_bernoulli_y(X)
