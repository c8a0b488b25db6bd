"""CPU: the oracle's GPB_OptimCovPar restatement (oracle/fit_oracle.py) against the reference's
own fits (tests/golden/golden_fit.json, make_golden_fit.py) and the R-test golden
(test_GPModel_gaussian_process.R:233-237). Pins the optimizer algorithm the product's
optim.cpp follows; the product itself is checked on the GPU (tests/test_gpu_optim.py)."""
import json
import os

import numpy as np
import pytest

from gpboost_amd import synthetic
from oracle import fit_oracle as F
from oracle import oracle as O

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def golden_fit():
    with open(os.path.join(HERE, "golden", "golden_fit.json")) as f:
        return json.load(f)


@pytest.mark.parametrize("name", ["rtest_dense_exponential", "rtest_vecchia_m30_random", "rtest_dense_matern15_init"])
def test_oracle_fit_matches_reference(golden_fit, name):
    case = golden_fit[name]
    sp = case["spec"]
    X, Y = synthetic.rtest_gaussian_y(100)
    init = [float(v) for v in sp["init_cov_pars"].split(",")] if "init_cov_pars" in sp else None
    if init is None:
        ct = O.cov_code(sp["cov_fct"], float(sp.get("shape", 0.5)))
        np.testing.assert_allclose(F.init_trafo(X, Y, ct),
                                   O.transform(ct, case["init_cov_pars"]), rtol=1e-12)
    est, nll, k = F.fit_gaussian(X, Y, O.cov_code(sp["cov_fct"], float(sp.get("shape", 0.5))), sp["gp_approx"],
                                 m=sp.get("num_neighbors", 30), random=sp.get("ordering", "random") == "random",
                                 init_orig=init)
    assert k == case["num_it"]
    np.testing.assert_allclose(est, case["cov_pars"], rtol=1e-7)
    assert abs(nll - case["nll"]) <= 1e-10 * abs(case["nll"])


@pytest.mark.parametrize("name", ["synth2000_vecchia_m30_exp", "synth2000_vecchia_m20_gaussian",
                                  "synth2000_vecchia_m30_matern25_init"])   # (dense n=2000: minutes on CPU)
def test_oracle_fit_matches_reference_2000(golden_fit, name):
    # n > 1000: the initial range comes from a 1000-point sample of the model's RNG stream
    case = golden_fit[name]
    sp = case["spec"]
    X, Y = synthetic.bench_coords(2000), synthetic.bench_gaussian_y(2000)
    ct = O.cov_code(sp["cov_fct"], float(sp.get("shape", 0.5)))
    init = [float(v) for v in sp["init_cov_pars"].split(",")] if "init_cov_pars" in sp else None
    if init is None:
        random = sp.get("ordering", "random") == "random" and sp["gp_approx"] == "vecchia"
        cx = X[O.vecchia_order(2000, 0, True)] if random else X
        np.testing.assert_allclose(F.init_trafo(cx, Y, ct, 0, random), O.transform(ct, case["init_cov_pars"]),
                                   rtol=1e-12)
    est, nll, k = F.fit_gaussian(X, Y, ct, sp["gp_approx"], m=sp.get("num_neighbors", 30),
                                 random=sp.get("ordering", "random") == "random", init_orig=init)
    assert k == case["num_it"]
    np.testing.assert_allclose(est, case["cov_pars"], rtol=1e-6)
    assert abs(nll - case["nll"]) <= 1e-10 * abs(case["nll"])


def test_reference_fit_fixture_meets_r_golden(golden_fit):
    case = golden_fit["rtest_dense_exponential"]
    assert np.sum(np.abs(np.array(case["cov_pars"]) - [0.03784221, 1.07390943, 0.11451432])) < 1e-2
    assert abs(case["nll"] - 122.7771373) < 1e-2
