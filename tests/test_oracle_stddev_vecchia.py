"""The CPU restatement of the Gaussian Vecchia model's covariance-parameter standard deviations
(oracle/vecchia_fisher_oracle.py: CalcStdDevCovPar re_model_template.h:9775-9789, the stochastic-trace
CalcFisherInformation_Vecchia :9246-9298) pinned to the reference's own outputs
(tests/golden/golden_stddev_vecchia.json, made by make_golden_stddev_vecchia.py from oracle/_ref/ref_harness).
Same probes (GenRandVecNormalParallel), so only rounding separates them: 1e-12 relative.
"""
import json
import os

import numpy as np
import pytest

from gpboost_amd import synthetic
from oracle import oracle as O
from oracle.vecchia_fisher_oracle import vecchia_fisher

HERE = os.path.dirname(os.path.abspath(__file__))
with open(os.path.join(HERE, "golden", "golden_stddev_vecchia.json")) as _f:
    GOLDEN = json.load(_f)


@pytest.mark.parametrize("name", [k for k in GOLDEN if GOLDEN[k]["n"] <= 3000])
def test_oracle_stddev_vecchia_matches_reference(name):
    c = GOLDEN[name]
    sp = c["spec"]
    X = synthetic.bench_coords(c["n"])
    ct = O.cov_code(sp["cov_fct"], float(sp["shape"]))
    _, xv, nb = O.vecchia_setup(X, c["num_neighbors"], sp["seed"], sp["ordering"] == "random")
    FI, sd = vecchia_fisher(xv, nb, ct, c["cov_pars"], t=c["num_rand_vec_trace"] or 50,
                            seed=c["seed_rand_vec_trace"] or 1)
    np.testing.assert_allclose(sd, c["std_dev"], rtol=1e-12)
    assert np.allclose(FI, FI.T) and np.all(np.linalg.eigvalsh(FI) > 0)


def test_oracle_stddev_vecchia_probe_count_matters():
    """The estimate is stochastic: t = 10 and t = 50 give different numbers (both reference fixtures), and
    the oracle reproduces each only with its own probe count."""
    a, b = GOLDEN["sdv_exp_n2000_nn20"], GOLDEN["sdv_exp_n2000_nn20_t10"]
    assert np.max(np.abs(np.array(a["std_dev"]) / b["std_dev"] - 1)) > 1e-3
