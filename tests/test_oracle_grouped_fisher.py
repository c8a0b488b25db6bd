"""The dense CPU restatement of the grouped random effects models' covariance-parameter standard deviations
(oracle/grouped_fisher_oracle.py) pinned to the reference's own outputs (tests/golden/golden_grouped_sd.json,
make_golden_grouped_sd.py from oracle/_ref/ref_harness_grouped): 1e-10 relative on the cases small enough
for dense n x n algebra."""
import json
import os

import numpy as np
import pytest

from gpboost_amd import synthetic
from oracle.grouped_fisher_oracle import grouped_fisher

HERE = os.path.dirname(os.path.abspath(__file__))
with open(os.path.join(HERE, "golden", "golden_grouped_sd.json")) as _f:
    GOLDEN = json.load(_f)


@pytest.mark.parametrize("name", [k for k in GOLDEN if GOLDEN[k]["n"] <= 5000])
def test_oracle_grouped_fisher_matches_reference(name):
    c = GOLDEN[name]
    g = synthetic.bench_groups(c["n"], tuple(c["levels"]))
    _, sd = grouped_fisher(g, c["cov_pars"])
    np.testing.assert_allclose(sd, c["std_dev"], rtol=1e-10)
