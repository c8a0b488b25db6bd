#!/usr/bin/env python3
"""Reference fixtures for the Newton mode-change cap of count likelihoods (CapChangeModeUpdateNewton,
likelihoods.h:11800-11810, active for poisson / gamma, :481-490, in the Vecchia and full-scale Vecchia mode finding
:2974, :2606): Poisson counts of a few hundred make the first Newton step from mode 0 exceed log(100), so the
capped trajectory differs from the uncapped one. From the reference itself (oracle/_ref/ref_harness):

    make -C oracle ref && python3 tests/golden/make_golden_mode_cap.py

Counts are deterministic (no random draws): y_i = round(300 exp(sin(4 x_i1) cos(3 x_i2))).
"""
from __future__ import annotations

import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden import ROOT, fmt_pars, run_ref  # noqa: E402

sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

from gpboost_amd import synthetic  # noqa: E402

OUT = os.path.join(HERE, "golden_mode_cap.json")


def data(n):
    X = synthetic.bench_coords(n)
    y = np.round(300. * np.exp(np.sin(4. * X[:, 0]) * np.cos(3. * X[:, 1])))
    return X, y


def main():
    out = {}
    X, y = data(1500)
    cases = [
        ("vecchia_chol_pois_m20", dict(cov_fct="exponential", shape="0.5", gp_approx="vecchia", num_neighbors=20,
                                       ordering="random", likelihood="poisson", matrix_inversion_method="cholesky")),
        ("vif_pois_m40_nn15", dict(cov_fct="exponential", shape="0.5", gp_approx="full_scale_vecchia", num_ind_points=40,
                                   num_neighbors=15, ind_points_selection="kmeans++", seed=0, ordering="random",
                                   likelihood="poisson", matrix_inversion_method="cholesky")),
    ]
    cp = [0.5, 0.2]
    for name, sp in cases:
        r = run_ref(X, y, cov_pars=fmt_pars(cp), mode="eval", **sp)
        out[name] = dict(n=len(y), spec=sp, cov_pars=cp, nll=r["nll"], grad=r["grad"])
        print(name, r["nll"], r["grad"], file=sys.stderr)
    with open(OUT, "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
