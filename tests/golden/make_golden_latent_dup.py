#!/usr/bin/env python3
"""Golden fixtures for latent Vecchia models with REPEATED coordinates from the reference itself
(oracle/_ref/ref_harness): the reference runs the latent GP on the unique locations with an
incidence matrix (Vecchia_utils.cpp:1121-1139, re_comp.h:845-870; likelihood terms summed per
location). Inputs are regenerated from gpboost_amd.synthetic (repeated_coords / cycled_coords).

    make -C oracle ref && python3 tests/golden/make_golden_latent_dup.py [--big]

--big adds n = 100k on the round-1/2 cycling-LCG coordinates (20318 distinct locations).
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, HERE)
from gpboost_amd import synthetic  # noqa: E402
from make_golden import fmt_pars, run_ref  # noqa: E402

OUT = os.path.join(HERE, "golden_latent_dup.json")


def data(kind, n, nu, lik):
    X = synthetic.repeated_coords(n, nu) if kind == "repeated" else synthetic.cycled_coords(n)
    y = synthetic.bench_bernoulli_y(X) if lik == "bernoulli_logit" else synthetic.bench_gaussian_y(n)
    return X, y


def case(kind, n, nu, lik, cov_pars, fe=False, **opts):
    X, y = data(kind, n, nu, lik)
    f = 0.3 * np.sin(3.0 * X[:, 0]) if fe else None
    spec = dict(cov_fct="exponential", gp_approx="vecchia" if lik == "bernoulli_logit" else "vecchia_latent",
                likelihood=lik, num_neighbors=opts.pop("m", 20), ordering="random",
                matrix_inversion_method="iterative", num_rand_vec_trace=opts.pop("t", 50))
    spec.update(opts)
    ev = run_ref(X, y, fe=f, cov_pars=fmt_pars(cov_pars), mode="eval", **spec)
    return dict(kind=kind, n=n, nu=nu, n_unique=int(len(np.unique(X, axis=0))), lik=lik, cov_pars=list(cov_pars),
                fe=fe, spec=spec, nll=ev["nll"], grad=ev["grad"], ref_time=ev["median_time"])


def main():
    cases = json.load(open(OUT)) if os.path.exists(OUT) else {}
    tight = dict(cg_delta_conv="1e-10")
    if "--big" not in sys.argv:
        cases["bern_rep_n2000_tight"] = case("repeated", 2000, 700, "bernoulli_logit", (1.0, 0.1), **tight)
        cases["bern_rep_n2000_default"] = case("repeated", 2000, 700, "bernoulli_logit", (1.0, 0.1),
                                               cg_delta_conv="1e-2")
        cases["bern_rep_n2000_fe_tight"] = case("repeated", 2000, 700, "bernoulli_logit", (0.8, 0.2), fe=True, **tight)
        cases["gauss_rep_n2000_tight"] = case("repeated", 2000, 700, "gaussian", (1.0, 0.1), aux_pars="0.1", **tight)
        cases["gauss_rep_n3000_m10_t20_tight"] = case("repeated", 3000, 1500, "gaussian", (0.7, 0.15),
                                                      aux_pars="0.3", m=10, t=20, **tight)
    else:
        cases["bern_cycled_n100k_default"] = case("cycled", 100000, 0, "bernoulli_logit", (1.0, 0.1),
                                                  cg_delta_conv="1e-2", m=30)
        cases["bern_cycled_n100k_tight"] = case("cycled", 100000, 0, "bernoulli_logit", (1.0, 0.1),
                                                cg_delta_conv="1e-8", m=30)
        # the reference's own rounding sensitivity at the default tolerance: the same evaluation at
        # parameters perturbed by 1e-14 relative (as make_golden_100k_sens.py for config 5)
        runs = []
        for pars in ((1.0 * (1 + 1e-14), 0.1), (1.0 * (1 - 1e-14), 0.1), (1.0, 0.1 * (1 + 1e-14)),
                     (1.0, 0.1 * (1 - 1e-14))):
            c = case("cycled", 100000, 0, "bernoulli_logit", pars, cg_delta_conv="1e-2", m=30)
            runs.append(dict(cov_pars=list(pars), nll=c["nll"], grad=c["grad"]))
        cases["bern_cycled_n100k_sensitivity"] = dict(rel_perturbation=1e-14, runs=runs, n_unique=c["n_unique"],
                                                      nll=None, grad=None, ref_time=None)
    for k, v in cases.items():
        print(k, v.get("n_unique"), v.get("nll"), v.get("grad"), v.get("ref_time"), file=sys.stderr)
    with open(OUT, "w") as f:
        json.dump(cases, f, indent=1)


if __name__ == "__main__":
    main()
