#!/usr/bin/env python3
"""Reference fixtures for the full-scale Vecchia approximation ("VIF", gp_approx = "full_scale_vecchia",
Gaussian likelihood, cholesky) from the reference itself (oracle/_ref/ref_harness):

    make -C oracle ref && python3 tests/golden/make_golden_vif.py

Per case: the nll and gradient at the given parameters (CalcCovFactor -> CalcCovFactorVecchia +
CalcCovFactorFITC_FSA, CalcYAux, log det re_model_template.h:2698-2714, CalcGradPars_FITC_FSA_GaussLikelihood
:1985-2232) with the nugget as a parameter ("eval") and profiled out ("lbfgs", the L-BFGS objective unit),
log det Psi and y^T Psi^-1 y, the inducing points, and at n <= 3000 the ordering and neighbour lists; plus
fits (GPB_OptimCovPar). Inputs are regenerated from the portable LCG generators (gpboost_amd/synthetic.py).
"""
from __future__ import annotations

import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden import ROOT, fmt_pars, run_ref  # noqa: E402

sys.path.insert(0, ROOT)
from gpboost_amd import synthetic  # noqa: E402

OUT = os.path.join(HERE, "golden_vif.json")


def data(n):
    X = synthetic.bench_coords(n)
    return X, synthetic.bench_spatial_gaussian_y(X)


def spec_of(m, nn, cov_fct="exponential", shape=0.5, sel="kmeans++", seed=0, ordering="random"):
    return dict(cov_fct=cov_fct, shape=str(shape), gp_approx="full_scale_vecchia", num_ind_points=m, num_neighbors=nn,
                ind_points_selection=sel, seed=seed, ordering=ordering)


def case(n, m, nn, cov_pars, dump=True, **kw):
    X, y = data(n)
    spec = spec_of(m, nn, **kw)
    ev = run_ref(X, y, cov_pars=fmt_pars(cov_pars), mode="eval", dump_nn=int(dump), **spec)
    lb = run_ref(X, y, cov_pars=fmt_pars(cov_pars), mode="lbfgs", **spec)
    out = dict(n=n, m=m, num_neighbors=nn, cov_pars=list(cov_pars), spec=spec, nll=ev["nll"], grad=ev["grad"],
               log_det_Psi=ev["log_det_Psi"], yTPsiInvy=ev["yTPsiInvy"], ind_points=ev["ind_points"],
               nll_profiled=lb["nll"], grad_profiled=lb["grad"], sigma2_profiled=lb["sigma2"],
               ref_time_s=ev["median_time"])
    if dump:
        out["perm"] = ev["perm"]
        out["neighbors"] = ev["neighbors"]
    return out


def fit_case(n, m, nn, **kw):
    X, y = data(n)
    spec = spec_of(m, nn, **kw)
    r = run_ref(X, y, mode="fit", **spec)
    return dict(n=n, m=m, num_neighbors=nn, spec=spec, **{k: r[k] for k in r if k not in ("ok", "n", "d")})


def main():
    cases = {
        "vif_exp_n2000_m50_nn10": case(2000, 50, 10, (0.1, 1.0, 0.1)),
        "vif_matern15_n2000_m100_nn20": case(2000, 100, 20, (0.2, 1.3, 0.15), cov_fct="matern", shape=1.5),
        "vif_gauss_n1500_m60_nn15_random": case(1500, 60, 15, (0.3, 0.8, 0.2), cov_fct="gaussian", shape=0.0,
                                                sel="random", seed=3),
        "vif_matern25_n3000_m200_nn30": case(3000, 200, 30, (0.1, 1.0, 0.1), cov_fct="matern", shape=2.5, seed=7),
        "vif_exp_n1000_m40_nn8_none": case(1000, 40, 8, (0.25, 0.7, 0.05), ordering="none"),
        "vif_exp_n20000_m200_nn30": case(20000, 200, 30, (0.25, 1.0, 0.1), dump=False),
    }
    for k, v in cases.items():
        print(k, v["nll"], v["grad"], v["nll_profiled"], v["ref_time_s"], file=sys.stderr)
    fits = {
        "fit_vif_exp_n1000_m30_nn10": fit_case(1000, 30, 10),
        "fit_vif_matern15_n1500_m50_nn15": fit_case(1500, 50, 15, cov_fct="matern", shape=1.5),
    }
    for k, v in fits.items():
        print(k, v["cov_pars"], v["nll"], v["num_it"], file=sys.stderr)
    cases.update(fits)
    with open(OUT, "w") as f:
        json.dump(cases, f)


if __name__ == "__main__":
    main()
