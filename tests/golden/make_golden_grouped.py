#!/usr/bin/env python3
"""Golden fixtures for grouped random effects (BASELINE config 4's expressible proxy)
from the REFERENCE implementation: oracle/_ref/ref_harness_grouped (REModelTemplate<sp_mat_rm_t,
chol_sp_mat_rm_t>, num_gp = 0, compiled from /root/reference by oracle/Makefile).

    make -C oracle ref && python3 tests/golden/make_golden_grouped.py [--big]

Inputs are regenerated from gpboost_amd.synthetic (bench_groups / bench_grouped_y); outputs are the
reference's nll, gradient and fitted parameters. --big adds the config-4-size case (n = 500000,
5000 + 500 levels), whose reference timings are the bench's cpu_baseline source.
"""
from __future__ import annotations

import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, HERE)
from gpboost_amd import synthetic  # noqa: E402
from make_golden import fmt_pars, run_ref  # noqa: E402

OUT = os.path.join(HERE, "golden_grouped.json")


def case(n, levels, cov_pars, **opts):
    g = synthetic.bench_groups(n, levels)
    y = synthetic.bench_grouped_y(g)
    ev = run_ref(None, y, groups=g, cov_pars=fmt_pars(cov_pars), mode="eval", **opts)
    lb = run_ref(None, y, groups=g, cov_pars=fmt_pars(cov_pars), mode="lbfgs", **opts)
    return dict(n=n, levels=list(levels), cov_pars=list(cov_pars), opts=opts,
                nll=ev["nll"], grad=ev["grad"], ref_time=ev["median_time"],
                lbfgs_nll=lb["nll"], lbfgs_grad=lb["grad"], lbfgs_sigma2=lb["sigma2"])


def fit_case(n, levels, **opts):
    g = synthetic.bench_groups(n, levels)
    y = synthetic.bench_grouped_y(g)
    t0 = time.time()
    ft = run_ref(None, y, groups=g, mode="fit", **opts)
    return dict(n=n, levels=list(levels), opts=opts, init_cov_pars=ft["init_cov_pars"], cov_pars=ft["cov_pars"],
                nll=ft["nll"], num_it=ft["num_it"], fit_time=ft["fit_time"], wall=time.time() - t0)


def pred_case(n, levels, cov_pars, calc_var, **opts):
    g = synthetic.bench_groups(n, levels)
    y = synthetic.bench_grouped_y(g)
    r = run_ref(None, y, groups=g, cov_pars=fmt_pars(cov_pars), mode="pred_train", calc_var=int(calc_var), **opts)
    # per observation the reference writes its level's value (mean_pred_id[i] = sigma ZtYAux[level(i)],
    # re_model_template.h:4085, 4113): stored per level (order of first appearance), checked exact
    K = g.shape[1]
    out = dict(n=n, levels=list(levels), cov_pars=list(cov_pars), opts=opts)
    for key in (("mean", "var") if calc_var else ("mean",)):
        v = np.asarray(r[key]).reshape(K, n)
        per = []
        for k in range(K):
            _, first, inv = np.unique(g[:, k], return_index=True, return_inverse=True)
            order = np.argsort(first)              # levels by first appearance
            lev = v[k, first[order]]
            rank = np.empty_like(order)
            rank[order] = np.arange(order.size)
            assert np.array_equal(lev[rank[inv]], v[k]), "per-level values differ within a level"
            per.append(lev.tolist())
        out[key + "_levels"] = per
    return out


def main():
    cases = json.load(open(OUT)) if os.path.exists(OUT) else {}
    it_tight = dict(matrix_inversion_method="iterative", cg_delta_conv="1e-10", num_rand_vec_trace="50")
    it_default = dict(matrix_inversion_method="iterative", cg_delta_conv="1e-2", num_rand_vec_trace="50")
    if "--big" not in sys.argv:
        cases["k1_n5000_cholesky"] = case(5000, (300,), (1.0, 0.5), matrix_inversion_method="cholesky")
        cases["k2_n20000_tight"] = case(20000, (500, 50), (1.0, 1.0, 0.25), **it_tight)
        cases["k2_n20000_default"] = case(20000, (500, 50), (1.0, 1.0, 0.25), **it_default)
        cases["k3_n20000_tight"] = case(20000, (400, 60, 7), (1.0, 1.0, 0.25, 0.1), **it_tight)
        cases["k2_n20000_t20_tight"] = case(20000, (500, 50), (0.8, 0.3, 2.0),
                                            matrix_inversion_method="iterative", cg_delta_conv="1e-10",
                                            num_rand_vec_trace="20", seed_rand_vec_trace="7")
        cases["fit_k1_n5000"] = fit_case(5000, (300,), matrix_inversion_method="cholesky")
        cases["fit_k2_n20000_tight"] = fit_case(20000, (500, 50), matrix_inversion_method="iterative",
                                                cg_delta_conv="1e-10")
        cases["fit_k2_n20000_default"] = fit_case(20000, (500, 50), matrix_inversion_method="iterative")
        cases["pred_train_k1_n5000"] = pred_case(5000, (300,), (1.0, 0.5), True, matrix_inversion_method="cholesky")
        cases["pred_train_k2_n20000_tight"] = pred_case(20000, (500, 50), (1.0, 1.0, 0.25), False, **it_tight)
        cases["pred_train_k3_n20000_default"] = pred_case(20000, (400, 60, 7), (1.0, 1.0, 0.25, 0.1), False,
                                                          **it_default)
        # K >= 2 with matrix_inversion_method = "cholesky" (the reference's sparse Cholesky of
        # Sigma^-1 + Z^T Z, re_model_template.h:8571-8598)
        chol = dict(matrix_inversion_method="cholesky")
        cases["k2_n20000_cholesky"] = case(20000, (500, 50), (1.0, 1.0, 0.25), **chol)
        cases["k3_n20000_cholesky"] = case(20000, (400, 60, 7), (1.0, 1.0, 0.25, 0.1), **chol)
        cases["k2_n3000_cholesky_small"] = case(3000, (900, 3), (0.5, 2.0, 0.05), **chol)
        cases["fit_k2_n20000_cholesky"] = fit_case(20000, (500, 50), **chol)
        cases["fit_k3_n20000_cholesky"] = fit_case(20000, (400, 60, 7), **chol)
        cases["pred_train_k2_n20000_cholesky"] = pred_case(20000, (500, 50), (1.0, 1.0, 0.25), True, **chol)
        cases["pred_train_k3_n20000_cholesky"] = pred_case(20000, (400, 60, 7), (1.0, 1.0, 0.25, 0.1), True, **chol)
    else:
        cases["k2_n500000_default"] = case(500000, (5000, 500), (1.0, 1.0, 0.25), **it_default)
        cases["k2_n500000_tight"] = case(500000, (5000, 500), (1.0, 1.0, 0.25), **it_tight)
        cases["fit_k2_n500000_default"] = fit_case(500000, (5000, 500), matrix_inversion_method="iterative")
    for k, v in cases.items():
        print(k, v.get("nll"), v.get("grad", v.get("cov_pars")), file=sys.stderr)
    with open(OUT, "w") as f:
        json.dump(cases, f, indent=1)


if __name__ == "__main__":
    main()
