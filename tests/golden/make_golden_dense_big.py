#!/usr/bin/env python3
"""Reference values for the dense Gaussian path (gp_approx="none") at the sizes where the GPU's
fast paths switch on: n = 8192 and n = 20000 (BASELINE config 2). At these sizes the output of the
trailing updates has >= 512 tiles of 128, so `gemm_f64_big_kernel` and the two-stream lookahead
POTRF run; the n <= 2000 fixtures never reach them.

Build container only (the reference dense path needs ~15 CPU-minutes per evaluation at n = 20000
on 8 cores, ~25 GB of host memory):

    make -C oracle ref && python3 tests/golden/make_golden_dense_big.py [8192] [20000]

Both evaluation modes are recorded: "eval" (nll + gradient incl. the nugget, cov_pars on the
original scale) and "lbfgs" (the L-BFGS objective unit, sigma^2 profiled out). Each finished case is
merged into golden_dense_big.json immediately, so the script can be rerun per size.
"""
from __future__ import annotations

import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden import ROOT, run_ref  # noqa: E402

sys.path.insert(0, ROOT)
from gpboost_amd import synthetic  # noqa: E402

OUT = os.path.join(HERE, "golden_dense_big.json")
PARS = [0.1, 1.0, 0.1]


def main(sizes):
    cases = {}
    if os.path.exists(OUT):
        with open(OUT) as f:
            cases = json.load(f)
    for n in sizes:
        X = synthetic.bench_coords(n)
        y = synthetic.bench_gaussian_y(n)
        t0 = time.time()
        ev = run_ref(X, y, mode="eval", cov_fct="exponential", gp_approx="none", cov_pars="0.1,1.0,0.1")
        t1 = time.time()
        lb = run_ref(X, y, mode="lbfgs", cov_fct="exponential", gp_approx="none", cov_pars="0.1,1.0,0.1")
        t2 = time.time()
        cases[f"synth{n}_dense_exp"] = dict(
            data="bench", n=n, spec=dict(cov_fct="exponential", gp_approx="none"), cov_pars=PARS,
            nll=ev["nll"], grad=ev["grad"], lbfgs_nll=lb["nll"], lbfgs_grad=lb["grad"],
            lbfgs_sigma2=lb["sigma2"], ref_seconds=[round(t1 - t0, 1), round(t2 - t1, 1)], ref_threads=8)
        print(n, ev["nll"], ev["grad"], lb["nll"], lb["grad"], f"{t1 - t0:.0f}s {t2 - t1:.0f}s",
              file=sys.stderr, flush=True)
        with open(OUT, "w") as f:
            json.dump(cases, f, indent=1)


if __name__ == "__main__":
    main([int(a) for a in sys.argv[1:]] or [8192, 20000])
