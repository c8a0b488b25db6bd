#!/usr/bin/env python3
"""Benchmark: neg-log-lik + grad evaluations / second, n=100k Vecchia m=30 (BASELINE.json).

One "step" = one evaluation of the reference's L-BFGS objective unit
(include/GPBoost/optim_utils.h:243-364): Vecchia factor for all rows, y^T Psi^-1 y,
log|Psi|, sigma2 profiled out, and the gradient w.r.t. the two remaining log-parameters,
at fixed theta, inputs already resident in HBM. Synthetic data from the reference's
portable LCG (gpboost_amd/synthetic.py).

    python bench.py [--gpus N] [--steps K] [--warmup W]

N > 1 is launched by torch.distributed.run (one process per GPU): observations (rows in
Vecchia order) are split into N contiguous blocks, every rank evaluates its rows, and the
six partial sums are all-reduced over RCCL inside the library (strong scaling: the total
problem is fixed). The secondary latent/iterative leg runs at N > 1 with its probe columns
sharded over the ranks (SURVEY.md §8e Option A). Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

N_DATA = 100_000
PRED_N = 100_000                 # prediction points of the secondary prediction leg
M_NEIGHBORS = 30
THETA = [0.1, 1.0, 0.1]          # sigma2, sigma1^2, rho (original scale), exponential kernel
FP64_PEAK_TFLOPS = 78.6          # MI355X FP64 vector = FP64 matrix peak (spec)
RAMP_EVALS_MULTI = 2500          # untimed clock-ramp evaluations at N > 1 (~0.5 s of the 1-GPU rate)
HBM_PEAK_GBS = 8000.0


def vecchia_flops(n: int, m: int, P: int = 2) -> float:
    """F = sum_i [k^3/3 + 2k^2(2+2P) + 2k(2+P)], k_i = min(i, m)."""
    tot = 0.0
    for k in range(0, m):
        tot += k ** 3 / 3 + 2 * k * k * (2 + 2 * P) + 2 * k * (2 + P)
    k = m
    tot += (n - m) * (k ** 3 / 3 + 2 * k * k * (2 + 2 * P) + 2 * k * (2 + P))
    return tot


def vecchia_exps(n: int, m: int) -> float:
    return sum(min(i, m) * (min(i, m) + 1) / 2 for i in range(min(n, m))) + (n - m) * m * (m + 1) / 2


def pmc_traffic(scale: float) -> dict | None:
    """HBM bytes per launch of the row kernel from the committed rocprofv3 PMC passes of this
    same command (profiles/<round>/pmc_rows.json: FETCH_SIZE + WRITE_SIZE, KB per dispatch;
    PMC counters cannot be read from inside the process)."""
    path = None
    for rnd in ("r06", "r05", "r04", "r03", "r02", "r01"):   # the latest round's passes
        cand = os.path.join(ROOT, "profiles", rnd, "pmc_rows.json")
        if os.path.exists(cand):
            path = cand
            break
    if path is None:
        return None
    with open(path) as f:
        p = json.load(f)
    return {"bytes": (p["FETCH_SIZE_KB"] + p["WRITE_SIZE_KB"]) * 1024.0 * scale,
            "source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes), " + os.path.relpath(path, ROOT)}


def cpu_baseline(X, Y, reps: int = 3) -> dict:
    """Reference CPU path on this host (oracle/_ref/ref_harness, the reference GPBoost REModelTemplate
    compiled from its own sources), bounded sample: `reps` evaluations of the same n=100k unit."""
    harness = os.path.join(ROOT, "oracle", "_ref", "ref_harness")
    threads = int(os.environ.get("OMP_NUM_THREADS", str(os.cpu_count() or 1)))
    threads = max(1, min(threads, 16))
    if os.path.exists(harness):
        import numpy as np
        with tempfile.NamedTemporaryFile(suffix=".bin", delete=False) as f:
            f.write(np.array([X.shape[0], X.shape[1]], dtype=np.int32).tobytes())
            f.write(np.ascontiguousarray(X.T).tobytes())
            f.write(np.ascontiguousarray(Y).tobytes())
            path = f.name
        try:
            env = dict(os.environ, OMP_NUM_THREADS=str(threads))
            out = subprocess.run([harness, path, "cov_fct=exponential", "gp_approx=vecchia",
                                  f"num_neighbors={M_NEIGHBORS}", "ordering=random", "mode=lbfgs",
                                  f"reps={reps}", "cov_pars=" + ",".join(map(str, THETA))],
                                 capture_output=True, text=True, timeout=600, env=env, check=True)
            r = json.loads(out.stdout)
            t = r["median_time"]
            return {"value": 1.0 / t, "unit": "evals/s", "cores": threads, "kind": "reference",
                    "sample": f"{reps} L-BFGS-unit evals at n={X.shape[0]} m={M_NEIGHBORS} (median {t:.3f} s/eval; "
                              f"construction {r['t_construct']:.2f} s excluded)", "nll": r["nll"]}
        except Exception as e:  # noqa: BLE001
            sys.stderr.write(f"reference CPU baseline failed: {e}\n")
        finally:
            os.unlink(path)
    # fallback: the oracle restatement, single thread
    from oracle import oracle as O
    perm, xv, nb = O.vecchia_setup(X, M_NEIGHBORS, 0, True)
    tp = O.transform(0, THETA)
    t0 = time.perf_counter()
    O.vecchia_nll_grad(xv, Y[perm], nb, 0, tp, 1)
    t = time.perf_counter() - t0
    return {"value": 1.0 / t, "unit": "evals/s", "cores": 1, "kind": "port",
            "sample": f"1 eval at n={X.shape[0]} (oracle restatement, 1 thread)"}



def pmc_eval_traffic(tag: str, evals: int) -> dict | None:
    """HBM-side bytes per evaluation of a whole path from the latest round's per-kernel PMC passes
    (profiles/<round>/pmc/<tag>_p1.txt FETCH_SIZE, _p2.txt WRITE_SIZE; KiB per dispatch x dispatches, over the
    `evals` evaluations of scripts/time_<tag>.py; raw counter bytes: the gfx950 x2 for 16-B-per-lane streaming reads
    is not applied, the GEMM tiles load 8 B per lane)."""
    import re
    for rnd in ("r06",):
        f1 = os.path.join(ROOT, "profiles", rnd, "pmc", f"{tag}_p1.txt")
        f2 = os.path.join(ROOT, "profiles", rnd, "pmc", f"{tag}_p2.txt")
        if not (os.path.exists(f1) and os.path.exists(f2)):
            continue
        tot = 0.
        for f, key in ((f1, "FETCH_SIZE"), (f2, "WRITE_SIZE")):
            for line in open(f):
                m = re.search(key + r"=([0-9.e+-]+)", line)
                if m and not line.split()[1].startswith("__amd"):
                    tot += int(line.split()[0]) * float(m.group(1)) * 1024.
        return {"bytes": tot / evals, "source": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes), "
                                                f"profiles/{rnd}/pmc/{tag}_p1.txt, _p2.txt, {evals} evaluations"}
    return None


def pmc_ops() -> dict | None:
    """The latest round's PMC summary of the operator / preconditioner kernels (scripts/pmc_ops_json.py)."""
    for rnd in ("r06", "r05", "r04", "r03"):
        path = os.path.join(ROOT, "profiles", rnd, "pmc_ops.json")
        if os.path.exists(path):
            with open(path) as f:
                d = json.load(f)
            d["path"] = ("rocprofv3 --pmc FETCH_SIZE (x2, gfx950 correction) + WRITE_SIZE, separate passes, "
                         + os.path.relpath(path, ROOT))
            return d
    return None


def ops_traffic(ops: dict | None, t: int, part: str) -> float | None:
    """HBM-side bytes per application of the operator ("operator") or the VADU preconditioner
    ("preconditioner") at t columns, from the committed PMC summary."""
    if ops is None:
        return None
    return ops.get("columns", {}).get(str(t), {}).get(part + "_bytes")


def vadu_bytes(n: int, nnz: int, r: int) -> float:
    """one VADU application (B^-T solve and ((D^-1+W)B)^-1 solve) to r columns."""
    return 2 * nnz * 12 + 2 * (n + 1) * 4 + n * 8 + 2 * r * n * 8


def vadu_roofline(n: int, nnz: int, r: int, ms: float, ops: dict | None) -> dict:
    b = vadu_bytes(n, nnz, r)
    ach = b / (ms * 1e-3) / 1e9
    return {"bound": "hbm", "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": ach / HBM_PEAK_GBS,
            "traffic": ops_traffic(ops, r, "preconditioner"), "kernel_ms": ms, "columns": r,
            "algorithmic_bytes_per_launch": b,
            "note": "latency-bound dependency chain (sparse triangular solves over the Vecchia DAG), not bandwidth"}


LATENT_T = 50                     # num_rand_vec_trace (reference default, re_model_template.h:5376)
LATENT_PARS = [1.0, 0.1]          # sigma1^2, rho (original scale); Gaussian error variance (aux) 0.1


def latent_matvec_bytes(n: int, nnz: int, r: int) -> float:
    """one application of A = B^T D^-1 B + W to an n x r block."""
    return 2 * nnz * (8 + 4) + 2 * (n + 1) * 4 + 2 * n * 8 + 2 * r * n * 8


def latent_cpu_baseline(X, Y, reps: int = 1) -> dict | None:
    """The reference's latent-Vecchia iterative evaluation (oracle/_ref/ref_harness) on this host."""
    harness = os.path.join(ROOT, "oracle", "_ref", "ref_harness")
    if not os.path.exists(harness):
        return None
    import numpy as np
    threads = max(1, min(int(os.environ.get("OMP_NUM_THREADS", str(os.cpu_count() or 1))), 16))
    with tempfile.NamedTemporaryFile(suffix=".bin", delete=False) as f:
        f.write(np.array([X.shape[0], X.shape[1]], dtype=np.int32).tobytes())
        f.write(np.ascontiguousarray(X.T).tobytes())
        f.write(np.ascontiguousarray(Y).tobytes())
        path = f.name
    try:
        out = subprocess.run([harness, path, "cov_fct=exponential", "gp_approx=vecchia_latent", "likelihood=gaussian",
                              "matrix_inversion_method=iterative", f"num_neighbors={M_NEIGHBORS}", "ordering=random",
                              "cov_pars=" + ",".join(map(str, LATENT_PARS)), "aux_pars=0.1", "cg_delta_conv=1e-2",
                              f"num_rand_vec_trace={LATENT_T}", "seed_rand_vec_trace=1", f"reps={reps}"],
                             capture_output=True, text=True, timeout=600,
                             env=dict(os.environ, OMP_NUM_THREADS=str(threads)), check=True)
        r = json.loads(out.stdout)
        t = r["median_time"]
        return {"value": 1.0 / t, "unit": "evals/s", "cores": threads, "kind": "reference",
                "sample": f"{reps} latent-Vecchia iterative eval(s) at n={X.shape[0]} (nll+grad, {t:.2f} s/eval)",
                "nll": r["nll"], "grad": r["grad"]}
    except Exception as e:  # noqa: BLE001
        sys.stderr.write(f"reference latent CPU baseline failed: {e}\n")
        return None
    finally:
        os.unlink(path)


def latent_leg(X, Y, steps: int, cpu: bool) -> dict:
    """Secondary measurement: BASELINE config 3 in its PCG + stochastic-trace realisation
    (gp_approx='vecchia_latent', matrix_inversion_method='iterative': Newton solve, block PCG
    with the VADU preconditioner, SLQ log-determinant, stochastic-trace gradient), plus the
    operator roofline of the CG matvec (SURVEY.md §8d bytes / HIP-event time)."""
    import numpy as np

    from gpboost_amd import GPModel
    gm = GPModel(gp_coords=X, likelihood="gaussian", cov_function="exponential", gp_approx="vecchia_latent",
                 num_neighbors=M_NEIGHBORS, vecchia_ordering="random", seed=0, matrix_inversion_method="iterative")
    gm.set_optim_params(dict(num_rand_vec_trace=LATENT_T, init_aux_pars=[0.1]))
    nll, g, _ = gm.neg_log_likelihood_and_grad(LATENT_PARS, Y)          # construction + first eval (warm-up)
    ts = []
    for _ in range(steps):
        t0 = time.perf_counter()
        nll, g, _ = gm.neg_log_likelihood_and_grad(LATENT_PARS, None)
        ts.append(time.perf_counter() - t0)
    info = gm.last_iteration_info()
    r = LATENT_T + 1     # the Gaussian Newton column rides along the probe block (latent.cpp)
    ms_a, ms_p, nnz, nlev = gm.bench_latent_operators(r, 20)
    n = X.shape[0]
    byts = latent_matvec_bytes(n, int(nnz), r)
    ach = byts / (ms_a * 1e-3) / 1e9
    t_med = float(np.median(ts))
    leg = {
        "metric": "latent Vecchia iterative neg-log-lik + grad evals/sec, n=100k m=30",
        "value": 1.0 / t_med, "unit": "evals/s", "steps": steps, "ms_per_step": t_med * 1e3,
        "config": {"workload": "vecchia_latent_gaussian_iterative_vadu", "n": n, "num_neighbors": M_NEIGHBORS,
                   "cov_pars": LATENT_PARS, "aux": 0.1, "num_rand_vec_trace": LATENT_T, "cg_delta_conv": 1e-2,
                   "preconditioner": "vadu", "nll": nll, "grad": [float(x) for x in g],
                   "newton_its": int(info[0]), "cg_its_block": int(info[2])},
        "cg_matvec_roofline": {"bound": "hbm", "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                               "frac": ach / HBM_PEAK_GBS, "traffic": None, "kernel": "b_apply_wave + bt_apply_wave",
                               "kernel_ms": ms_a, "columns": r, "algorithmic_bytes_per_launch": byts},
        "preconditioner": {"kernel": "VaduPrecond: dense MFMA head block (first 2048 Vecchia rows) + LDS segment "
                                     "(rows 2048-14335, one workgroup per column) + merged tail levels (up to 16 "
                                     "dependency levels per launch), replayed from a hipGraph", "ms": ms_p,
                           "launches": int(nlev), "us_per_launch": ms_p * 1e3 / max(nlev, 1),
                           "share_of_eval": None},
    }
    # HBM-side bytes per application from the committed PMC passes of the same operator kernels
    # (scripts/gpu_pmc_ops.sh -> profiles/<round>/pmc_ops.json; FETCH_SIZE doubled, see there)
    ops = pmc_ops()
    if ops is not None:
        leg["cg_matvec_roofline"]["traffic"] = ops_traffic(ops, r, "operator")
        leg["cg_matvec_roofline"]["traffic_source"] = ops["path"]
    # the single-vector CG of the Newton / mode-finding solves (CGVecchiaLaplaceVec, CG_utils.cpp:21-108)
    ms_a1, ms_p1, _, _ = gm.bench_latent_operators(1, 50)
    byts1 = latent_matvec_bytes(n, int(nnz), 1)
    ach1 = byts1 / (ms_a1 * 1e-3) / 1e9
    leg["cg_matvec_roofline_single"] = {"bound": "hbm", "achieved": ach1, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                        "frac": ach1 / HBM_PEAK_GBS,
                                        "traffic": ops_traffic(ops, 1, "operator") if ops else None,
                                        "kernel": "b_apply1e (ELL) + bt_apply1p (paired segmented runs)", "kernel_ms": ms_a1, "columns": 1,
                                        "algorithmic_bytes_per_launch": byts1, "preconditioner_ms": ms_p1}
    leg["preconditioner"]["roofline"] = vadu_roofline(n, int(nnz), r, ms_p, ops)
    leg["preconditioner"]["roofline_single"] = vadu_roofline(n, int(nnz), 1, ms_p1, ops)
    its = int(info[2])
    leg["preconditioner"]["share_of_eval"] = min(1.0, its * ms_p / (t_med * 1e3)) if its > 0 else None
    if cpu:
        leg["cpu_baseline"] = latent_cpu_baseline(X, Y)
    return leg


DENSE_N = 20_000                  # BASELINE config 2: dense Cholesky fp64 on one GPU
DENSE_CPU_N = 4_000               # bounded CPU sample of the same unit (the n=20000 unit is ~800 s)


def bernoulli_cpu_baseline(X, y) -> dict | None:
    """The reference's bernoulli_logit Laplace evaluation (Vecchia m = 30, iterative, VADU, default
    settings) on this host: one nll + gradient evaluation (oracle/_ref/ref_harness; ~30-45 s)."""
    harness = os.path.join(ROOT, "oracle", "_ref", "ref_harness")
    if not os.path.exists(harness):
        return None
    import numpy as np
    threads = max(1, min(int(os.environ.get("OMP_NUM_THREADS", str(os.cpu_count() or 1))), 16))
    with tempfile.NamedTemporaryFile(suffix=".bin", delete=False) as f:
        f.write(np.array([X.shape[0], X.shape[1]], dtype=np.int32).tobytes())
        f.write(np.ascontiguousarray(X.T).tobytes())
        f.write(np.ascontiguousarray(y, dtype=np.float64).tobytes())
        path = f.name
    try:
        out = subprocess.run([harness, path, "cov_fct=exponential", "gp_approx=vecchia", "likelihood=bernoulli_logit",
                              "matrix_inversion_method=iterative", f"num_neighbors={M_NEIGHBORS}", "ordering=random",
                              "cov_pars=" + ",".join(map(str, LATENT_PARS)), "cg_delta_conv=1e-2",
                              f"num_rand_vec_trace={LATENT_T}", "seed_rand_vec_trace=1", "reps=1", "mode=eval"],
                             capture_output=True, text=True, timeout=600,
                             env=dict(os.environ, OMP_NUM_THREADS=str(threads)), check=True)
        r = json.loads(out.stdout)
        t = r["median_time"]
        return {"value": 1.0 / t, "unit": "evals/s", "cores": threads, "kind": "reference",
                "sample": f"1 bernoulli_logit Laplace eval at n={X.shape[0]} (nll+grad, {t:.2f} s/eval; "
                          f"construction {r['t_construct']:.2f} s excluded)", "nll": r["nll"], "grad": r["grad"]}
    except Exception as e:  # noqa: BLE001
        sys.stderr.write(f"reference bernoulli CPU baseline failed: {e}\n")
        return None
    finally:
        os.unlink(path)


def bernoulli_leg(X, steps: int, cpu: bool) -> dict:
    """BASELINE config 5: bernoulli_logit Laplace approximation with Vecchia m = 30 and iterative
    methods (Newton mode finding by PCG, SLQ log-determinant, stochastic-trace gradient), n = 100k;
    the reference's own evaluation of the same data on the host cores beside it (one evaluation)."""
    import numpy as np

    from gpboost_amd import GPModel, synthetic
    y = synthetic.bench_bernoulli_y(X)
    gm = GPModel(gp_coords=X, likelihood="bernoulli_logit", cov_function="exponential", gp_approx="vecchia",
                 num_neighbors=M_NEIGHBORS, vecchia_ordering="random", seed=0, matrix_inversion_method="iterative")
    gm.set_optim_params(dict(num_rand_vec_trace=LATENT_T))
    nll, g, _ = gm.neg_log_likelihood_and_grad(LATENT_PARS, y)          # construction + first eval (warm-up)
    ts = []
    for _ in range(steps):
        t0 = time.perf_counter()
        nll, g, _ = gm.neg_log_likelihood_and_grad(LATENT_PARS, None)
        ts.append(time.perf_counter() - t0)
    info = gm.last_iteration_info()
    t_med = float(np.median(ts))
    n = X.shape[0]
    ms_a, ms_p, nnz, nlev = gm.bench_latent_operators(LATENT_T, 10)
    leg = {"metric": "bernoulli_logit Laplace (Vecchia, iterative) neg-log-lik + grad evals/sec, n=100k m=30",
           "value": 1.0 / t_med, "unit": "evals/s", "steps": steps, "ms_per_step": t_med * 1e3,
           "config": {"workload": "vecchia_bernoulli_logit_laplace_iterative_vadu", "n": n,
                      "num_neighbors": M_NEIGHBORS, "cov_pars": LATENT_PARS, "num_rand_vec_trace": LATENT_T,
                      "cg_delta_conv": 1e-2, "nll": nll, "grad": [float(v) for v in g],
                      "newton_its": int(info[0]), "cg_its_mode": int(info[1]), "lanczos_steps": int(info[2])},
           "preconditioner": {"ms": ms_p, "launches": int(nlev),
                              "roofline": vadu_roofline(n, int(nnz), LATENT_T, ms_p, None)},
           "cpu_baseline": bernoulli_cpu_baseline(X, y) if cpu else None}
    # §8f row f2 for latent models: 5000 new points, latent mean (mode at the parameters, found from
    # zero: one Laplace evaluation) and the response probabilities with simulated variances (1000 draws)
    Xp = synthetic.bench_coords(n + 5000)[n:]
    t0 = time.perf_counter()
    pm = gm.predict(gp_coords_pred=Xp, cov_pars=LATENT_PARS, predict_response=False)
    t_mean = time.perf_counter() - t0
    t0 = time.perf_counter()
    pr = gm.predict(gp_coords_pred=Xp, cov_pars=LATENT_PARS, predict_var=True, predict_response=True)
    t_resp = time.perf_counter() - t0
    leg["prediction"] = {"n_pred": 5000, "vecchia_pred_type": "latent_order_obs_first_cond_obs_only",
                         "mean_s": t_mean, "response_with_var_s": t_resp, "nsim_var_pred": 1000,
                         "mean_of_mu": float(np.mean(pm["mu"])), "mean_prob": float(np.mean(pr["mu"])),
                         "note": "end to end incl. the mode finding at the parameters; variances by 1000 "
                                 "simulated PCG solves in blocks of 50 columns"}
    return leg


CHOL_SAMPLE_N = 10_000            # bounded size of the reference's Cholesky Laplace-Vecchia baseline


def bernoulli_chol_cpu_baseline(n: int) -> dict | None:
    """The reference's bernoulli_logit Laplace evaluation with matrix_inversion_method = "cholesky" (Eigen
    SimplicialLLT per Newton step, L^-1 for the gradient; likelihoods.h:2935-2955, 5207-5336) on this host, at a
    bounded n (the reference's cost grows ~n^2: 6.6 / 23.5 / 97 s at n = 5k / 10k / 20k on 8 cores of the build
    container, so n = 100k is out of reach): one nll + gradient evaluation (oracle/_ref/ref_harness)."""
    harness = os.path.join(ROOT, "oracle", "_ref", "ref_harness")
    if not os.path.exists(harness):
        return None
    import numpy as np

    from gpboost_amd import synthetic
    X = synthetic.bench_coords(n)
    y = synthetic.bench_bernoulli_y(X)
    threads = max(1, min(int(os.environ.get("OMP_NUM_THREADS", str(os.cpu_count() or 1))), 16))
    with tempfile.NamedTemporaryFile(suffix=".bin", delete=False) as f:
        f.write(np.array([X.shape[0], X.shape[1]], dtype=np.int32).tobytes())
        f.write(np.ascontiguousarray(X.T).tobytes())
        f.write(np.ascontiguousarray(y, dtype=np.float64).tobytes())
        path = f.name
    try:
        out = subprocess.run([harness, path, "cov_fct=exponential", "gp_approx=vecchia", "likelihood=bernoulli_logit",
                              "matrix_inversion_method=cholesky", f"num_neighbors={M_NEIGHBORS}", "ordering=random",
                              "cov_pars=" + ",".join(map(str, LATENT_PARS)), "reps=1", "mode=eval"],
                             capture_output=True, text=True, timeout=600,
                             env=dict(os.environ, OMP_NUM_THREADS=str(threads)), check=True)
        r = json.loads(out.stdout)
        t = r["median_time"]
        return {"value": 1.0 / t, "unit": "evals/s", "cores": threads, "kind": "reference",
                "sample": f"1 bernoulli_logit Laplace eval (cholesky) at n={n} (nll+grad, {t:.2f} s/eval; "
                          f"construction {r['t_construct']:.2f} s excluded)", "n": n, "nll": r["nll"],
                "grad": r["grad"]}
    except Exception as e:  # noqa: BLE001
        sys.stderr.write(f"reference cholesky CPU baseline failed: {e}\n")
        return None
    finally:
        os.unlink(path)


def bernoulli_chol_leg(X, steps: int, cpu: bool) -> dict:
    """BASELINE config 5 with the reference's exact Laplace-Vecchia branch (matrix_inversion_method =
    "cholesky"): Newton mode finding on the sparse Cholesky of Sigma^-1 + W (one factorization per Newton step),
    the exact log-determinant and the selected-inverse gradient, n = 100k, m = 30; the same evaluation at the
    reference's bounded sample size beside the reference's own time there."""
    import numpy as np

    from gpboost_amd import GPModel, synthetic

    def model(Xs):
        return GPModel(gp_coords=Xs, likelihood="bernoulli_logit", cov_function="exponential", gp_approx="vecchia",
                       num_neighbors=M_NEIGHBORS, vecchia_ordering="random", seed=0, matrix_inversion_method="cholesky")

    y = synthetic.bench_bernoulli_y(X)
    gm = model(X)
    t0 = time.perf_counter()
    nll, g, _ = gm.neg_log_likelihood_and_grad(LATENT_PARS, y)          # construction + first eval (warm-up)
    t_first = time.perf_counter() - t0
    ts = []
    for _ in range(steps):
        t0 = time.perf_counter()
        nll, g, _ = gm.neg_log_likelihood_and_grad(LATENT_PARS, None)
        ts.append(time.perf_counter() - t0)
    info = gm.last_iteration_info()
    plan = gm.cholesky_plan_info()
    t_med = float(np.median(ts))
    fl, fms = plan["factor_flops"], plan["last_factor_ms"]
    leg = {"metric": "bernoulli_logit Laplace (Vecchia, cholesky) neg-log-lik + grad evals/sec, n=100k m=30",
           "value": 1.0 / t_med, "unit": "evals/s", "steps": steps, "ms_per_step": t_med * 1e3,
           "config": {"workload": "vecchia_bernoulli_logit_laplace_cholesky", "n": X.shape[0],
                      "num_neighbors": M_NEIGHBORS, "cov_pars": LATENT_PARS, "nll": nll,
                      "grad": [float(v) for v in g], "newton_its": int(info[0]), "factorizations": int(info[1])},
           "plan": plan, "construction_and_first_eval_s": t_first,
           "factor_roofline": {"bound": "mfma", "achieved": fl / (fms * 1e-3) / 1e12, "peak": FP64_PEAK_TFLOPS,
                               "unit": "TFLOP/s", "frac": fl / (fms * 1e-3) / 1e12 / FP64_PEAK_TFLOPS,
                               "flops_per_factorization": fl, "ms_per_factorization": fms,
                               "note": "plan flops (POTRF + TRSM + SYRK per front) / HIP-event time of one "
                                       "numeric factorization (all levels, assembly included)"}}
    if cpu:
        base = bernoulli_chol_cpu_baseline(CHOL_SAMPLE_N)
        if base is not None:   # the GPU at the reference's sample size, for a same-size ratio
            Xs = synthetic.bench_coords(CHOL_SAMPLE_N)
            gs = model(Xs)
            ys = synthetic.bench_bernoulli_y(Xs)
            a = gs.neg_log_likelihood_and_grad(LATENT_PARS, ys)
            t0 = time.perf_counter()
            for _ in range(3):
                a = gs.neg_log_likelihood_and_grad(LATENT_PARS, None)
            base["gpu_at_sample_ms"] = (time.perf_counter() - t0) / 3 * 1e3
            base["gpu_nll_at_sample"] = a[0]
        leg["cpu_baseline"] = base
    return leg


GROUPED_N = 500_000               # BASELINE config 4 (expressible proxy)
GROUPED_LEVELS = (5000, 500)
GROUPED_PARS = [1.0, 1.0, 0.25]   # sigma^2, sigma_1^2, sigma_2^2


def grouped_cpu_baseline(g, y, reps: int = 3, fit: bool = True) -> dict | None:
    """The reference's grouped-RE path (oracle/_ref/ref_harness_grouped: REModelTemplate<sp_mat_rm_t>,
    iterative SSOR-PCG + SLQ, default settings) on this host: `reps` L-BFGS-unit evaluations, and one
    fit of the same data."""
    harness = os.path.join(ROOT, "oracle", "_ref", "ref_harness_grouped")
    if not os.path.exists(harness):
        return None
    import numpy as np
    threads = max(1, min(int(os.environ.get("OMP_NUM_THREADS", str(os.cpu_count() or 1))), 16))
    with tempfile.NamedTemporaryFile(suffix=".bin", delete=False) as f:
        f.write(np.array([g.shape[0], 0], dtype=np.int32).tobytes())
        f.write(np.ascontiguousarray(y, dtype=np.float64).tobytes())
        f.write(np.array([0, 0, g.shape[1]], dtype=np.int32).tobytes())   # no covariates, no offset, K
        f.write(np.ascontiguousarray(g.T, dtype=np.int32).tobytes())
        path = f.name
    env = dict(os.environ, OMP_NUM_THREADS=str(threads))
    base = [harness, path, "matrix_inversion_method=iterative", "cg_delta_conv=1e-2", "num_rand_vec_trace=50"]
    try:
        r = json.loads(subprocess.run(base + ["mode=lbfgs", f"reps={reps}", "cov_pars=" + ",".join(map(str, GROUPED_PARS))],
                                      capture_output=True, text=True, timeout=600, env=env, check=True).stdout)
        t = r["median_time"]
        out = {"value": 1.0 / t, "unit": "evals/s", "cores": threads, "kind": "reference", "nll": r["nll"],
               "sample": f"{reps} L-BFGS-unit evals at n={g.shape[0]}, levels {GROUPED_LEVELS} "
                         f"(median {t:.3f} s/eval; construction {r['t_construct']:.2f} s excluded)"}
        if fit:
            rf = json.loads(subprocess.run(base + ["mode=fit"], capture_output=True, text=True, timeout=600,
                                           env=env, check=True).stdout)
            out["fit"] = {"s": rf["fit_time"], "num_it": rf["num_it"], "nll": rf["nll"], "cov_pars": rf["cov_pars"]}
        return out
    except Exception as e:  # noqa: BLE001
        sys.stderr.write(f"reference grouped CPU baseline failed: {e}\n")
        return None
    finally:
        os.unlink(path)


def grouped_leg(steps: int, cpu: bool) -> dict:
    """BASELINE config 4's expressible proxy: n = 500k, two crossed grouped random effects (5000 and
    500 levels), Gaussian likelihood, the reference's default iterative method (SSOR-PCG for
    A^-1 Z^T y, SLQ log-determinant on 50 probes, stochastic-trace gradient), cg_delta_conv 1e-2:
    the L-BFGS unit (nll + gradient, sigma^2 profiled) at fixed parameters, then a whole fit."""
    import numpy as np

    from gpboost_amd import GPModel, synthetic
    g = synthetic.bench_groups(GROUPED_N, GROUPED_LEVELS)
    y = synthetic.bench_grouped_y(g)
    t0 = time.perf_counter()
    gm = GPModel(group_data=g)
    nll, gr, _ = gm.neg_log_likelihood_and_grad(GROUPED_PARS, y, profile_sigma2=True)   # SetY + first eval
    t_construct = time.perf_counter() - t0
    ts = []
    for _ in range(steps):
        t0 = time.perf_counter()
        nll, gr, _ = gm.neg_log_likelihood_and_grad(GROUPED_PARS, None, profile_sigma2=True)
        ts.append(time.perf_counter() - t0)
    t = float(np.median(ts))
    gf = GPModel(group_data=g)
    t0 = time.perf_counter()
    gf.fit(y)
    tf = time.perf_counter() - t0
    leg = {"metric": "grouped RE (2 crossed effects) neg-log-lik + grad evals/sec, n=500k",
           "value": 1.0 / t, "unit": "evals/s", "steps": steps, "ms_per_step": t * 1e3,
           "config": {"workload": "grouped_gaussian_iterative_ssor_lbfgs_unit", "n": GROUPED_N,
                      "levels": list(GROUPED_LEVELS), "cov_pars": GROUPED_PARS, "num_rand_vec_trace": 50,
                      "cg_delta_conv": 1e-2, "construction_s": round(t_construct, 3), "nll": nll,
                      "grad": [float(v) for v in gr]},
           "fit": {"s": tf, "num_it": gf.get_num_optim_iter(), "nll": gf.get_current_neg_log_likelihood(),
                   "cov_pars": [float(v) for v in gf.get_cov_pars()]},
           "cpu_baseline": grouped_cpu_baseline(g, y) if cpu else None}
    return leg


def fit_leg(X, Y, cpu: bool) -> dict:
    """GPB_OptimCovPar end to end on the headline data (reference default optimizer "lbfgs",
    initial values from the reference's FindInitCovPar heuristic), from model construction; the
    reference's own fit of the same data on the host cores beside it (bounded: one fit)."""
    from gpboost_amd import GPModel
    t0 = time.perf_counter()
    gm = GPModel(gp_coords=X, cov_function="exponential", gp_approx="vecchia", num_neighbors=M_NEIGHBORS,
                 vecchia_ordering="random", seed=0)
    gm.fit(Y)
    t = time.perf_counter() - t0
    out = {"workload": f"GPB_OptimCovPar (lbfgs, default settings), n={X.shape[0]} Vecchia m={M_NEIGHBORS}, "
                       "from GPB_CreateREModel (ordering + neighbour search included)",
           "s": t, "num_it": gm.get_num_optim_iter(), "nll": gm.get_current_neg_log_likelihood(),
           "cov_pars": [float(v) for v in gm.get_cov_pars()], "cpu_baseline": None}
    harness = os.path.join(ROOT, "oracle", "_ref", "ref_harness")
    if cpu and os.path.exists(harness):
        import numpy as np
        threads = max(1, min(int(os.environ.get("OMP_NUM_THREADS", str(os.cpu_count() or 1))), 16))
        with tempfile.NamedTemporaryFile(suffix=".bin", delete=False) as f:
            f.write(np.array([X.shape[0], X.shape[1]], dtype=np.int32).tobytes())
            f.write(np.ascontiguousarray(X.T).tobytes())
            f.write(np.ascontiguousarray(Y).tobytes())
            path = f.name
        try:
            r = json.loads(subprocess.run([harness, path, "cov_fct=exponential", "gp_approx=vecchia",
                                           f"num_neighbors={M_NEIGHBORS}", "ordering=random", "mode=fit"],
                                          capture_output=True, text=True, timeout=900, check=True,
                                          env=dict(os.environ, OMP_NUM_THREADS=str(threads))).stdout)
            out["cpu_baseline"] = {"s": r["fit_time"] + r["t_construct"], "fit_s": r["fit_time"],
                                   "construction_s": r["t_construct"], "num_it": r["num_it"],
                                   "num_ll_evaluations": r["num_ll_evaluations"], "nll": r["nll"],
                                   "cov_pars": r["cov_pars"], "cores": threads, "kind": "reference",
                                   "sample": "one reference fit of the same data (construction + OptimLinRegrCoefCovPar)"}
        except Exception as e:  # noqa: BLE001
            sys.stderr.write(f"reference fit baseline failed: {e}\n")
        finally:
            os.unlink(path)
    return out


def dense_flops(n: int) -> float:
    """Algorithmic FLOPs of one dense nll+grad: POTRF n^3/3 + TRTRI n^3/3 + LAUUM n^3/3 (Psi^-1
    for the gradient traces, re_model_template.h:5987-6007); the O(n^2) covariance build, trace
    and triangular-solve terms are left out."""
    return float(n) ** 3


def dense_leg(steps: int, cpu: bool) -> dict:
    """BASELINE config 2: n=20000 2-D spatial GP, dense Cholesky fp64 (gp_approx='none'), the same
    L-BFGS unit (nll + gradient, sigma2 profiled), inputs resident on the GPU."""
    import numpy as np

    from gpboost_amd import GPModel, synthetic
    X = synthetic.bench_coords(DENSE_N)
    Y = synthetic.bench_gaussian_y(DENSE_N)
    gm = GPModel(gp_coords=X, cov_function="exponential", gp_approx="none")
    gm.neg_log_likelihood_and_grad(THETA, Y, profile_sigma2=True)   # warm-up (allocation, first eval)
    ts = []
    for _ in range(steps):
        t0 = time.perf_counter()
        nll, g, _ = gm.neg_log_likelihood_and_grad(THETA, None, profile_sigma2=True)
        ts.append(time.perf_counter() - t0)
    t = float(np.median(ts))
    fl = dense_flops(DENSE_N)
    traffic = pmc_eval_traffic("dense", 4)
    leg = {"metric": "dense nll + grad evals/sec, n=20000", "value": 1.0 / t, "unit": "evals/s", "steps": steps,
           "ms_per_step": t * 1e3,
           "config": {"workload": "dense_gaussian_lbfgs_unit", "n": DENSE_N, "cov_function": "exponential",
                      "theta": THETA, "nll": nll, "grad": [float(x) for x in g]},
           "roofline": {"bound": "mfma", "achieved": fl / t / 1e12, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                        "frac": fl / t / 1e12 / FP64_PEAK_TFLOPS,
                        "traffic": traffic["bytes"] if traffic else None,
                        "traffic_source": traffic["source"] if traffic else None,
                        "kernel": "whole evaluation (POTRF + TRTRI + LAUUM through gemm_f64_big_kernel / "
                                  "gemm_f64_kernel, v_mfma_f64_16x16x4f64)",
                        "algorithmic_flops_per_eval": fl}}
    del gm
    if cpu:
        leg["cpu_baseline"] = dense_cpu_baseline()
    return leg


FITC_N, FITC_M, FITC_CPU_N = 100_000, 500, 20_000


def fitc_flops(n: int, m: int) -> float:
    """Algorithmic fp64 flops of one FITC nll + gradient evaluation (fitc_kernels.hip): the GEMMs
    V = L^-1 K_mn (triangular, m^2 n), W = K_mn K_d^T (2 m^2 n), A = L^-T V (m^2 n), G^T = W^-1 K_mn
    (2 m^2 n), M = dK_mm A (2 m^2 n); the m^3 factorizations and O(n m) passes are not counted."""
    return 8.0 * m * m * n


def fitc_leg(steps: int, cpu: bool) -> dict:
    """FITC (gp_approx='fitc', 500 kmeans++ inducing points) on the headline's
    n=100k coordinates and spatial response, the L-BFGS unit (nll + gradient, sigma2 profiled)."""
    import numpy as np

    from gpboost_amd import GPModel, synthetic
    X = synthetic.bench_coords(FITC_N)
    Y = synthetic.bench_spatial_gaussian_y(X)
    t0 = time.perf_counter()
    gm = GPModel(gp_coords=X, cov_function="exponential", gp_approx="fitc", num_ind_points=FITC_M, seed=0)
    t_construct = time.perf_counter() - t0
    gm.neg_log_likelihood_and_grad(THETA, Y, profile_sigma2=True)   # warm-up
    gm.last_kernel_ms()
    ts, kms = [], []
    for _ in range(steps):
        t0 = time.perf_counter()
        nll, g, _ = gm.neg_log_likelihood_and_grad(THETA, None, profile_sigma2=True)
        ts.append(time.perf_counter() - t0)
        kms.append(gm.last_kernel_ms()[1])
    t = float(np.median(ts))
    fl = fitc_flops(FITC_N, FITC_M)
    kt = float(np.median(kms)) * 1e-3
    leg = {"metric": "FITC nll + grad evals/sec, n=100k, m=500", "value": 1.0 / t, "unit": "evals/s", "steps": steps,
           "ms_per_step": t * 1e3,
           "config": {"workload": "fitc_gaussian_lbfgs_unit", "n": FITC_N, "num_ind_points": FITC_M,
                      "ind_points_selection": "kmeans++", "cov_function": "exponential", "theta": THETA,
                      "construction_s": round(t_construct, 3), "nll": nll, "grad": [float(x) for x in g]},
           "roofline": {"bound": "mfma", "achieved": fl / kt / 1e12, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                        "frac": fl / kt / 1e12 / FP64_PEAK_TFLOPS, "traffic": None, "device_ms": kt * 1e3,
                        "kernel": "whole device evaluation (gemm_f64_big_kernel / gemm_f64_splitk_kernel GEMMs, "
                                  "fitc column kernels)",
                        "algorithmic_flops_per_eval": fl}}
    del gm
    if cpu:
        leg["cpu_baseline"] = fitc_cpu_baseline()
    return leg


def fitc_cpu_baseline() -> dict | None:
    """The reference's FITC path (oracle/_ref/ref_harness gp_approx=fitc) on this host, bounded sample
    at n=20000 (m=500); `value_scaled_n100k` scales it by 20000/100000 (the unit is n m^2-bound)."""
    harness = os.path.join(ROOT, "oracle", "_ref", "ref_harness")
    if not os.path.exists(harness):
        return None
    import numpy as np

    from gpboost_amd import synthetic
    threads = max(1, min(int(os.environ.get("OMP_NUM_THREADS", str(os.cpu_count() or 1))), 16))
    X = synthetic.bench_coords(FITC_CPU_N)
    Y = synthetic.bench_spatial_gaussian_y(X)
    with tempfile.NamedTemporaryFile(suffix=".bin", delete=False) as f:
        f.write(np.array([X.shape[0], X.shape[1]], dtype=np.int32).tobytes())
        f.write(np.ascontiguousarray(X.T).tobytes())
        f.write(np.ascontiguousarray(Y).tobytes())
        path = f.name
    try:
        out = subprocess.run([harness, path, "cov_fct=exponential", "gp_approx=fitc", f"num_ind_points={FITC_M}",
                              "mode=lbfgs", "reps=1", "cov_pars=" + ",".join(map(str, THETA))], capture_output=True,
                             text=True, timeout=600, env=dict(os.environ, OMP_NUM_THREADS=str(threads)), check=True)
        r = json.loads(out.stdout)
        t = r["median_time"]
        return {"value": 1.0 / t, "unit": "evals/s", "cores": threads, "kind": "reference",
                "sample": f"1 FITC L-BFGS-unit eval at n={FITC_CPU_N}, m={FITC_M} ({t:.2f} s; kmeans++ not timed)",
                "value_scaled_n100k": (1.0 / t) * FITC_CPU_N / FITC_N}
    except Exception as e:  # noqa: BLE001
        sys.stderr.write(f"reference FITC CPU baseline failed: {e}\n")
        return None
    finally:
        os.unlink(path)


def fitc_laplace_leg(steps: int, cpu: bool) -> dict:
    """SURVEY §8 row f4, the Laplace rows: FITC with likelihood bernoulli_logit (FindModePostRandEffCalcMLLFITC
    + CalcGradNegMargLikelihoodLaplaceApproxFITC) on the headline's n=100k coordinates, 500 kmeans++
    inducing points: one approximate-marginal-likelihood + gradient evaluation from the zero mode per step
    (the Newton iterations included); the reference on the box's cores at n=20000 beside it."""
    import numpy as np

    from gpboost_amd import GPModel, synthetic
    X = synthetic.bench_coords(FITC_N)
    y = synthetic.bench_bernoulli_y(X)
    gm = GPModel(gp_coords=X, cov_function="exponential", gp_approx="fitc", num_ind_points=FITC_M,
                 likelihood="bernoulli_logit", seed=0)
    gm.neg_log_likelihood_and_grad(LATENT_PARS, y)   # warm-up
    ts = []
    for _ in range(steps):
        t0 = time.perf_counter()
        nll, g, _ = gm.neg_log_likelihood_and_grad(LATENT_PARS, None)
        ts.append(time.perf_counter() - t0)
    info = gm.last_iteration_info()
    t = float(np.median(ts))
    leg = {"metric": "FITC bernoulli_logit Laplace nll + grad evals/sec, n=100k, m=500", "value": 1.0 / t,
           "unit": "evals/s", "steps": steps, "ms_per_step": t * 1e3,
           "config": {"workload": "fitc_bernoulli_logit_laplace_cholesky", "n": FITC_N, "num_ind_points": FITC_M,
                      "cov_function": "exponential", "cov_pars": LATENT_PARS, "nll": nll,
                      "grad": [float(v) for v in g], "newton_its": int(info[0])},
           "note": "per Newton step one split-K MFMA Gram K_mn diag(w) K_nm (2 m^2 n flops) + m x m POTRF/TRTRI + "
                   "five matrix-vector passes over K_mn; gradient: three m^2 n GEMMs + three fused passes"}
    del gm
    if cpu:
        leg["cpu_baseline"] = fitc_laplace_cpu_baseline()
    return leg


def fitc_laplace_cpu_baseline() -> dict | None:
    """The reference's FITC bernoulli_logit evaluation (oracle/_ref/ref_harness) at n=20000, m=500 on this host;
    `value_scaled_n100k` scales it by 20000/100000 (the unit is n m^2-bound)."""
    harness = os.path.join(ROOT, "oracle", "_ref", "ref_harness")
    if not os.path.exists(harness):
        return None
    import numpy as np

    from gpboost_amd import synthetic
    threads = max(1, min(int(os.environ.get("OMP_NUM_THREADS", str(os.cpu_count() or 1))), 16))
    X = synthetic.bench_coords(FITC_CPU_N)
    y = synthetic.bench_bernoulli_y(X)
    with tempfile.NamedTemporaryFile(suffix=".bin", delete=False) as f:
        f.write(np.array([X.shape[0], X.shape[1]], dtype=np.int32).tobytes())
        f.write(np.ascontiguousarray(X.T).tobytes())
        f.write(np.ascontiguousarray(y, dtype=np.float64).tobytes())
        path = f.name
    try:
        out = subprocess.run([harness, path, "cov_fct=exponential", "gp_approx=fitc", f"num_ind_points={FITC_M}",
                              "likelihood=bernoulli_logit", "mode=eval", "reps=1",
                              "cov_pars=" + ",".join(map(str, LATENT_PARS))], capture_output=True, text=True,
                             timeout=600, env=dict(os.environ, OMP_NUM_THREADS=str(threads)), check=True)
        r = json.loads(out.stdout)
        t = r["median_time"]
        return {"value": 1.0 / t, "unit": "evals/s", "cores": threads, "kind": "reference", "nll": r["nll"],
                "sample": f"1 FITC bernoulli_logit eval at n={FITC_CPU_N}, m={FITC_M} ({t:.2f} s; kmeans++ not timed)",
                "value_scaled_n100k": (1.0 / t) * FITC_CPU_N / FITC_N}
    except Exception as e:  # noqa: BLE001
        sys.stderr.write(f"reference FITC-Laplace CPU baseline failed: {e}\n")
        return None
    finally:
        os.unlink(path)


VIF_N, VIF_M, VIF_NN, VIF_CPU_N = 100_000, 200, 30, 20_000   # the reference's VIF defaults (200 / 30)


def vif_flops(n: int, m: int, nn: int) -> float:
    """Algorithmic flops of one VIF nll + gradient: the residual rows' Gram blocks V_S^T [V P_0 P_1]_S
    (3 (nn + 1)^2 m FMAs per point) and the m^2 n GEMMs (V, A, K_mm A, dK_mm A, two L^-1 products, the
    Woodbury Gram, M^-1 X, M^-1 BK: 14 m^2 n); the small Cholesky solves and sparse passes are not counted."""
    return 2.0 * 3 * (nn + 1) ** 2 * m * n + 14.0 * m * m * n


def vif_leg(steps: int, cpu: bool) -> dict:
    """full-scale Vecchia ("VIF", gp_approx='full_scale_vecchia') with the reference's
    defaults (200 kmeans++ inducing points, 30 neighbours) on the headline's n=100k coordinates and spatial
    response, the L-BFGS unit (nll + gradient, sigma2 profiled)."""
    import numpy as np

    from gpboost_amd import GPModel, synthetic
    X = synthetic.bench_coords(VIF_N)
    Y = synthetic.bench_spatial_gaussian_y(X)
    t0 = time.perf_counter()
    gm = GPModel(gp_coords=X, cov_function="exponential", gp_approx="full_scale_vecchia", num_ind_points=VIF_M,
                 num_neighbors=VIF_NN, seed=0)
    t_construct = time.perf_counter() - t0
    gm.neg_log_likelihood_and_grad(THETA, Y, profile_sigma2=True)   # warm-up
    gm.last_kernel_ms()
    ts, kms = [], []
    for _ in range(steps):
        t0 = time.perf_counter()
        nll, g, _ = gm.neg_log_likelihood_and_grad(THETA, None, profile_sigma2=True)
        ts.append(time.perf_counter() - t0)
        kms.append(gm.last_kernel_ms()[1])
    t = float(np.median(ts))
    fl = vif_flops(VIF_N, VIF_M, VIF_NN)
    kt = float(np.median(kms)) * 1e-3
    leg = {"metric": "VIF (full-scale Vecchia) nll + grad evals/sec, n=100k, m=200, nn=30", "value": 1.0 / t,
           "unit": "evals/s", "steps": steps, "ms_per_step": t * 1e3,
           "config": {"workload": "vif_gaussian_lbfgs_unit", "n": VIF_N, "num_ind_points": VIF_M,
                      "num_neighbors": VIF_NN, "ind_points_selection": "kmeans++", "cov_function": "exponential",
                      "theta": THETA, "construction_s": round(t_construct, 3), "nll": nll,
                      "grad": [float(x) for x in g]},
           "roofline": {"bound": "fp64", "achieved": fl / kt / 1e12, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                        "frac": fl / kt / 1e12 / FP64_PEAK_TFLOPS, "traffic": None, "device_ms": kt * 1e3,
                        "kernel": "whole device evaluation (vif_rows_kernel residual factor, MFMA GEMMs, sparse "
                                  "B / B^T passes)",
                        "algorithmic_flops_per_eval": fl}}
    del gm
    if cpu:
        leg["cpu_baseline"] = vif_cpu_baseline()
    return leg


VIFL_CPU_N = 6_000                # bounded size of the reference's VIF Laplace baseline (~n^2 cost: 240 s at 20k)


def vif_laplace_cpu_baseline(n: int) -> dict | None:
    """The reference's VIF Laplace evaluation (FSVA, matrix_inversion_method = "cholesky", bernoulli_logit;
    likelihoods.h:2316-2742, 3886-4925) on this host at a bounded n: one nll + gradient evaluation
    (oracle/_ref/ref_harness)."""
    harness = os.path.join(ROOT, "oracle", "_ref", "ref_harness")
    if not os.path.exists(harness):
        return None
    import numpy as np

    from gpboost_amd import synthetic
    X = synthetic.bench_coords(n)
    y = synthetic.bench_bernoulli_y(X)
    threads = max(1, min(int(os.environ.get("OMP_NUM_THREADS", str(os.cpu_count() or 1))), 16))
    with tempfile.NamedTemporaryFile(suffix=".bin", delete=False) as f:
        f.write(np.array([X.shape[0], X.shape[1]], dtype=np.int32).tobytes())
        f.write(np.ascontiguousarray(X.T).tobytes())
        f.write(np.ascontiguousarray(y, dtype=np.float64).tobytes())
        path = f.name
    try:
        out = subprocess.run([harness, path, "cov_fct=exponential", "gp_approx=full_scale_vecchia",
                              "likelihood=bernoulli_logit", "matrix_inversion_method=cholesky",
                              f"num_ind_points={VIF_M}", f"num_neighbors={VIF_NN}", "ordering=random",
                              "cov_pars=" + ",".join(map(str, LATENT_PARS)), "reps=1", "mode=eval"],
                             capture_output=True, text=True, timeout=600,
                             env=dict(os.environ, OMP_NUM_THREADS=str(threads)), check=True)
        r = json.loads(out.stdout)
        t = r["median_time"]
        return {"value": 1.0 / t, "unit": "evals/s", "cores": threads, "kind": "reference",
                "sample": f"1 bernoulli_logit VIF Laplace eval (cholesky) at n={n}, m={VIF_M}, nn={VIF_NN} (nll+grad, "
                          f"{t:.2f} s/eval; construction excluded)", "n": n, "nll": r["nll"], "grad": r["grad"]}
    except Exception as e:  # noqa: BLE001
        sys.stderr.write(f"reference VIF Laplace CPU baseline failed: {e}\n")
        return None
    finally:
        os.unlink(path)


def vif_laplace_leg(steps: int, cpu: bool) -> dict:
    """SURVEY §8 row f4, non-Gaussian: full-scale Vecchia with the Laplace approximation (the reference's FSVA,
    matrix_inversion_method = "cholesky"): bernoulli_logit on the headline's n = 100k coordinates with the
    reference's VIF defaults (200 kmeans++ inducing points, 30 neighbours): Newton mode finding on the GPU sparse
    Cholesky of B^T D^-1 B + W with the m x m Woodbury correction, exact log-determinant, selected-inverse gradient."""
    import numpy as np

    from gpboost_amd import GPModel, synthetic

    def model(Xs):
        return GPModel(gp_coords=Xs, likelihood="bernoulli_logit", cov_function="exponential",
                       gp_approx="full_scale_vecchia", num_ind_points=VIF_M, num_neighbors=VIF_NN, seed=0,
                       matrix_inversion_method="cholesky")

    X = synthetic.bench_coords(VIF_N)
    y = synthetic.bench_bernoulli_y(X)
    t0 = time.perf_counter()
    gm = model(X)
    nll, g, _ = gm.neg_log_likelihood_and_grad(LATENT_PARS, y)   # construction + first eval (warm-up)
    t_first = time.perf_counter() - t0
    ts = []
    for _ in range(steps):
        t0 = time.perf_counter()
        nll, g, _ = gm.neg_log_likelihood_and_grad(LATENT_PARS, None)
        ts.append(time.perf_counter() - t0)
    info = gm.last_iteration_info()
    plan = gm.cholesky_plan_info()
    t_med = float(np.median(ts))
    leg = {"metric": "bernoulli_logit VIF Laplace (full-scale Vecchia, cholesky) neg-log-lik + grad evals/sec, "
                     "n=100k m=200 nn=30",
           "value": 1.0 / t_med, "unit": "evals/s", "steps": steps, "ms_per_step": t_med * 1e3,
           "config": {"workload": "vif_bernoulli_logit_laplace_cholesky", "n": VIF_N, "num_ind_points": VIF_M,
                      "num_neighbors": VIF_NN, "cov_pars": LATENT_PARS, "nll": nll, "grad": [float(v) for v in g],
                      "newton_its": int(info[0])},
           "plan": plan, "construction_and_first_eval_s": t_first}
    del gm
    if cpu:
        base = vif_laplace_cpu_baseline(VIFL_CPU_N)
        if base is not None:   # the GPU at the reference's sample size
            Xs = synthetic.bench_coords(VIFL_CPU_N)
            gs = model(Xs)
            ys = synthetic.bench_bernoulli_y(Xs)
            a = gs.neg_log_likelihood_and_grad(LATENT_PARS, ys)
            t0 = time.perf_counter()
            for _ in range(3):
                a = gs.neg_log_likelihood_and_grad(LATENT_PARS, None)
            base["gpu_at_sample_ms"] = (time.perf_counter() - t0) / 3 * 1e3
            base["gpu_nll_at_sample"] = a[0]
        leg["cpu_baseline"] = base
    return leg


def vif_cpu_baseline() -> dict | None:
    """The reference's VIF path (oracle/_ref/ref_harness gp_approx=full_scale_vecchia) on this host at
    n=20000 (m=200, nn=30); `value_scaled_n100k` scales it by 20000/100000 (the unit is linear in n)."""
    harness = os.path.join(ROOT, "oracle", "_ref", "ref_harness")
    if not os.path.exists(harness):
        return None
    import numpy as np

    from gpboost_amd import synthetic
    threads = max(1, min(int(os.environ.get("OMP_NUM_THREADS", str(os.cpu_count() or 1))), 16))
    X = synthetic.bench_coords(VIF_CPU_N)
    Y = synthetic.bench_spatial_gaussian_y(X)
    with tempfile.NamedTemporaryFile(suffix=".bin", delete=False) as f:
        f.write(np.array([X.shape[0], X.shape[1]], dtype=np.int32).tobytes())
        f.write(np.ascontiguousarray(X.T).tobytes())
        f.write(np.ascontiguousarray(Y).tobytes())
        path = f.name
    try:
        out = subprocess.run([harness, path, "cov_fct=exponential", "gp_approx=full_scale_vecchia",
                              f"num_ind_points={VIF_M}", f"num_neighbors={VIF_NN}", "mode=lbfgs", "reps=1",
                              "cov_pars=" + ",".join(map(str, THETA))], capture_output=True, text=True, timeout=600,
                             env=dict(os.environ, OMP_NUM_THREADS=str(threads)), check=True)
        r = json.loads(out.stdout)
        t = r["median_time"]
        return {"value": 1.0 / t, "unit": "evals/s", "cores": threads, "kind": "reference",
                "sample": f"1 VIF L-BFGS-unit eval at n={VIF_CPU_N}, m={VIF_M}, nn={VIF_NN} ({t:.2f} s; "
                          f"construction not timed)",
                "value_scaled_n100k": (1.0 / t) * VIF_CPU_N / VIF_N}
    except Exception as e:  # noqa: BLE001
        sys.stderr.write(f"reference VIF CPU baseline failed: {e}\n")
        return None
    finally:
        os.unlink(path)


def dense_cpu_baseline() -> dict | None:
    """The reference's dense path (oracle/_ref/ref_harness) on this host, bounded sample at
    n=4000; `value_scaled_n20000` scales it by (4000/20000)^3 (the unit is n^3-bound)."""
    harness = os.path.join(ROOT, "oracle", "_ref", "ref_harness")
    if not os.path.exists(harness):
        return None
    import numpy as np

    from gpboost_amd import synthetic
    threads = max(1, min(int(os.environ.get("OMP_NUM_THREADS", str(os.cpu_count() or 1))), 16))
    X = synthetic.bench_coords(DENSE_CPU_N)
    Y = synthetic.bench_gaussian_y(DENSE_CPU_N)
    with tempfile.NamedTemporaryFile(suffix=".bin", delete=False) as f:
        f.write(np.array([X.shape[0], X.shape[1]], dtype=np.int32).tobytes())
        f.write(np.ascontiguousarray(X.T).tobytes())
        f.write(np.ascontiguousarray(Y).tobytes())
        path = f.name
    try:
        out = subprocess.run([harness, path, "cov_fct=exponential", "gp_approx=none", "mode=lbfgs", "reps=1",
                              "cov_pars=" + ",".join(map(str, THETA))], capture_output=True, text=True, timeout=600,
                             env=dict(os.environ, OMP_NUM_THREADS=str(threads)), check=True)
        r = json.loads(out.stdout)
        t = r["median_time"]
        rec = {"value": 1.0 / t, "unit": "evals/s", "cores": threads, "kind": "reference",
               "sample": f"1 dense L-BFGS-unit eval at n={DENSE_CPU_N} ({t:.2f} s)",
               "value_scaled_n20000": (1.0 / t) * (DENSE_CPU_N / DENSE_N) ** 3}
        # the full-size reference evaluation measured once on an MI355X box's host cores (230.8 s on 16
        # threads, scripts/ref_dense_n20000.py; too long for every bench run)
        meas = os.path.join(ROOT, "profiles", "r05", "ref_dense_n20000.json")
        if os.path.exists(meas):
            with open(meas) as f:
                m = json.load(f)
            rec["measured_n20000"] = {"value": 1.0 / m["median_time_s"], "unit": "evals/s", "s": m["median_time_s"],
                                      "cores": m["threads"], "nll": m["nll"], "source": "profiles/r05/ref_dense_n20000.json"}
        return rec
    except Exception as e:  # noqa: BLE001
        sys.stderr.write(f"reference dense CPU baseline failed: {e}\n")
        return None
    finally:
        os.unlink(path)


def host_transport() -> bool:
    """GPBOOST_AMD_BENCH_TRANSPORT=host (rehearsal of the N > 1 flow on a one-GPU box): every
    rank on device 0, cross-rank sums through a gloo all-reduce instead of RCCL."""
    return os.environ.get("GPBOOST_AMD_BENCH_TRANSPORT", "rccl") == "host"


def join_ranks(gm, rank: int, world: int, dist) -> None:
    if host_transport():
        import torch

        def allreduce(a):
            dist.all_reduce(torch.from_numpy(a), op=dist.ReduceOp.SUM)
        gm.set_distributed_host(rank, world, allreduce)
        return
    from gpboost_amd import comm_create_id
    obj = [comm_create_id() if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0)
    gm.set_distributed(rank, world, obj[0])


def row_shard_leg(X, Y, reps: int = 200) -> dict:
    """Single-GPU rehearsal of the N-rank row sharding of the headline evaluation: the first and the
    last rank's row range at N = 2, 4, 8 (the shard GPB_EvalVecchiaPartials evaluates, the same launch
    path a rank takes) with the host wall time of the partial evaluation (a fresh model: no kernel HIP
    events are recorded in these evaluations, as in the timed headline loop) and, in a second pass, the
    row-kernel HIP-event time. The N-rank evaluation costs about max(wall over ranks) + one 6-double
    all-reduce."""
    import numpy as np

    from gpboost_amd import GPModel
    gm = GPModel(gp_coords=X, cov_function="exponential", gp_approx="vecchia", num_neighbors=M_NEIGHBORS,
                 vecchia_ordering="random", seed=0)
    gm.neg_log_likelihood_and_grad(THETA, Y, profile_sigma2=True)
    t_end = time.perf_counter() + 0.3
    while time.perf_counter() < t_end:   # clock ramp
        gm.vecchia_partials(THETA, 0, N_DATA)
    n = N_DATA
    out = {}
    shards = {}
    for nr in (2, 4, 8):
        base, rem = divmod(n, nr)   # the library's split (re_model.cpp SetDistributed)
        shards[nr] = {"first": (0, base + (1 if rem else 0)), "last": (n - base, n)}
    for nr, ranges in shards.items():
        res = {}
        for name, (r0, r1) in ranges.items():
            for _ in range(20):
                gm.vecchia_partials(THETA, r0, r1)
            ws = []
            for _ in range(reps):
                t0 = time.perf_counter()
                gm.vecchia_partials(THETA, r0, r1)
                ws.append(time.perf_counter() - t0)
            res[name] = {"rows": [r0, r1], "wall_ms": float(np.median(ws)) * 1e3}
        out[f"n{nr}"] = res
    gm.last_kernel_ms()   # from here on the evaluations record their kernel events
    for nr, ranges in shards.items():
        res = out[f"n{nr}"]
        for name, (r0, r1) in ranges.items():
            ks = []
            for _ in range(20):
                gm.vecchia_partials(THETA, r0, r1)
                ks.append(gm.last_kernel_ms()[0])
            res[name]["kernel_ms"] = float(np.median(ks))
        res["projected_evals_per_s"] = 1e3 / max(v["wall_ms"] for v in res.values() if isinstance(v, dict))
    out["note"] = ("row ranges of an N-rank run evaluated on one GPU (wall: host time of the partial evaluation "
                   "without kernel events; kernel: row-kernel HIP-event time, separate pass); projection excludes "
                   "the all-reduce of 6 doubles over RCCL")
    del gm
    return out


def latent_leg_sharded(X, Y, steps: int, rank: int, world: int, dist) -> dict | None:
    """The latent leg at N > 1: probe columns sharded over the ranks (SURVEY.md §8e Option A,
    RCCL inside the library: one all-reduce of 1 double per PCG iteration + the per-probe terms
    at the end); every rank times its evaluations, the max over ranks is reported."""
    import numpy as np
    import torch

    from gpboost_amd import GPModel
    gm = GPModel(gp_coords=X, likelihood="gaussian", cov_function="exponential", gp_approx="vecchia_latent",
                 num_neighbors=M_NEIGHBORS, vecchia_ordering="random", seed=0, matrix_inversion_method="iterative")
    gm.set_optim_params(dict(num_rand_vec_trace=LATENT_T, init_aux_pars=[0.1]))
    join_ranks(gm, rank, world, dist)
    nll, g, _ = gm.neg_log_likelihood_and_grad(LATENT_PARS, Y)          # construction + first eval (warm-up)
    dist.barrier()
    ts = []
    for _ in range(steps):
        t0 = time.perf_counter()
        nll, g, _ = gm.neg_log_likelihood_and_grad(LATENT_PARS, None)
        ts.append(time.perf_counter() - t0)
    t = torch.tensor([float(np.median(ts))], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    info = gm.last_iteration_info()
    t_med = float(t.item())
    if rank != 0:
        return None
    return {
        "metric": "latent Vecchia iterative neg-log-lik + grad evals/sec, n=100k m=30",
        "value": 1.0 / t_med, "unit": "evals/s", "n_gpus": world, "steps": steps, "ms_per_step": t_med * 1e3,
        "scaling": "strong",
        "config": {"workload": "vecchia_latent_gaussian_iterative_vadu", "n": X.shape[0],
                   "num_neighbors": M_NEIGHBORS, "cov_pars": LATENT_PARS, "aux": 0.1,
                   "num_rand_vec_trace": LATENT_T, "cg_delta_conv": 1e-2, "preconditioner": "vadu",
                   "parallelism": f"probes{world}", "nll": nll, "grad": [float(x) for x in g],
                   "newton_its": int(info[0]), "cg_its_block": int(info[2])},
    }


def spawn_ranks(world: int, argv: list[str]) -> int:
    """`bench.py --gpus N` without an external launcher: start N fresh rank processes (this process
    never touches the GPU), with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT set as
    torch.distributed.run would; relay rank 0's JSON line; non-zero exit if any rank fails."""
    import signal
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    out0 = tempfile.TemporaryFile()
    for r in range(world):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(world), LOCAL_WORLD_SIZE=str(world),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=env,
                                      stdout=out0 if r == 0 else subprocess.DEVNULL, start_new_session=True))
    codes: list = [None] * world
    while any(c is None for c in codes):
        for r, p in enumerate(procs):
            if codes[r] is None:
                codes[r] = p.poll()
        if any(c not in (None, 0) for c in codes):   # a failed rank leaves its peers blocked in a collective
            for r, p in enumerate(procs):
                if codes[r] is None:
                    os.killpg(p.pid, signal.SIGKILL)
                    codes[r] = p.wait()
            break
        time.sleep(0.05)
    out0.seek(0)
    for ln in out0.read().decode().splitlines():   # rank 0's JSON line only
        if ln.startswith("{"):
            sys.stdout.write(ln + "\n")
    sys.stdout.flush()
    bad = [(r, c) for r, c in enumerate(codes) if c]
    if bad:
        sys.stderr.write(f"bench.py: rank(s) failed (rank, exit code): {bad}\n")
        return 1
    return 0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-latent", action="store_true", help="skip the secondary latent/iterative leg")
    ap.add_argument("--latent-steps", type=int, default=3)
    ap.add_argument("--no-dense", action="store_true", help="skip the secondary dense (config 2) leg")
    ap.add_argument("--no-fit", action="store_true", help="skip the secondary GPB_OptimCovPar (fit) leg")
    ap.add_argument("--no-grouped", action="store_true", help="skip the grouped random effects (config 4) leg")
    ap.add_argument("--only-grouped", action="store_true", help="run only the grouped leg (prints its JSON)")
    ap.add_argument("--no-fitc", action="store_true", help="skip the secondary FITC (§8 row f4) leg")
    ap.add_argument("--no-row-shards", action="store_true",
                    help="skip the per-rank row-range measurements (profiling the headline kernel alone)")
    ap.add_argument("--only-fitc", action="store_true", help="run only the FITC legs (prints their JSON)")
    args = ap.parse_args()
    launched = os.environ.get("WORLD_SIZE")
    if launched is not None and int(launched) != args.gpus:
        sys.stderr.write(f"bench.py: --gpus {args.gpus} disagrees with the launcher's WORLD_SIZE={launched}\n")
        sys.exit(2)
    if launched is None and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus, sys.argv[1:]))
    if args.only_grouped:
        print(json.dumps(grouped_leg(args.steps, not args.no_cpu_baseline)))
        return
    if args.only_fitc:
        print(json.dumps({"fitc": fitc_leg(args.steps, not args.no_cpu_baseline),
                          "fitc_laplace": fitc_laplace_leg(3, not args.no_cpu_baseline),
                          "vif": vif_leg(args.steps, not args.no_cpu_baseline)}))
        return

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    os.environ["GPBOOST_AMD_DEVICE"] = "0" if host_transport() else str(local_rank)

    dist = None
    json_out = sys.stdout
    if world > 1:
        # the one-JSON-line contract: gloo / RCCL write status lines to fd 1 from C++; send fd 1 to stderr
        # and keep the real stdout for the JSON line only
        json_out = os.fdopen(os.dup(1), "w")
        sys.stdout.flush()
        os.dup2(2, 1)
        import torch.distributed as dist  # bootstrap + timing only (gloo); data path is RCCL in the library
        dist.init_process_group("gloo")

    import numpy as np

    from gpboost_amd import GPModel, synthetic

    X = synthetic.bench_coords(N_DATA)
    Y = synthetic.bench_gaussian_y(N_DATA)
    t0 = time.perf_counter()
    gm = GPModel(gp_coords=X, cov_function="exponential", gp_approx="vecchia", num_neighbors=M_NEIGHBORS,
                 vecchia_ordering="random", seed=0)
    if world > 1:
        join_ranks(gm, rank, world, dist)
    gm.neg_log_likelihood_and_grad(THETA, Y, profile_sigma2=True)   # SetY + neighbour search + first eval
    t_construct = time.perf_counter() - t0

    # untimed clock ramp before the W counted warm-up steps: the GPU leaves its idle clocks only after
    # some tens of ms of load (a 5-step warm-up measured the row kernel ~8 % slower than after ~100 ms,
    # profiles/r03/rows_env_ab_r03m.log vs bench_r03n.json)
    # Several ranks: a fixed count (every evaluation is a collective, so all ranks must run the same
    # number; a per-rank clock would leave one rank waiting in an all-reduce the others never join)
    if world > 1:
        for _ in range(RAMP_EVALS_MULTI):
            gm.neg_log_likelihood_and_grad(THETA, None, profile_sigma2=True)
    t_ramp = time.perf_counter()
    while world == 1 and time.perf_counter() - t_ramp < 0.5:
        gm.neg_log_likelihood_and_grad(THETA, None, profile_sigma2=True)
    for _ in range(args.warmup):
        gm.neg_log_likelihood_and_grad(THETA, None, profile_sigma2=True)

    if dist is not None:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        nll, g, s2 = gm.neg_log_likelihood_and_grad(THETA, None, profile_sigma2=True)
    elapsed = time.perf_counter() - t0   # each eval returns to the host (synchronised), so wall = device time
    kms = []   # row-kernel HIP-event times, read outside the timed region (same evaluation, repeated)
    gm.last_kernel_ms()   # switches the model's event recording on (off during the timed loop)
    for _ in range(min(args.steps, 20)):
        gm.neg_log_likelihood_and_grad(THETA, None, profile_sigma2=True)
        kms.append(gm.last_kernel_ms())
    latent_sharded = None
    if dist is not None:
        import torch
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        dist.barrier()
        if not args.no_latent:   # every rank takes part (probe-sharded latent leg)
            latent_sharded = latent_leg_sharded(X, Y, args.latent_steps, rank, world, dist)
            dist.barrier()
    if rank != 0:
        dist.destroy_process_group()
        return

    kms = np.array(kms)
    kernel_ms = float(np.mean(kms[:, 0]))
    rows_local = (N_DATA + world - 1) // world
    flops = vecchia_flops(N_DATA, M_NEIGHBORS) * rows_local / N_DATA
    achieved_tf = flops / (kernel_ms * 1e-3) / 1e12
    ms_per_step = elapsed / args.steps * 1e3
    value = args.steps / elapsed
    line = {
        "metric": "neg-log-lik + grad evals/sec, n=100k Vecchia m=30",
        "value": value,
        "unit": "evals/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (the R-test LCG in exact integer arithmetic: 100k distinct uniform 2-D coords, Box-Muller N(0,1) y)",
        "config": {"workload": "vecchia_gaussian_exact_lbfgs_unit", "n": N_DATA, "num_neighbors": M_NEIGHBORS,
                   "cov_function": "exponential", "theta": THETA, "ordering": "random",
                   "parallelism": f"rows{world}", "construction_s": round(t_construct, 3),
                   **({"note": "RCCL row sharding at world_size > 1: first hardware run is this one"} if world > 1 else {}),
                   "nll": nll, "grad": [float(x) for x in g]},
        "roofline": {"bound": "valu", "achieved": achieved_tf, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                     "frac": achieved_tf / FP64_PEAK_TFLOPS, "traffic": None,
                     "kernel": "vecchia_rows16_kernel<matern05,2>", "kernel_ms": kernel_ms,
                     "algorithmic_flops_per_launch": flops,
                     "exp_per_launch": vecchia_exps(N_DATA, M_NEIGHBORS) * rows_local / N_DATA,
                     "note": "fp64 VALU-bound (per-row k<=30 Gauss-Jordan by DPP broadcasts + exp); FP64 vector peak = FP64 matrix peak"},
    }
    traffic = pmc_traffic(rows_local / N_DATA)
    if traffic is not None:
        line["roofline"]["traffic"] = traffic["bytes"]
        line["roofline"]["traffic_source"] = traffic["source"]
    if world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(X, Y)
    else:
        line["cpu_baseline"] = None
    if world == 1:   # §8f row f2: predictions at new points from the same model (end-to-end, incl. the search)
        import numpy as np
        Xp = synthetic.bench_coords(N_DATA + PRED_N)[N_DATA:]
        gm.predict(gp_coords_pred=Xp, cov_pars=THETA, predict_var=True)   # warm-up
        ts = []
        for _ in range(3):
            t0 = time.perf_counter()
            pr = gm.predict(gp_coords_pred=Xp, cov_pars=THETA, predict_var=True)
            ts.append(time.perf_counter() - t0)
        tp = float(np.median(ts))
        line["prediction"] = {"n_pred": PRED_N, "num_neighbors_pred": 2 * M_NEIGHBORS,
                              "vecchia_pred_type": "order_obs_first_cond_obs_only", "ms": tp * 1e3,
                              "predictions_per_s": PRED_N / tp, "mean_of_mu": float(np.mean(pr["mu"])),
                              "note": "end to end: neighbour search among the 100k observed points (GPU), "
                                      "prediction rows (row kernel, 64-lane groups), mean/variance"}
    if world == 1 and not args.no_row_shards:
        line["row_shards"] = row_shard_leg(X, Y)
    if world == 1 and not args.no_fit:
        line["fit"] = fit_leg(X, Y, not args.no_cpu_baseline)
    if world == 1 and not args.no_dense:
        line["dense"] = dense_leg(3, not args.no_cpu_baseline)
    if world == 1 and not args.no_grouped:
        line["grouped"] = grouped_leg(5, not args.no_cpu_baseline)
    if world == 1 and not args.no_fitc:
        line["fitc"] = fitc_leg(5, not args.no_cpu_baseline)
        line["fitc_laplace"] = fitc_laplace_leg(3, not args.no_cpu_baseline)
        line["vif"] = vif_leg(5, not args.no_cpu_baseline)
        line["vif_laplace"] = vif_laplace_leg(3, not args.no_cpu_baseline)
    if world == 1 and not args.no_latent:
        del gm
        if os.environ.get("GPBOOST_AMD_DUMP_MAPS"):   # symbolising a crash under a tracer: the loaded libraries
            with open("/proc/self/maps") as src, open(os.environ["GPBOOST_AMD_DUMP_MAPS"], "w") as dst:
                dst.write(src.read())
        line["latent_iterative"] = latent_leg(X, Y, args.latent_steps, not args.no_cpu_baseline)
        line["bernoulli_laplace"] = bernoulli_leg(X, args.latent_steps, not args.no_cpu_baseline)
        line["bernoulli_laplace_cholesky"] = bernoulli_chol_leg(X, args.latent_steps, not args.no_cpu_baseline)
    elif latent_sharded is not None:
        line["latent_iterative"] = latent_sharded
    print(json.dumps(line), file=json_out)
    json_out.flush()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
    # the JSON line is out: end now instead of tearing down the HIP runtime and the models' device
    # buffers at interpreter exit (a slow teardown outlived the driver's clock, procs_at_end = 1).
    # Profiling runs set GPBOOST_AMD_BENCH_FAST_EXIT=0: a tracer writes its results at normal exit.
    # no child of the bench may outlive it (the driver counts processes at the end): the reference harness runs
    # are waited for by subprocess.run; reap anything else this process started
    try:
        import psutil
        kids = psutil.Process().children(recursive=True)
        for k in kids:
            k.terminate()
        psutil.wait_procs(kids, timeout=5)
    except Exception:  # noqa: BLE001
        pass
    if os.environ.get("GPBOOST_AMD_BENCH_FAST_EXIT", "1") != "0":
        sys.stdout.flush()
        sys.stderr.flush()
        os._exit(0)
