"""GPU parity for the latent Vecchia + iterative-methods path (Laplace approximation with
PCG, stochastic Lanczos quadrature and stochastic-trace gradients; VADU preconditioner).

Reference fixtures: tests/golden/golden_latent.json (the reference run through
oracle/_ref/ref_harness with identical probe vectors). Tolerance: nll and gradient within
1e-6 relative (BASELINE.json north_star). The GPU sums in a different order than Eigen;
with a tight CG tolerance the iterates agree to ~1e-12, at the default cg_delta_conv the
observed gap stays ~1e-8 because both sides stop at the same iteration.
"""
import numpy as np
import pytest

from conftest import latent_case_data
from oracle import oracle as O

pytestmark = pytest.mark.gpu

RTOL = 1e-6


def _model(X, case_like, t=50, seed=1, dc=1e-2):
    from gpboost_amd import GPModel
    lik = case_like["likelihood"]
    gm = GPModel(gp_coords=X, likelihood=lik, cov_function=case_like["cov_fct"],
                 cov_fct_shape=case_like.get("shape", 0.5),
                 gp_approx="vecchia_latent" if lik == "gaussian" else "vecchia",
                 num_neighbors=case_like["num_neighbors"], vecchia_ordering="random",
                 matrix_inversion_method="iterative", seed=0)
    params = dict(num_rand_vec_trace=t, seed_rand_vec_trace=seed, cg_delta_conv=dc)
    if lik == "gaussian":
        params["init_aux_pars"] = [case_like["aux"]]
    gm.set_optim_params(params)
    return gm


def _check(nll, g, ref_nll, ref_g, rtol=RTOL, atol_g=0.):
    assert abs(nll - ref_nll) <= rtol * abs(ref_nll), (nll, ref_nll)
    ref_g = np.asarray(ref_g)
    assert g.shape == ref_g.shape, (g, ref_g)
    np.testing.assert_allclose(g, ref_g, rtol=rtol, atol=max(rtol * np.abs(ref_g).max(), atol_g))


@pytest.mark.parametrize("name", ["gauss_m30_exp_tight", "gauss_m30_exp_default", "gauss_m20_matern15_t20",
                                  "bern_m30_exp_tight", "bern_m30_exp_default", "bern_m10_gaussian_t30",
                                  "bern_m16_matern25", "rtest_bern_m30_exp"])
def test_latent_matches_reference(golden_latent, name):
    case = golden_latent[name]
    X, y = latent_case_data(case)
    gm = _model(X, case, t=case["num_rand_vec_trace"], seed=case["seed_rand_vec_trace"], dc=case["cg_delta_conv"])
    nll = gm.neg_log_likelihood(case["cov_pars"], y)
    assert abs(nll - case["nll"]) <= RTOL * abs(case["nll"])
    nll2, g, _ = gm.neg_log_likelihood_and_grad(case["cov_pars"], None)
    _check(nll2, g, case["nll"], case["grad"], atol_g=COND_LIMITED_ATOL.get(name, 0.))


# Conditioning-limited case (Gaussian kernel, no nugget: kappa(C_i) ~ 1e8+): its gradient carries
# implementation noise, measured ONCE as the largest gap between two independent CPU implementations
# (the reference and the oracle restatement, max |g_oracle - g_ref| = 1.55e-4 at n = 2000); the GPU
# must stay within 10x that fixed value. Every other case is held to 1e-6 relative (their measured
# oracle-reference gaps are 1e-14 .. 9e-5 absolute, all below 1e-6 relative).
COND_LIMITED_ATOL = {"bern_m10_gaussian_t30": 1.6e-3}


def test_latent_factor_matches_oracle():
    from gpboost_amd import synthetic
    X = synthetic.bench_coords(3000)
    # the Gaussian kernel at a short range keeps C_i moderately conditioned (no nugget)
    for cov, shape, ct, m, pars in [("exponential", 0.5, 0, 30, [1.2, 0.13]), ("matern", 1.5, 1, 17, [1.2, 0.13]),
                                    ("matern", 2.5, 2, 5, [1.2, 0.13]), ("gaussian", 0.5, 3, 48, [1.2, 0.02])]:
        case = dict(likelihood="bernoulli_logit", cov_fct=cov, shape=shape, num_neighbors=m)
        gm = _model(X, case)
        f = gm.latent_vecchia_factor(pars)
        perm, xv, nb = O.vecchia_setup(X, m, 0, True)
        ref = O.latent_factor(xv, nb, ct, O.transform_latent(ct, pars))
        # D = var - a.c cancels for well-predicted points: compare D on the scale of var
        np.testing.assert_allclose(1 / f["Dinv"], 1 / ref["Dinv"], rtol=1e-8, atol=1e-9 * pars[0])
        np.testing.assert_allclose(f["dD"], ref["dD"], rtol=1e-7, atol=1e-9)
        np.testing.assert_allclose(f["B"], ref["B"], rtol=1e-7, atol=1e-9)
        np.testing.assert_allclose(f["dB"], ref["dB"], rtol=1e-6, atol=1e-8)


@pytest.mark.parametrize("lik", ["gaussian", "bernoulli_logit"])
def test_latent_vs_oracle_20000(lik):
    """Larger n at a tight CG tolerance. (At the default cg_delta_conv the hundreds of
    block-CG steps amplify summation-order differences, so two correct implementations
    stop a few iterations apart and agree only to ~1e-5; the tight tolerance removes that
    truncation sensitivity.)"""
    from gpboost_amd import synthetic
    n = 20000
    X = synthetic.bench_coords(n)
    y = synthetic.bench_gaussian_y(n) if lik == "gaussian" else synthetic.bench_bernoulli_y(X)
    case = dict(likelihood=lik, cov_fct="exponential", shape=0.5, num_neighbors=30, aux=0.1)
    gm = _model(X, case, t=10, dc=1e-8)
    nll, g, _ = gm.neg_log_likelihood_and_grad([1.0, 0.1], y)
    perm, xv, nb = O.vecchia_setup(X, 30, 0, True)
    ref = O.latent_iterative(xv, y[perm], nb, 0, O.transform_latent(0, [1.0, 0.1]), lik, 0.1, t=10,
                             cg_delta_conv=1e-8)
    _check(nll, g, ref["nll"], ref["grad"])
    info = gm.last_iteration_info()
    assert info[0] == ref["newton_its"]
    assert abs(info[2] - ref["lanczos_steps"]) <= 0.05 * ref["lanczos_steps"]


def test_latent_edge_cases():
    """Few probes (t = 1), one neighbour, tiny n (levels of size 1), probes wider than 64
    (two column chunks)."""
    from gpboost_amd import synthetic
    for n, m, t, lik in [(400, 1, 1, "bernoulli_logit"), (5, 3, 7, "gaussian"), (600, 8, 70, "gaussian"),
                         (50, 49, 4, "bernoulli_logit")]:
        X = synthetic.bench_coords(n)
        y = synthetic.bench_gaussian_y(n) if lik == "gaussian" else synthetic.bench_bernoulli_y(X)
        case = dict(likelihood=lik, cov_fct="exponential", shape=0.5, num_neighbors=m, aux=0.4)
        gm = _model(X, case, t=t, seed=2, dc=1e-6)
        nll, g, _ = gm.neg_log_likelihood_and_grad([0.9, 0.2], y)
        mm = min(m, n - 1)
        perm, xv, nb = O.vecchia_setup(X, mm, 0, True)
        ref = O.latent_iterative(xv, y[perm], nb, 0, O.transform_latent(0, [0.9, 0.2]), lik, 0.4, t=t, seed=2,
                                 cg_delta_conv=1e-6)
        _check(nll, g, ref["nll"], ref["grad"])


@pytest.mark.parametrize("lik", ["gaussian", "bernoulli_logit"])
def test_latent_100k_deterministic(lik):
    """BASELINE config 3b / 5 size: repeated evaluations are bitwise identical (fixed-order
    reductions, probes drawn once) and finite."""
    from gpboost_amd import synthetic
    n = 100_000
    X = synthetic.bench_coords(n)
    y = synthetic.bench_gaussian_y(n) if lik == "gaussian" else synthetic.bench_bernoulli_y(X)
    case = dict(likelihood=lik, cov_fct="exponential", shape=0.5, num_neighbors=30, aux=0.1)
    gm = _model(X, case)
    a = gm.neg_log_likelihood_and_grad([1.0, 0.1], y)
    b = gm.neg_log_likelihood_and_grad([1.0, 0.1], None)
    assert a[0] == b[0] and np.array_equal(a[1], b[1])
    assert np.isfinite(a[0]) and np.all(np.isfinite(a[1]))


def test_latent_errors():
    from gpboost_amd import GPBoostError, GPModel, synthetic
    X = synthetic.bench_coords(200)
    gm = GPModel(gp_coords=X, likelihood="bernoulli_logit", gp_approx="vecchia", num_neighbors=10,
                 matrix_inversion_method="iterative")
    with pytest.raises(GPBoostError, match="0 or 1"):
        gm.neg_log_likelihood([1.0, 0.1], np.linspace(0, 2, 200))
    with pytest.raises(GPBoostError, match="cholesky"):
        GPModel(gp_coords=X, likelihood="bernoulli_logit", gp_approx="vecchia", matrix_inversion_method="lu")
    with pytest.raises(GPBoostError, match="profile_sigma2"):
        gm.neg_log_likelihood_and_grad([1.0, 0.1], synthetic.bench_bernoulli_y(X), profile_sigma2=True)


@pytest.mark.parametrize("dense_rows,head_rows,merge", [("0", "100", "1"), ("0", "6000", "4"), ("2048", "2048", "4"),
                                                         ("512", "5000", "2"), ("2048", "8000", "4"),
                                                         ("8000", "8000", "4"), ("0", "0", "4"), ("1024", "3000", "9")])
def test_preconditioner_plans_agree(monkeypatch, dense_rows, head_rows, merge):
    """The three-part VADU plan (vadu_precond.h: dense head [0, K0), LDS segment [K0, K), merged
    level kernels for the tail, g levels per launch) against the plain level schedule (K0 = K = 0,
    g = 1) on the same model. The solves are the same algebra; the dense block (an explicit
    inverse), the substituted coefficients of merged levels and the entry splits change only the
    rounding, so at a tight CG tolerance the evaluations agree to ~1e-10. Covers a tiny segment,
    segment only, dense + tail, all three parts, dense + segment (no tail), dense only, and merged
    tails without a head."""
    from gpboost_amd import synthetic
    n = 8000
    X = synthetic.bench_coords(n)
    for lik in ("gaussian", "bernoulli_logit"):
        y = synthetic.bench_gaussian_y(n) if lik == "gaussian" else synthetic.bench_bernoulli_y(X)
        case = dict(likelihood=lik, cov_fct="exponential", shape=0.5, num_neighbors=30, aux=0.1)
        out = {}
        for key, (k0, k, g) in {"levels": ("0", "0", "1"), "plan": (dense_rows, head_rows, merge)}.items():
            monkeypatch.setenv("GPBOOST_AMD_DENSE_ROWS", k0)
            monkeypatch.setenv("GPBOOST_AMD_HEAD_ROWS", k)
            monkeypatch.setenv("GPBOOST_AMD_TAIL_MERGE", g)
            gm = _model(X, case, t=12, dc=1e-9)
            out[key] = gm.neg_log_likelihood_and_grad([1.0, 0.1], y)
        a, b = out["levels"], out["plan"]
        assert abs(a[0] - b[0]) <= 1e-9 * abs(a[0]), (lik, a[0], b[0])
        np.testing.assert_allclose(b[1], a[1], rtol=1e-7, atol=1e-7 * np.abs(a[1]).max())


@pytest.mark.parametrize("seg_form,tail_order", [("wave", "row"), ("block", "row"), ("wave", "level")])
def test_segment_and_tail_forms_agree(monkeypatch, seg_form, tail_order):
    """The LDS segment solved by the 1024-thread barrier form (default) or by one wave per column
    (SegWave), and the merged tail launched in storage (Morton) order or in level order, against
    the plain level schedule: the same algebra in other summation orders (~1e-10 at a tight CG
    tolerance). The segment here holds long B^T rows (2 and 4 lanes per row in the wave form)."""
    from gpboost_amd import synthetic
    n = 8000
    X = synthetic.bench_coords(n)
    for lik in ("gaussian", "bernoulli_logit"):
        y = synthetic.bench_gaussian_y(n) if lik == "gaussian" else synthetic.bench_bernoulli_y(X)
        case = dict(likelihood=lik, cov_fct="exponential", shape=0.5, num_neighbors=30, aux=0.1)
        out = {}
        for key, (k0, k, g, form, order) in {"levels": ("0", "0", "1", "wave", "row"),
                                             "plan": ("256", "6000", "4", seg_form, tail_order)}.items():
            monkeypatch.setenv("GPBOOST_AMD_DENSE_ROWS", k0)
            monkeypatch.setenv("GPBOOST_AMD_HEAD_ROWS", k)
            monkeypatch.setenv("GPBOOST_AMD_TAIL_MERGE", g)
            monkeypatch.setenv("GPBOOST_AMD_SEG_FORM", form)
            monkeypatch.setenv("GPBOOST_AMD_TAIL_ORDER", order)
            gm = _model(X, case, t=12, dc=1e-9)
            out[key] = gm.neg_log_likelihood_and_grad([1.0, 0.1], y)
        a, b = out["levels"], out["plan"]
        assert abs(a[0] - b[0]) <= 1e-9 * abs(a[0]), (lik, a[0], b[0])
        np.testing.assert_allclose(b[1], a[1], rtol=1e-7, atol=1e-7 * np.abs(a[1]).max())


@pytest.mark.parametrize("dense_rows,head_rows,merge,w", [("256", "6000", "4", "64"), ("0", "0", "1", "8"),
                                                           ("2048", "2048", "16", "3")])
def test_persistent_tail_agrees(monkeypatch, dense_rows, head_rows, merge, w):
    """The persistent tail solve (GPBOOST_AMD_TAIL_FORM=persist: all merged levels in one launch with
    grid barriers, values through a padded copy) against the plain level schedule at a tight CG
    tolerance (same algebra, other summation order: ~1e-10), and bit for bit repeatable (fixed entry
    order per row). Covers a tail after dense + segment heads, a tail without heads at g = 1 (many
    barriers, head rows of the lower solve read from the caller's buffer) and few workgroups per XCD
    group (rows looped per wave)."""
    from gpboost_amd import synthetic
    n = 8000
    X = synthetic.bench_coords(n)
    for lik in ("gaussian", "bernoulli_logit"):
        y = synthetic.bench_gaussian_y(n) if lik == "gaussian" else synthetic.bench_bernoulli_y(X)
        case = dict(likelihood=lik, cov_fct="exponential", shape=0.5, num_neighbors=30, aux=0.1)
        out = {}
        for key, (k0, k, g, form) in {"levels": ("0", "0", "1", "launch"),
                                      "persist": (dense_rows, head_rows, merge, "persist"),
                                      "again": (dense_rows, head_rows, merge, "persist")}.items():
            monkeypatch.setenv("GPBOOST_AMD_DENSE_ROWS", k0)
            monkeypatch.setenv("GPBOOST_AMD_HEAD_ROWS", k)
            monkeypatch.setenv("GPBOOST_AMD_TAIL_MERGE", g)
            monkeypatch.setenv("GPBOOST_AMD_TAIL_FORM", form)
            monkeypatch.setenv("GPBOOST_AMD_TAIL_W", w)
            gm = _model(X, case, t=12, dc=1e-9)
            out[key] = gm.neg_log_likelihood_and_grad([1.0, 0.1], y)
        a, b = out["levels"], out["persist"]
        assert np.isfinite(b[0]) and np.all(np.isfinite(b[1]))
        assert abs(a[0] - b[0]) <= 1e-9 * abs(a[0]), (lik, a[0], b[0])
        np.testing.assert_allclose(b[1], a[1], rtol=1e-7, atol=1e-7 * np.abs(a[1]).max())
        assert out["again"][0] == b[0]
        np.testing.assert_array_equal(out["again"][1], b[1])


def test_graph_replay_matches_eager(monkeypatch):
    """VaduPrecond replays one captured hipGraph per buffer set (vadu_precond.cpp Apply). Replays after
    captures at other widths (bench_latent_operators at t = 51 and t = 1 on the model's scratch block),
    after new parameters (refreshed factor and preconditioner values through the same captured
    pointers) and in a second model created after the first one is freed (allocations at reused
    addresses) must give bit for bit the results of eager launches (GPBOOST_AMD_NO_GRAPH=1)."""
    from gpboost_amd import synthetic
    n = 8000
    X = synthetic.bench_coords(n)
    y = synthetic.bench_gaussian_y(n)
    case = dict(likelihood="gaussian", cov_fct="exponential", shape=0.5, num_neighbors=30, aux=0.1)

    def sequence():
        res = []
        gm = _model(X, case, t=12, dc=1e-9)
        res.append(gm.neg_log_likelihood_and_grad([1.0, 0.1], y))
        gm.bench_latent_operators(51, 2)
        gm.bench_latent_operators(1, 2)
        res.append(gm.neg_log_likelihood_and_grad([0.8, 0.15], y))
        res.append(gm.neg_log_likelihood_and_grad([1.0, 0.1], y))
        del gm
        gm2 = _model(X, case, t=12, dc=1e-9)
        res.append(gm2.neg_log_likelihood_and_grad([1.0, 0.1], y))
        return res

    monkeypatch.delenv("GPBOOST_AMD_NO_GRAPH", raising=False)
    graph = sequence()
    monkeypatch.setenv("GPBOOST_AMD_NO_GRAPH", "1")
    eager = sequence()
    for g, e in zip(graph, eager):
        assert g[0] == e[0]
        np.testing.assert_array_equal(g[1], e[1])
    assert graph[0][0] == graph[2][0] == graph[3][0]


def test_latent_zero_response(monkeypatch):
    """y == 0 under the Gaussian latent model: the Newton right-hand side y / aux is zero, so its
    CG column (fused with the probes) must stop at u = 0 without iterating (CG_utils.cpp:42-45)
    instead of dividing 0 by 0; checked against the oracle."""
    from gpboost_amd import synthetic
    n = 3000
    X = synthetic.bench_coords(n)
    y = np.zeros(n)
    case = dict(likelihood="gaussian", cov_fct="exponential", shape=0.5, num_neighbors=20, aux=0.3)
    for k0 in ("0", "2048"):
        monkeypatch.setenv("GPBOOST_AMD_DENSE_ROWS", k0)
        gm = _model(X, case, t=10, dc=1e-8)
        nll, g, _ = gm.neg_log_likelihood_and_grad([0.8, 0.15], y)
        perm, xv, nb = O.vecchia_setup(X, 20, 0, True)
        ref = O.latent_iterative(xv, y[perm], nb, 0, O.transform_latent(0, [0.8, 0.15]), "gaussian", 0.3, t=10,
                                 cg_delta_conv=1e-8)
        assert np.isfinite(nll) and np.all(np.isfinite(g))
        _check(nll, g, ref["nll"], ref["grad"])


def test_latent_many_neighbours_vs_oracle():
    """m = 40 > 32: the t = 1 operator's generic (one row per lane group) form and head rows
    wider than one lane slot, against the oracle at a tight CG tolerance."""
    from gpboost_amd import synthetic
    n, m = 3000, 40
    X = synthetic.bench_coords(n)
    y = synthetic.bench_bernoulli_y(X)
    case = dict(likelihood="bernoulli_logit", cov_fct="exponential", shape=0.5, num_neighbors=m, aux=0.1)
    gm = _model(X, case, t=10, dc=1e-8)
    nll, g, _ = gm.neg_log_likelihood_and_grad([1.0, 0.1], y)
    perm, xv, nb = O.vecchia_setup(X, m, 0, True)
    ref = O.latent_iterative(xv, y[perm], nb, 0, O.transform_latent(0, [1.0, 0.1]), "bernoulli_logit", 0.1, t=10,
                             cg_delta_conv=1e-8)
    _check(nll, g, ref["nll"], ref["grad"])


def test_two_live_models_different_head_sizes(monkeypatch):
    """Two models alive in one process with different head sizes (the kernel's dynamic-LDS limit
    is per function, so the second model must not lower it under the first)."""
    from gpboost_amd import synthetic
    case = dict(likelihood="gaussian", cov_fct="exponential", shape=0.5, num_neighbors=20, aux=0.1)
    X = synthetic.bench_coords(9000)
    y = synthetic.bench_gaussian_y(9000)
    monkeypatch.setenv("GPBOOST_AMD_DENSE_ROWS", "0")
    monkeypatch.setenv("GPBOOST_AMD_HEAD_ROWS", "8000")
    a = _model(X, case, t=8, dc=1e-8)
    ra = a.neg_log_likelihood_and_grad([1.0, 0.1], y)
    monkeypatch.setenv("GPBOOST_AMD_HEAD_ROWS", "50")
    b = _model(X, case, t=8, dc=1e-8)
    rb = b.neg_log_likelihood_and_grad([1.0, 0.1], y)
    ra2 = a.neg_log_likelihood_and_grad([1.0, 0.1], None)   # the large-head model again
    assert ra2[0] == ra[0] and np.array_equal(ra2[1], ra[1])
    assert abs(rb[0] - ra[0]) <= 1e-8 * abs(ra[0])


def test_baseline_size_matches_reference():
    """BASELINE config 3 at its full size (n = 100k, m = 30, t = 50, cg_delta_conv = 1e-2, VADU) against
    the reference run here (tests/golden/make_golden_100k.py): the stochastic estimates use the
    same probe streams and stopping rules, so they agree to the 1e-6 north-star tolerance (observed
    ~1e-15 nll, ~1e-9 gradient)."""
    import json
    import os

    from gpboost_amd import synthetic
    with open(os.path.join(os.path.dirname(__file__), "golden", "golden_100k.json")) as f:
        case = json.load(f)["latent"]
    n = case["n"]
    X = synthetic.bench_coords(n)
    y = synthetic.bench_gaussian_y(n)
    gm = _model(X, dict(likelihood="gaussian", cov_fct="exponential", shape=0.5, num_neighbors=30, aux=case["aux"]),
                t=case["num_rand_vec_trace"], seed=1, dc=case["cg_delta_conv"])
    nll, g, _ = gm.neg_log_likelihood_and_grad(case["cov_pars"], y)
    _check(nll, g, case["nll"], case["grad"])


def _golden100k():
    import json
    import os
    with open(os.path.join(os.path.dirname(__file__), "golden", "golden_100k.json")) as f:
        return json.load(f)


def test_baseline_size_bernoulli_tight_matches_reference():
    """BASELINE config 5 (bernoulli_logit, Laplace + PCG / SLQ, n = 100k, m = 30) with the mode-finding
    and SLQ solves converged to cg_delta_conv = 1e-8, against the reference at the same setting
    (tests/golden/make_golden_100k_tight.py): nll and gradient at the 1e-6 north-star tolerance."""
    from gpboost_amd import synthetic
    case = _golden100k()["bernoulli_tight"]
    X = synthetic.bench_coords(case["n"])
    y = synthetic.bench_bernoulli_y(X)
    gm = _model(X, dict(likelihood="bernoulli_logit", cov_fct="exponential", shape=0.5, num_neighbors=30),
                t=case["num_rand_vec_trace"], seed=1, dc=case["cg_delta_conv"])
    nll, g, _ = gm.neg_log_likelihood_and_grad(case["cov_pars"], y)
    _check(nll, g, case["nll"], case["grad"])


def test_baseline_size_bernoulli_default_within_reference_sensitivity():
    """Config 5 at the default cg_delta_conv = 1e-2. nll at 1e-6. The gradient at this tolerance is
    rounding-limited, which the REFERENCE itself shows (tests/golden/make_golden_100k_sens.py): its
    thread-count spread is zero, but moving the covariance parameters by 1e-14 relative (a few ulps)
    moves its own gradient by up to ~1e-5 relative, because the six Newton solves stop on an absolute
    residual of 1e-2 and their iteration counts flip. The bound is twice the reference's own largest
    ulp-perturbation deviation per component, read from the fixture (no value of this implementation
    enters it)."""
    from gpboost_amd import synthetic
    gold = _golden100k()
    case, sens = gold["bernoulli"], gold["bernoulli_sensitivity"]
    ref_g = np.asarray(case["grad"])
    spread = np.max([np.abs(np.asarray(r["grad"]) - ref_g) for r in sens["runs"]], axis=0)
    assert np.all(spread > 0) and np.all(spread < 1e-4 * np.abs(ref_g))   # the fixture's own statement
    X = synthetic.bench_coords(case["n"])
    y = synthetic.bench_bernoulli_y(X)
    gm = _model(X, dict(likelihood="bernoulli_logit", cov_fct="exponential", shape=0.5, num_neighbors=30),
                t=case["num_rand_vec_trace"], seed=1, dc=case["cg_delta_conv"])
    nll, g, _ = gm.neg_log_likelihood_and_grad(case["cov_pars"], y)
    assert abs(nll - case["nll"]) <= 1e-6 * abs(case["nll"]), (nll, case["nll"])
    assert np.all(np.abs(g - ref_g) <= 2 * spread), (g, ref_g, spread)
