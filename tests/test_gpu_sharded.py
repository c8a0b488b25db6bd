"""GPU: the sharded paths of SURVEY.md §8e through the C ABI.

* Latent Vecchia (iterative): probe columns sharded over ranks (GPB_SetDistributed /
  GPB_SetDistributedHostReduce). Every rank runs its share of the SLQ probes (padded to equal
  block widths), the Newton / mode columns replicated; the block stopping rule's norm sum is
  all-reduced every PCG iteration, the per-probe log-determinant and trace terms and the
  mode-derivative row moments at the end. The result must match the reference fixtures
  (tests/golden/golden_latent.json, the reference run with the same probe streams) exactly
  as the single-GPU path does, and every rank must return the same numbers.
* Exact Vecchia: rows sharded, six partial sums all-reduced.

Several ranks cannot share one GPU under RCCL, so the multi-rank cases run two processes on
the box's one GPU with the host-reduce transport (a gloo all-reduce behind a callback); the
RCCL code path itself is exercised by a one-rank communicator, which must reproduce the
plain single-GPU evaluation bit for bit.
"""
import os
import socket
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
RTOL = 1e-6


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _latent_model(X, case):
    from gpboost_amd import GPModel
    lik = case["likelihood"]
    gm = GPModel(gp_coords=X, likelihood=lik, cov_function=case["cov_fct"], cov_fct_shape=case.get("shape", 0.5),
                 gp_approx="vecchia_latent" if lik == "gaussian" else "vecchia",
                 num_neighbors=case["num_neighbors"], vecchia_ordering="random",
                 matrix_inversion_method="iterative", seed=0)
    params = dict(num_rand_vec_trace=case["num_rand_vec_trace"], seed_rand_vec_trace=case["seed_rand_vec_trace"],
                  cg_delta_conv=case["cg_delta_conv"])
    if lik == "gaussian":
        params["init_aux_pars"] = [case["aux"]]
    gm.set_optim_params(params)
    return gm


def _exact_model(X):
    from gpboost_amd import GPModel
    return GPModel(gp_coords=X, cov_function="exponential", gp_approx="vecchia", num_neighbors=20,
                   vecchia_ordering="random", seed=0)


EXACT_THETA = [0.2, 1.1, 0.12]


def _worker(rank, world, port, kind, case, out_q):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, HERE)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist
    from gpboost_amd import synthetic
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        def allreduce(a):
            t = torch.from_numpy(a)   # shares the library's host buffer
            dist.all_reduce(t, op=dist.ReduceOp.SUM)

        if kind == "latent":
            from conftest import latent_case_data
            X, y = latent_case_data(case)
            gm = _latent_model(X, case)
            gm.set_distributed_host(rank, world, allreduce)
            nll = gm.neg_log_likelihood(case["cov_pars"], y)
            nll2, g, _ = gm.neg_log_likelihood_and_grad(case["cov_pars"], None)
            out_q.put((rank, nll, nll2, np.asarray(g).tolist(), gm.last_iteration_info().tolist()))
        else:
            n = 3000
            X = synthetic.bench_coords(n)
            y = synthetic.bench_gaussian_y(n)
            gm = _exact_model(X)
            gm.set_distributed_host(rank, world, allreduce)
            nll, g, s2 = gm.neg_log_likelihood_and_grad(EXACT_THETA, y, profile_sigma2=True)
            out_q.put((rank, nll, nll, np.asarray(g).tolist(), [s2]))
        dist.barrier()
    finally:
        dist.destroy_process_group()


def _run_ranks(world, kind, case=None):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, kind, case, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r = q.get(timeout=240)
        res[r[0]] = r[1:]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0, p.exitcode
    return res


@pytest.mark.parametrize("name", ["gauss_m30_exp_tight", "gauss_m20_matern15_t20", "bern_m30_exp_tight",
                                  "bern_m16_matern25"])
def test_latent_probe_shards_match_reference(golden_latent, name):
    case = golden_latent[name]
    res = _run_ranks(2, "latent", case)
    nll0, nll2_0, g0, info0 = res[0]
    for r in (1,):
        nll, nll2, g, info = res[r]
        assert nll == nll0 and nll2 == nll2_0, (nll, nll0)   # all-reduced terms: identical on every rank
        np.testing.assert_array_equal(g, g0)
        assert info[2] == info0[2]                           # same Lanczos length (global stopping rule)
    assert abs(nll0 - case["nll"]) <= RTOL * abs(case["nll"]), (nll0, case["nll"])
    ref_g = np.asarray(case["grad"])
    np.testing.assert_allclose(g0, ref_g, rtol=RTOL, atol=RTOL * np.abs(ref_g).max())


def test_latent_probe_shards_three_ranks_uneven(golden_latent):
    # 50 probes over 3 ranks: 16 / 17 / 17 columns, padded to 17 on every rank
    case = golden_latent["gauss_m30_exp_tight"]
    res = _run_ranks(3, "latent", case)
    for r in (1, 2):
        assert res[r][0] == res[0][0]
        np.testing.assert_array_equal(res[r][2], res[0][2])
    assert abs(res[0][0] - case["nll"]) <= RTOL * abs(case["nll"])


@pytest.mark.parametrize("name", ["gauss_m30_exp_default", "bern_m30_exp_default"])
def test_latent_rccl_one_rank_bitwise(golden_latent, name):
    from conftest import latent_case_data
    from gpboost_amd import comm_create_id
    case = golden_latent[name]
    X, y = latent_case_data(case)
    plain = _latent_model(X, case)
    n0 = plain.neg_log_likelihood(case["cov_pars"], y)
    _, g0, _ = plain.neg_log_likelihood_and_grad(case["cov_pars"], None)
    gm = _latent_model(X, case)
    gm.set_distributed(0, 1, comm_create_id())
    n1 = gm.neg_log_likelihood(case["cov_pars"], y)
    _, g1, _ = gm.neg_log_likelihood_and_grad(case["cov_pars"], None)
    assert n1 == n0
    np.testing.assert_array_equal(g1, g0)


def test_exact_row_shards_host_reduce():
    from gpboost_amd import synthetic
    res = _run_ranks(2, "exact")
    n = 3000
    gm = _exact_model(synthetic.bench_coords(n))
    nll, g, s2 = gm.neg_log_likelihood_and_grad(EXACT_THETA, synthetic.bench_gaussian_y(n), profile_sigma2=True)
    for r in (0, 1):
        assert abs(res[r][0] - nll) <= 1e-10 * abs(nll)
        np.testing.assert_allclose(res[r][2], g, rtol=1e-10)


def test_latent_shards_need_a_probe_each():
    from conftest import latent_case_data
    import json
    with open(os.path.join(HERE, "golden", "golden_latent.json")) as f:
        case = dict(json.load(f)["gauss_m30_exp_default"])
    case["num_rand_vec_trace"] = 1
    X, y = latent_case_data(case)
    gm = _latent_model(X, case)
    gm.set_distributed_host(0, 2, lambda a: None)
    from gpboost_amd import GPBoostError
    with pytest.raises(GPBoostError, match="at least one probe column"):
        gm.neg_log_likelihood(case["cov_pars"], y)


def test_host_reduce_callback_error_is_raised():
    """An exception inside the host all-reduce callback is not swallowed by ctypes: the buffer is
    poisoned (NaN) so the library stops, and the Python call re-raises the callback's error."""
    from gpboost_amd import GPBoostError, GPModel, synthetic
    X = synthetic.bench_coords(1000)
    Y = synthetic.bench_gaussian_y(1000)
    gm = GPModel(gp_coords=X, cov_function="exponential", gp_approx="vecchia", num_neighbors=10)

    def bad(_a):
        raise RuntimeError("transport down")
    gm.set_distributed_host(0, 1, bad)
    with pytest.raises(GPBoostError, match="transport down"):
        gm.neg_log_likelihood_and_grad([0.1, 1.0, 0.1], Y)
