"""CPU, world_size 2 (gloo): the N>1 Vecchia path's host logic.

The GPU path shards Vecchia rows into contiguous blocks (GPB_PartitionRows), each rank
reduces its rows to six partial sums, one all-reduce (RCCL on the GPU box) combines them,
and GPB_CombinePartials assembles nll + gradient. Here each rank computes its block's
partials with the oracle, the all-reduce runs over gloo, and the assembled result must
equal the single-rank result. (The device kernel's row-range arguments are exercised by
the GPU tests; RCCL itself needs >= 2 GPUs and runs in the driver's scaling bench.)"""
import os
import socket

import numpy as np
import pytest


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, profile, out_q):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist
    from gpboost_amd import combine_partials, partition_rows, synthetic
    from oracle import oracle as O
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n = 1500
    X = synthetic.bench_coords(n)
    Y = synthetic.bench_gaussian_y(n)
    perm, xv, nb = O.vecchia_setup(X, 20, 0, True)
    tp = O.transform(0, [0.2, 1.1, 0.12])
    r0, r1 = partition_rows(n, world, rank)
    part = torch.tensor(O.vecchia_partials(xv, Y[perm], nb, 0, tp, r0, r1), dtype=torch.float64)
    dist.all_reduce(part, op=dist.ReduceOp.SUM)
    nll, g, s2 = combine_partials(part.numpy(), n, tp[0], profile)
    if rank == 0:
        ref = O.vecchia_nll_grad(xv, Y[perm], nb, 0, tp, int(profile))
        out_q.put((nll, g.tolist(), ref["nll"], ref["grad"].tolist()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("profile", [False, True])
def test_two_rank_gloo_matches_single_rank(profile):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, profile, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
        assert p.exitcode == 0
    nll, g, ref_nll, ref_g = q.get(timeout=10)
    assert abs(nll - ref_nll) <= 1e-12 * abs(ref_nll)
    np.testing.assert_allclose(g, ref_g, rtol=1e-11)
