"""RCCL communicator (otf_comm_*) and the one-call row-sharded solve on one GPU.

A single-rank communicator exercises the whole C path (unique id, init, the RCCL
collectives enqueued on the torch stream, otf_sinkhorn_row_sharded's pass + all-reduce
loop); the multi-rank protocol itself is covered by the gloo tests
(tests/test_distributed_cpu.py, tests/test_gpu_sharded.py) and runs on RCCL in the
driver's multi-GPU bench.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def comm(dev):
    from otfuse.comm import Communicator
    c = Communicator(device=dev)
    yield c
    c.close()


def test_single_rank_collectives(comm, dev):
    assert comm.nranks == 1 and comm.rank == 0
    x = torch.arange(1000, dtype=torch.float32, device=dev)
    ref = x.clone()
    comm.all_reduce(x, "sum")
    comm.all_reduce(x, "max")
    assert torch.equal(x, ref)
    y = torch.randn(7, 5, dtype=torch.float64, device=dev)
    assert torch.equal(comm.all_gather(y), y)
    h = torch.randn(33, dtype=torch.float16, device=dev)
    assert torch.equal(comm.all_gather(h), h)


@pytest.mark.parametrize("dt", [torch.float32, torch.float64])
def test_row_sharded_one_call_equals_whole_solve(comm, orc, dev, dt):
    from otfuse import ops
    from otfuse.distributed import sinkhorn_row_sharded
    rng = np.random.default_rng(3)
    n, m = 700, 450
    C = rng.random((n, m))
    a = np.full(n, 1.0 / n)
    b = np.full(m, 1.0 / m)
    Ct = torch.as_tensor(C, device=dev, dtype=dt)
    at = torch.as_tensor(a, device=dev, dtype=dt)
    bt = torch.as_tensor(b, device=dev, dtype=dt)
    whole = ops.sinkhorn(at, bt, Ct, 0.05, max_iter=120, stop_thr=0.0, engine="stream")
    same = 1e-5 if dt == torch.float32 else 1e-12   # float column-sum atomics: order varies
    for c in (comm, None):
        res = sinkhorn_row_sharded(at, bt, Ct, 0.05, max_iter=120, stop_thr=0.0, comm=c) \
            if c is not None else sinkhorn_row_sharded(at, bt, Ct, 0.05, max_iter=120, stop_thr=0.0)
        d = (res.plan.double() - whole.plan.double()).abs().max() / whole.plan.double().abs().max()
        assert d.item() < same
        assert res.info()["niter"] == whole.info()["niter"]
    Pr, *_ = orc.sinkhorn_knopp(a, b, C, 0.05, 120, 0.0)
    tol = 1e-4 if dt == torch.float32 else 1e-10
    assert np.abs(res.plan.cpu().numpy() - Pr).max() / Pr.max() < tol


def test_coupled_solve_with_comm_config5_shape(comm, dev):
    """The config-5 per-epoch pipeline (all-gather, fp16 cost rows, max all-reduce,
    row-sharded solve) through the communicator at N = 2048 on one rank."""
    from otfuse import ops
    from otfuse.distributed import coupled_solve_sharded
    from otfuse.synthetic import paired_embeddings
    X, Y, _ = paired_embeddings(2048, 256, seed=11)
    Xd = torch.as_tensor(X.astype(np.float16), device=dev)
    Yd = torch.as_tensor(Y.astype(np.float16), device=dev)
    res, n_total = coupled_solve_sharded(Xd, Yd, 0.1, max_iter=50, comm=comm)
    assert n_total == 2048
    C, cmax, _ = ops.pairwise_cost_ex(Xd, Yd, out_dtype=torch.float16)
    a = torch.full((2048,), 1.0 / 2048, device=dev)
    ref = ops.sinkhorn(a, a, C, 0.1, max_iter=50, stop_thr=0.0, cost_scale=cmax)
    P, Pr = res.plan.double(), ref.plan.double()
    assert ((P - Pr).abs().max() / Pr.abs().max()).item() < 1e-5
