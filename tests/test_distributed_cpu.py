"""World-size-2 gloo tests of the collective logic in otfuse.distributed (CPU).

The per-rank feature-cost partial normally comes from the HIP kernel; on CPU the
test injects the oracle restatement as that partial so the test checks exactly
the distributed part: the shard decomposition M = sum_r M_r and the row gather.
"""
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import PKG, REPO


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, out_dir):
    import sys
    for p in (PKG, REPO):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import oracle as orc
    import otfuse.distributed as D

    def oracle_partial(X, Y, Ts=None, ts_diag=None, weights="pot"):
        T = np.diag(ts_diag.numpy()) if ts_diag is not None else Ts.numpy()
        return torch.from_numpy(orc.feature_cost(X.numpy(), Y.numpy(), T))

    D._local_feature_cost = oracle_partial
    rng = np.random.default_rng(100)
    B, d, d2 = 6, 9, 7
    X = rng.random((B * world, d)).astype(np.float32)
    Y = rng.random((B * world, d2)).astype(np.float32)
    sl = slice(rank * B, (rank + 1) * B)
    ts = torch.full((B,), 1.0 / (B * world), dtype=torch.float64)
    M = D.sharded_feature_cost(torch.from_numpy(X[sl]), torch.from_numpy(Y[sl]), ts_diag_local=ts)
    ref = orc.feature_cost(X, Y, np.eye(B * world) / (B * world))
    np.testing.assert_allclose(M.numpy(), ref, rtol=1e-12, atol=1e-12)

    # ragged all-gather: rank r contributes r + 2 rows
    local = torch.arange((rank + 2) * 3, dtype=torch.float32).reshape(rank + 2, 3) + 100 * rank
    g = D.all_gather_rows(local)
    expect = torch.cat([torch.arange((r + 2) * 3, dtype=torch.float32).reshape(r + 2, 3) + 100 * r
                        for r in range(world)])
    assert torch.equal(g, expect)
    lab = torch.tensor([rank] * (rank + 1), dtype=torch.int64)
    mri, pet, labels = D.gather_epoch_features(local, local * 2, lab)
    assert labels.tolist() == sum([[r] * (r + 1) for r in range(world)], [])
    assert torch.equal(pet, 2 * expect)
    open(os.path.join(out_dir, f"ok{rank}"), "w").write("ok")
    dist.barrier()
    dist.destroy_process_group()


def test_sharded_feature_cost_and_gather_world2(tmp_path):
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    assert all((tmp_path / f"ok{r}").exists() for r in range(world))
