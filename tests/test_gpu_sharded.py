"""Row-sharded coupled Sinkhorn on the device (needs an MI355X).

Two processes share cuda:0 (the 8-GPU runs belong to the driver); they exchange
over gloo, which handles device tensors, so the test exercises exactly the
product path — otf_sinkhorn_pass / otf_sinkhorn_finish on each rank's rows and
one all-reduce of the column sums per iteration — and compares the assembled
rows with the float64 oracle on the whole problem.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import PKG, REPO

pytestmark = pytest.mark.gpu


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
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import otfuse.distributed as D
    from otfuse.synthetic import paired_embeddings
    dev = torch.device("cuda", 0)

    # (1) fp32 cost rows, ragged shards, early stop decided identically on both ranks
    rng = np.random.default_rng(3)
    rows = [700, 1301]
    n, m = sum(rows), 900
    C = rng.random((n, m))
    a = np.full(n, 1.0 / n)
    b = rng.random(m) + 0.5
    b /= b.sum()
    r0 = sum(rows[:rank])
    sl = slice(r0, r0 + rows[rank])
    res = D.sinkhorn_row_sharded(torch.tensor(a[sl], device=dev), torch.tensor(b, device=dev),
                                 torch.tensor(C[sl], device=dev, dtype=torch.float32), 0.05,
                                 max_iter=400, stop_thr=1e-6, sync_every=20)
    info = res.info()
    np.savez(os.path.join(out_dir, f"r{rank}.npz"), P=res.plan.cpu().numpy(), sl=[sl.start, sl.stop],
             niter=info["niter"], status=info["status"], err=np.array(info["err"]))

    # (2) the per-epoch pipeline: all-gather PET shards, fp16 cost rows, global max
    X, Y, _ = paired_embeddings(1536, 256, seed=11)
    half = 1536 // world
    xs = torch.tensor(X[rank * half:(rank + 1) * half], device=dev, dtype=torch.float16)
    ys = torch.tensor(Y[rank * half:(rank + 1) * half], device=dev, dtype=torch.float16)
    res2, n_total = D.coupled_solve_sharded(xs, ys, 0.1, max_iter=60)
    assert n_total == 1536
    np.save(os.path.join(out_dir, f"c{rank}.npy"), res2.plan.cpu().numpy())
    # the cost rows that solve consumed (same deterministic kernels): stored fp16 x unit
    from otfuse import ops
    C16, _, unit = ops.pairwise_cost_ex(xs, D.all_gather_rows(ys), zero_diag=False,
                                        out_dtype=torch.float16)
    np.save(os.path.join(out_dir, f"k{rank}.npy"),
            C16.float().cpu().numpy().astype(np.float64) * float(unit))
    dist.barrier()
    dist.destroy_process_group()


def test_row_sharded_solve_matches_whole_problem(tmp_path, orc):
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    rng = np.random.default_rng(3)
    n, m = 2001, 900
    C = rng.random((n, m))
    a = np.full(n, 1.0 / n)
    b = rng.random(m) + 0.5
    b /= b.sum()
    P_ref, _, _, info_r = orc.sinkhorn_knopp(a, b, C, 0.05, 400, 1e-6)
    P = np.zeros_like(P_ref)
    for r in range(world):
        z = np.load(tmp_path / f"r{r}.npz")
        s0, s1 = z["sl"]
        P[s0:s1] = z["P"]
        assert int(z["niter"]) == info_r["niter"]
        # fp32 arithmetic: the error bottoms out near 1e-8 where fp64 reaches 1e-18
        np.testing.assert_allclose(z["err"], info_r["err"], rtol=1e-4, atol=1e-8)
    assert np.abs(P - P_ref).max() / np.abs(P_ref).max() < 1e-4

    # pipeline: the assembled plan equals the whole-problem POT solve on the cost the
    # ranks consumed (fp16-stored rows x their power-of-two units; "max_cost" = the
    # max over both ranks)
    Pc = np.concatenate([np.load(tmp_path / f"c{r}.npy") for r in range(world)])
    Cd = np.concatenate([np.load(tmp_path / f"k{r}.npy") for r in range(world)])
    u = np.full(1536, 1.0 / 1536)
    Pr, *_ = orc.sinkhorn_knopp(u, u, Cd / Cd.max(), 0.1, 60, 0.0)
    assert np.abs(Pc - Pr).max() / np.abs(Pr).max() < 1e-4
    np.testing.assert_allclose(Pc.sum(1), 1.0 / 1536, rtol=1e-4)
