"""Cross-rank persistent sweep (otf_sinkhorn_xsweep, otfuse.distributed.sinkhorn_xsweep):
one problem's rows over the ranks, the column sums exchanged inside the launch through
the peers' exchange buffers (needs an MI355X).

The 8-GPU runs belong to the driver: here two processes share cuda:0, each running a
capped persistent grid (OTF_SWEEP_GRID) so both are resident at once, and exchange IPC
handles over gloo.  The assembled rows are compared with the float64 oracle on the whole
problem (POT's sinkhorn_knopp restated, MRI_PET_OT_nojax.py:143), including the early
stop that every rank must take at the same check.
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


def _problem():
    rng = np.random.default_rng(3)
    rows = [700, 1301]
    n, m = sum(rows), 900
    C = rng.random((n, m))
    a = np.full(n, 1.0 / n)
    b = rng.random(m) + 0.5
    b /= b.sum()
    return rows, C, a, b


def test_xsweep_single_rank_vs_oracle(orc, dev):
    """world = 1: the exchange degenerates to the granule-flush sweep engine."""
    import otfuse.distributed as D
    rows, C, a, b = _problem()
    xp = D.XPeer(C.shape[1])
    try:
        res = D.sinkhorn_xsweep(torch.tensor(a, device=dev), torch.tensor(b, device=dev),
                                torch.tensor(C, device=dev, dtype=torch.float32), 0.05, xp,
                                n_total=C.shape[0], max_iter=400, stop_thr=1e-6)
        info = res.info()
        P_ref, _, _, info_r = orc.sinkhorn_knopp(a, b, C, 0.05, 400, 1e-6)
        assert info["niter"] == info_r["niter"] and info["engine_name"] == "sweep"
        P = res.plan.cpu().numpy()
        assert np.abs(P - P_ref).max() / np.abs(P_ref).max() < 1e-4
        # a second solve on the same exchange (epochs continue) gives the same bits
        res2 = D.sinkhorn_xsweep(torch.tensor(a, device=dev), torch.tensor(b, device=dev),
                                 torch.tensor(C, device=dev, dtype=torch.float32), 0.05, xp,
                                 n_total=C.shape[0], max_iter=400, stop_thr=1e-6)
        assert torch.equal(res2.plan, res.plan)
    finally:
        xp.close()


def _worker(rank, world, port, out_dir):
    import sys
    for p in (PKG, REPO):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ["OTF_SWEEP_GRID"] = "96"      # two ranks' grids resident on one device
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import otfuse.distributed as D
    from otfuse.synthetic import paired_embeddings
    dev = torch.device("cuda", 0)
    rows, C, a, b = _problem()
    r0 = sum(rows[:rank])
    sl = slice(r0, r0 + rows[rank])
    xp = D.XPeer(C.shape[1])
    res = D.sinkhorn_xsweep(torch.tensor(a[sl], device=dev), torch.tensor(b, device=dev),
                            torch.tensor(C[sl], device=dev, dtype=torch.float32), 0.05, xp,
                            n_total=C.shape[0], max_iter=400, stop_thr=1e-6)
    info = res.info()
    np.savez(os.path.join(out_dir, f"r{rank}.npz"), P=res.plan.cpu().numpy(), sl=[sl.start, sl.stop],
             niter=info["niter"], status=info["status"], err=np.array(info["err"]),
             v=res.v.cpu().numpy())
    xp.close()
    # the per-epoch pipeline on the exchange: fp16 cost rows vs all-gathered PET shards
    X, Y, _ = paired_embeddings(1536, 256, seed=11)
    half = 1536 // world
    xs = torch.tensor(X[rank * half:(rank + 1) * half], device=dev, dtype=torch.float16)
    ys = torch.tensor(Y[rank * half:(rank + 1) * half], device=dev, dtype=torch.float16)
    xp2 = D.XPeer(1536)
    res2, n_total = D.coupled_solve_sharded(xs, ys, 0.1, max_iter=60, xpeer=xp2)
    assert n_total == 1536 and res2.info()["status_name"] == "max_iter"
    np.save(os.path.join(out_dir, f"c{rank}.npy"), res2.plan.cpu().numpy())
    from otfuse import ops
    C16, _, unit = ops.pairwise_cost_ex(xs, D.all_gather_rows(ys), zero_diag=False,
                                        out_dtype=torch.float16)
    np.save(os.path.join(out_dir, f"k{rank}.npy"),
            C16.float().cpu().numpy().astype(np.float64) * float(unit))
    xp2.close()
    dist.barrier()
    dist.destroy_process_group()


def test_xsweep_two_ranks_match_whole_problem(tmp_path, orc):
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    rows, C, a, b = _problem()
    P_ref, _, v_ref, info_r = orc.sinkhorn_knopp(a, b, C, 0.05, 400, 1e-6)
    P = np.zeros_like(P_ref)
    vs = []
    for r in range(world):
        z = np.load(tmp_path / f"r{r}.npz")
        s0, s1 = z["sl"]
        P[s0:s1] = z["P"]
        assert int(z["niter"]) == info_r["niter"]
        np.testing.assert_allclose(z["err"], info_r["err"], rtol=1e-4, atol=1e-8)
        vs.append(z["v"])
    assert np.array_equal(vs[0], vs[1])      # every rank derives the same S, bit for bit
    assert np.abs(P - P_ref).max() / np.abs(P_ref).max() < 1e-4
    Pc = np.concatenate([np.load(tmp_path / f"c{r}.npy") for r in range(world)])
    Cd = np.concatenate([np.load(tmp_path / f"k{r}.npy") for r in range(world)])
    u = np.full(1536, 1.0 / 1536)
    Pr, *_ = orc.sinkhorn_knopp(u, u, Cd / Cd.max(), 0.1, 60, 0.0)
    assert np.abs(Pc - Pr).max() / np.abs(Pr).max() < 1e-4
