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


def test_xsweep_single_rank_mesh_is_the_mesh(dev):
    """world = 1 on a shape the mesh takes (whole 512-column tiles): the cross-rank call
    runs the register-resident mesh, bit for bit the single-GPU mesh solve."""
    import otfuse.distributed as D
    from otfuse import ops
    g = torch.Generator(device=dev).manual_seed(9)
    C = torch.rand(1024, 2048, device=dev, generator=g)
    a = torch.full((1024,), 1.0 / 1024, device=dev)
    b = torch.full((2048,), 1.0 / 2048, device=dev)
    xp = D.XPeer(2048)
    try:
        rx = D.sinkhorn_xsweep(a, b, C, 0.05, xp, n_total=1024, max_iter=80, stop_thr=0.0)
        rm = ops.sinkhorn(a, b, C, 0.05, max_iter=80, stop_thr=0.0, engine="mesh")
        assert rx.info()["engine_name"] == rm.info()["engine_name"] == "mesh"
        assert torch.equal(rx.plan, rm.plan) and torch.equal(rx.v, rm.v)
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


def _xmesh_worker(rank, world, port, out_dir):
    import sys
    for p in (PKG, REPO):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import otfuse.distributed as D
    from otfuse import ops
    from otfuse.synthetic import paired_embeddings
    dev = torch.device("cuda", 0)
    # (1) the metric shape's rows over two ranks: 2048 x 4096 float32 cost rows each
    # (16 x 8 register tiles per rank, one device holding both grids)
    N = 4096
    Cn = np.random.default_rng(5).random((N, N)).astype(np.float32)
    sl = slice(rank * N // world, (rank + 1) * N // world)
    a = torch.full((N // world,), 1.0 / N, device=dev)
    b = torch.full((N,), 1.0 / N, device=dev)
    xp = D.XPeer(N)
    res = D.sinkhorn_xsweep(a, b, torch.tensor(Cn[sl], device=dev), 0.05, xp, n_total=N,
                            max_iter=200, stop_thr=1e-7, engine="mesh")
    info = res.info()
    np.savez(os.path.join(out_dir, f"m{rank}.npz"), P=res.plan.cpu().numpy(), niter=info["niter"],
             err=np.array(info["err"]), v=res.v.cpu().numpy(), engine=info["engine_name"])
    # a second solve on the same exchange (the other slot set, epochs continue): same bits
    res2 = D.sinkhorn_xsweep(a, b, torch.tensor(Cn[sl], device=dev), 0.05, xp, n_total=N,
                             max_iter=200, stop_thr=1e-7, engine="mesh")
    assert torch.equal(res2.plan, res.plan)
    xp.close()
    # (2) BASELINE config 5's layout per rank at 8 ranks: 1024 fp16 cost rows x 8192 columns
    # (16 column tiles: two row-hop members per lane, blockIdx roles), via the per-epoch
    # pipeline (all-gathered PET shards, the max agreed over the ranks)
    X, Y, _ = paired_embeddings(8192, 128, seed=21)
    xs = torch.tensor(X[rank * 1024:(rank + 1) * 1024], device=dev, dtype=torch.float16)
    ys = torch.tensor(Y[rank * 4096:(rank + 1) * 4096], device=dev, dtype=torch.float16)
    xp2 = D.XPeer(8192)
    res3, n_total = D.coupled_solve_sharded(xs, ys, 0.1, max_iter=60, xpeer=xp2, engine="mesh")
    assert n_total == 2048 and res3.info()["engine_name"] == "mesh"
    np.save(os.path.join(out_dir, f"p{rank}.npy"), res3.plan.cpu().numpy())
    C16, _, unit = ops.pairwise_cost_ex(xs, D.all_gather_rows(ys), zero_diag=False,
                                        out_dtype=torch.float16)
    np.save(os.path.join(out_dir, f"q{rank}.npy"),
            C16.float().cpu().numpy().astype(np.float64) * float(unit))
    xp2.close()
    dist.barrier()
    dist.destroy_process_group()


def test_xmesh_two_ranks_match_whole_problem(tmp_path, orc):
    """The cross-rank mesh ("xmesh"): each rank's slab of K in its register files, the
    column-sum partials of the mesh's reducers exchanged over the peers' buffers inside
    the launch.  Two ranks on one device (N = 4096: 2048 x 4096 rows each; and config 5's
    per-rank layout at 8 ranks, 1024 x 8192 fp16 rows) against the whole-problem float64
    oracle: plans within 1e-4, the oracle's stop iteration and error log, and the same v
    bit for bit on both ranks."""
    world = 2
    mp.spawn(_xmesh_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    N = 4096
    Cn = np.random.default_rng(5).random((N, N)).astype(np.float32).astype(np.float64)
    u = np.full(N, 1.0 / N)
    P_ref, _, _, info_r = orc.sinkhorn_knopp(u, u, Cn, 0.05, 200, 1e-7)
    zs = [np.load(tmp_path / f"m{r}.npz") for r in range(world)]
    assert all(str(z["engine"]) == "mesh" for z in zs)
    assert all(int(z["niter"]) == info_r["niter"] for z in zs)
    for z in zs:
        np.testing.assert_allclose(z["err"], info_r["err"], rtol=1e-4, atol=1e-8)
    assert np.array_equal(zs[0]["v"], zs[1]["v"])
    P = np.concatenate([z["P"] for z in zs])
    assert np.abs(P - P_ref).max() / np.abs(P_ref).max() < 1e-4
    Pc = np.concatenate([np.load(tmp_path / f"p{r}.npy") for r in range(world)])
    Cd = np.concatenate([np.load(tmp_path / f"q{r}.npy") for r in range(world)])
    Pr, *_ = orc.sinkhorn_knopp(np.full(2048, 1.0 / 2048), np.full(8192, 1.0 / 8192), Cd / Cd.max(),
                                0.1, 60, 0.0)
    assert np.abs(Pc - Pr).max() / np.abs(Pr).max() < 1e-4


def _uneven_worker(rank, world, port, out_dir):
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
    dev = torch.device("cuda", 0)
    rows = [1024, 1536]
    n, m = sum(rows), 1024
    rng = np.random.default_rng(17)
    C = rng.random((n, m))
    r0 = sum(rows[:rank])
    sl = slice(r0, r0 + rows[rank])
    xp = D.XPeer(m)
    res = D.sinkhorn_xsweep(torch.full((rows[rank],), 1.0 / n, device=dev), torch.full((m,), 1.0 / m, device=dev),
                            torch.tensor(C[sl], device=dev, dtype=torch.float32), 0.05, xp, n_total=n,
                            max_iter=500, stop_thr=1e-6)
    info = res.info()
    np.savez(os.path.join(out_dir, f"u{rank}.npz"), P=res.plan.cpu().numpy(), niter=info["niter"],
             status=info["status"], engine=info["engine_name"], v=res.v.cpu().numpy())
    xp.close()
    dist.barrier()
    dist.destroy_process_group()


def test_xsweep_uneven_mesh_shaped_shards_agree(tmp_path, orc):
    """shards of 1024 and 1536 rows x 1024 columns -- each alone a float32 mesh
    slab, with different tilings -- under a converging stop (stopThr 1e-6): the ranks agree
    on one engine (the sweep, otfuse.distributed.xsweep_engine), stop at the oracle's
    iteration together and assemble its plan."""
    world = 2
    mp.spawn(_uneven_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    rows = [1024, 1536]
    n, m = sum(rows), 1024
    C = np.random.default_rng(17).random((n, m))
    P_ref, _, _, info_r = orc.sinkhorn_knopp(np.full(n, 1.0 / n), np.full(m, 1.0 / m), C, 0.05, 500, 1e-6)
    zs = [np.load(tmp_path / f"u{r}.npz") for r in range(world)]
    assert all(str(z["engine"]) == "sweep" for z in zs)
    assert all(int(z["niter"]) == info_r["niter"] < 499 for z in zs)
    assert np.array_equal(zs[0]["v"], zs[1]["v"])
    P = np.concatenate([z["P"] for z in zs])
    assert np.abs(P - P_ref).max() / np.abs(P_ref).max() < 1e-4
