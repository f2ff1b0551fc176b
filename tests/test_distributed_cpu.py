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


class NumpyPasses:
    """Per-pass restatement of POT sinkhorn_knopp on this rank's rows (test backend for
    the protocol of otfuse.distributed.sinkhorn_row_sharded; the product backend is
    DevicePasses over otf_sinkhorn_pass)."""

    def __init__(self, a_local, b, C_local, reg, max_iter, stop_thr, cost_scale, n_total,
                 check_every=10, err_squared=False):
        self.K = np.exp(-C_local.numpy() / reg)
        self.a = a_local.numpy()
        self.b = b.numpy()
        self.n_total = n_total
        self.m = self.K.shape[1]
        self.u = np.full(self.K.shape[0], 1.0 / n_total)
        self.v = np.full(self.m, 1.0 / self.m)
        self.cs = None

    def run_pass(self, p):
        if p >= 1:
            self.v = self.b / self.cs[: self.m].numpy()
            self.u = self.a / (self.K @ self.v)
        out = np.zeros(self.m + 1)
        out[: self.m] = self.K.T @ self.u
        out[self.m] = np.count_nonzero(~np.isfinite(self.u))
        self.cs = torch.from_numpy(out)
        return self.cs

    def stopped(self):
        return False

    def finish(self, want_plan=True, plan_dtype=None):
        return self.u[:, None] * self.K * self.v[None, :]


def _sharded_worker(rank, world, port, out_dir):
    import sys
    for p in (PKG, REPO):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import oracle as orc
    import otfuse.distributed as D
    rng = np.random.default_rng(7)
    rows = [5, 8]                      # ragged shards: u0 must be 1/n_total on every rank
    n, m = sum(rows), 11
    C = rng.random((n, m))
    a = rng.random(n) + 0.5
    a /= a.sum()
    b = rng.random(m) + 0.5
    b /= b.sum()
    r0 = sum(rows[:rank])
    sl = slice(r0, r0 + rows[rank])
    P_local = D.sinkhorn_row_sharded(torch.from_numpy(a[sl]), torch.from_numpy(b),
                                     torch.from_numpy(C[sl]), 0.2, max_iter=25, stop_thr=0.0,
                                     backend=NumpyPasses)
    P_ref, *_ = orc.sinkhorn_knopp(a, b, C, 0.2, 25, 0.0)
    np.testing.assert_allclose(P_local, P_ref[sl], rtol=1e-12, atol=1e-15)
    open(os.path.join(out_dir, f"sharded{rank}"), "w").write("ok")
    dist.barrier()
    dist.destroy_process_group()


def test_row_sharded_sinkhorn_protocol_world2(tmp_path):
    world = 2
    mp.spawn(_sharded_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    assert all((tmp_path / f"sharded{r}").exists() for r in range(world))


class GlooComm:
    """Stand-in for otfuse.comm.Communicator over gloo (CPU): same all_gather /
    all_reduce contract, so coupled_solve_sharded's communicator path runs here."""

    def __init__(self):
        self.rank, self.nranks = dist.get_rank(), dist.get_world_size()

    def all_gather(self, t):
        t = t.contiguous()
        out = t.new_empty((self.nranks * t.shape[0],) + tuple(t.shape[1:]))
        dist.all_gather_into_tensor(out, t)
        return out

    def all_reduce(self, t, op="sum"):
        dist.all_reduce(t, op=dist.ReduceOp.SUM if op == "sum" else dist.ReduceOp.MAX)
        return t


def _coupled_worker(rank, world, port, out_dir):
    import sys
    for p in (PKG, REPO):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import oracle as orc
    import otfuse.comm as CM
    import otfuse.distributed as D
    D.ops._dev = lambda t, name: t          # CPU tensors stand in for device tensors
    GlooComm.all_gather_rows = CM.Communicator.all_gather_rows

    def cost_ex(X, Y, zero_diag=False, out_dtype=None):
        C = torch.from_numpy(((X.double().numpy()[:, None, :] - Y.double().numpy()[None]) ** 2).sum(-1))
        return C, C.max().reshape(1), torch.ones(1, dtype=torch.float64)

    class Passes(NumpyPasses):
        def __init__(self, a_local, b, C_local, reg, max_iter, stop_thr, cost_scale, n_total,
                     *args):
            super().__init__(a_local.double(), b.double(), C_local / cost_scale, reg, max_iter,
                             stop_thr, None, n_total)
            self.max_iter = max_iter

        def solve_with_comm(self, comm, want_plan=True, plan_dtype=None):
            for p in range(self.max_iter + 1):
                comm.all_reduce(self.run_pass(p))
            return self.finish()

    D.ops.pairwise_cost_ex = cost_ex
    D.DevicePasses = Passes
    rng = np.random.default_rng(11)
    rows_x, rows_y = [5, 9], [7, 4]       # unequal shards on both sides
    X = rng.random((sum(rows_x), 3))
    Y = rng.random((sum(rows_y), 3))
    sx = slice(sum(rows_x[:rank]), sum(rows_x[:rank + 1]))
    sy = slice(sum(rows_y[:rank]), sum(rows_y[:rank + 1]))
    P_local, n_total = D.coupled_solve_sharded(torch.from_numpy(X[sx]), torch.from_numpy(Y[sy]),
                                               0.3, max_iter=20, comm=GlooComm())
    assert n_total == sum(rows_x)
    C = ((X[:, None, :] - Y[None]) ** 2).sum(-1)
    a = np.full(len(X), 1.0 / len(X))
    b = np.full(len(Y), 1.0 / len(Y))
    P_ref, *_ = orc.sinkhorn_knopp(a, b, C / C.max(), 0.3, 20, 0.0)
    # a, b are float32 in coupled_solve_sharded; a wrong n_total would be an O(1) error
    np.testing.assert_allclose(P_local, P_ref[sx], rtol=1e-6, atol=1e-12)
    open(os.path.join(out_dir, f"coupled{rank}"), "w").write("ok")
    dist.barrier()
    dist.destroy_process_group()


def test_coupled_solve_unequal_shards_through_communicator_world2(tmp_path):
    """with a communicator, unequal shard sizes must give n_total = sum of
    the rows (a sums to 1) and a ragged all-gather of Y, matching the single solve."""
    world = 2
    mp.spawn(_coupled_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    assert all((tmp_path / f"coupled{r}").exists() for r in range(world))


def _label_split_worker(rank, world, port, out_dir):
    import sys
    for p in (PKG, REPO):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import oracle as orc
    import otfuse.distributed as D

    # per-label sample couplings from the oracle's entropic GW (the device solver's CPU
    # restatement) on squared-Euclidean costs / max, as egw_label_plans builds them
    def solve(pets, mris):
        plans = []
        for x, y in zip(pets, mris):
            c1, _ = orc.pairwise_cost(x.numpy(), x.numpy(), scale_max=True)
            c2, _ = orc.pairwise_cost(y.numpy(), y.numpy(), scale_max=True)
            T, _ = orc.gw_entropic(c1, c2, 5e-2, max_iter=40)
            plans.append(torch.from_numpy(T))
        return plans, len(plans)

    rng = np.random.default_rng(5)
    sizes = [9, 14, 6, 11, 8]            # 5 labels over 2 ranks: 3 + 2, ragged groups
    pets = [torch.from_numpy(rng.random((s, 4)).astype(np.float32)) for s in sizes]
    mris = [torch.from_numpy(rng.random((s, 5)).astype(np.float32)) for s in sizes]
    plans, mine = D.split_label_plans(pets, mris, GlooComm(), solve)
    assert mine == len(range(rank, len(sizes), world))
    ref, _ = solve(pets, mris)
    assert len(plans) == len(ref)
    for T, R in zip(plans, ref):
        assert T.shape == R.shape and torch.equal(T, R)   # one contribution per plan: exact
    open(os.path.join(out_dir, f"labels{rank}"), "w").write("ok")
    dist.barrier()
    dist.destroy_process_group()


def test_per_epoch_label_split_world2(tmp_path):
    """Config 3's per-epoch chain split over ranks (otfuse.distributed.split_label_plans):
    labels dealt round-robin, one all-reduce of the padded plan stack; every rank ends with
    every label's plan, bit-identical to the unsplit per-label solve."""
    world = 2
    mp.spawn(_label_split_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    assert all((tmp_path / f"labels{r}").exists() for r in range(world))


def _xmesh_model(K_loc, a_loc, b, n_total, reg_iters, check_every, stop_thr, exchange, tile=128):
    """The cross-rank mesh's arithmetic order (csrc/otf_mesh.hip, XR instances), restated
    for the protocol test: per iteration every row block (producer) forms its column
    partials K_rb^T u, the rank's reducers sum them in producer order, the ranks' partials
    are exchanged and summed in rank order (``exchange``: the stand-in for the stores into
    the peers' buffers), v = b / S; the rows are local (u = a / K v).  POT's marginal error
    of iterate it - 1 every check_every iterations, from the global S; stop below stop_thr."""
    n_loc, m = K_loc.shape
    u = np.full(n_loc, 1.0 / n_total)
    nb = -(-n_loc // tile)

    def colsum(u):
        s = np.zeros(m)
        for rb in range(nb):
            sl = slice(rb * tile, min(n_loc, (rb + 1) * tile))
            s = s + K_loc[sl].T @ u[sl]
        return exchange(s)

    S = colsum(u)
    errs, niter = [], reg_iters - 1
    for it in range(reg_iters):
        v = b / S
        u_new = a_loc / (K_loc @ v)
        S_new = colsum(u_new)
        if it % check_every == 0:
            # POT: err of the current iterate (u_new, v): column marginal v * K^T u_new vs b
            r = v * S_new - b
            errs.append(float(np.sqrt(r @ r)))
            if errs[-1] < stop_thr:
                niter = it
                u = u_new
                break
        u, S = u_new, S_new
    return u[:, None] * K_loc * v[None, :], v, niter, errs


def _xmesh_protocol_worker(rank, world, port, out_dir):
    import sys
    for p in (PKG, REPO):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rng = np.random.default_rng(13)
    rows = [384, 256]                       # unequal slabs: 3 and 2 row blocks of 128
    n, m = sum(rows), 1024
    C = rng.random((n, m))
    K = np.exp(-C / 0.05)
    a = rng.random(n) + 0.5
    a /= a.sum()
    b = rng.random(m) + 0.5
    b /= b.sum()
    sl = slice(sum(rows[:rank]), sum(rows[:rank + 1]))

    def exchange(s):
        parts = [torch.empty(m, dtype=torch.float64) for _ in range(world)]
        dist.all_gather(parts, torch.from_numpy(s))
        out = np.zeros(m)
        for p_ in parts:                     # rank order, every rank the same sum
            out = out + p_.numpy()
        return out

    P, v, niter, errs = _xmesh_model(K[sl], a[sl], b, n, 300, 10, 1e-7, exchange)
    np.savez(os.path.join(out_dir, f"xm{rank}.npz"), P=P, v=v, niter=niter, errs=np.array(errs))
    dist.barrier()
    dist.destroy_process_group()


def test_xmesh_exchange_protocol_world2(tmp_path):
    """The cross-rank mesh's exchange protocol on CPU (gloo standing in for the xGMI
    stores): rank slabs of unequal height, partials summed in rank order -- both ranks
    derive the same v bit for bit, stop at the same check, and the assembled plan is POT's
    (the float64 oracle on the whole problem, MRI_PET_OT_nojax.py:143)."""
    from oracle import oracle as orc
    world = 2
    mp.spawn(_xmesh_protocol_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    zs = [np.load(tmp_path / f"xm{r}.npz") for r in range(world)]
    assert np.array_equal(zs[0]["v"], zs[1]["v"])
    assert int(zs[0]["niter"]) == int(zs[1]["niter"])
    rng = np.random.default_rng(13)
    rows = [384, 256]
    n, m = sum(rows), 1024
    C = rng.random((n, m))
    a = rng.random(n) + 0.5
    a /= a.sum()
    b = rng.random(m) + 0.5
    b /= b.sum()
    P_ref, _, _, info_r = orc.sinkhorn_knopp(a, b, C, 0.05, 300, 1e-7)
    assert int(zs[0]["niter"]) == info_r["niter"]
    np.testing.assert_allclose(zs[0]["errs"], info_r["err"], rtol=1e-9, atol=1e-15)
    P = np.concatenate([z["P"] for z in zs])
    assert np.abs(P - P_ref).max() / np.abs(P_ref).max() < 1e-12


def _engine_agreement_worker(rank, world, port, out_dir):
    import sys
    for p in (PKG, REPO):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import otfuse.distributed as D
    res = {}
    # uneven shards (rank 0: 1024 rows = a mesh slab, rank 1: 1536): "auto" -> the sweep on
    # both ranks; "mesh" refused on both; "sweep" unchanged
    n = 1024 if rank == 0 else 1536
    res["auto_uneven"] = D.xsweep_engine("auto", n, world)
    try:
        D.xsweep_engine("mesh", n, world)
        res["mesh_uneven"] = "accepted"
    except ValueError:
        res["mesh_uneven"] = "refused"
    res["sweep_uneven"] = D.xsweep_engine("sweep", n, world)
    # equal shards keep the request
    res["auto_equal"] = D.xsweep_engine("auto", 1024, world)
    res["mesh_equal"] = D.xsweep_engine("mesh", 1024, world)
    np.save(os.path.join(out_dir, f"e{rank}.npy"), np.array([res[k] for k in sorted(res)]))
    dist.destroy_process_group()


def test_xsweep_engine_agreed_over_ranks(tmp_path):
    """the cross-rank engine is agreed over the exchange's group, never picked
    by each rank from its own shard -- two engines (or two mesh tilings) round POT's error
    differently and could stop at different checks, leaving a peer waiting on the
    exchange.  Uneven shards: every rank takes the sweep (auto) or refuses the mesh."""
    world = 2
    mp.spawn(_engine_agreement_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    e0, e1 = (list(np.load(tmp_path / f"e{r}.npy")) for r in range(world))
    assert e0 == e1
    keys = sorted(["auto_uneven", "mesh_uneven", "sweep_uneven", "auto_equal", "mesh_equal"])
    got = dict(zip(keys, e0))
    assert got == {"auto_uneven": "sweep", "mesh_uneven": "refused", "sweep_uneven": "sweep",
                   "auto_equal": "auto", "mesh_equal": "mesh"}
