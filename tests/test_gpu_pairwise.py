"""Fused pairwise cost + float64 Sinkhorn (otf_sinkhorn_pairwise_f64, ops.sinkhorn_pairwise):
the reference's ``M = euclidean_distances(X, Y, squared=True); M /= M.max();
ot.sinkhorn(a, b, M, reg)`` (MRI_PET_OT_nojax.py:70-75, :143) with the cost tile of every
workgroup built on the float64 matrix cores inside the float64 mesh's launch.  Checked
against the float64 oracle (cost + POT sinkhorn_knopp) at 1e-9 and against the unfused
device path (gw.pairwise_cost_f64 + ops.sinkhorn) to float64 rounding (needs an MI355X)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

TOL64 = 1e-9  # normwise relative plan tolerance of the float64 paths


def nrel(x, ref):
    x = np.asarray(x, dtype=np.float64)
    ref = np.asarray(ref, dtype=np.float64)
    return np.abs(x - ref).max() / np.abs(ref).max()


def _emb(n, m, d, seed):
    rng = np.random.default_rng(seed)
    X = rng.standard_normal((n, d)).astype(np.float32)
    Y = (0.7 * X[np.arange(m) % n] + 0.5 * rng.standard_normal((m, d))).astype(np.float32)
    return X, Y


def _oracle(orc, X, Y, reg, iters, metric="sqeuclidean", scale_max=True, a=None, b=None, stop=0.0):
    C, mx = orc.pairwise_cost(X, Y, metric=metric)
    n, m = C.shape
    a = np.full(n, 1.0 / n) if a is None else a
    b = np.full(m, 1.0 / m) if b is None else b
    P, u, v, info = orc.sinkhorn_knopp(a, b, C, reg, iters, stop, cscale=1.0 / mx if scale_max else 1.0)
    return P, u, v, info, mx


@pytest.mark.parametrize("n,m,d", [(512, 512, 64), (1024, 2048, 128), (2048, 4096, 256), (512, 1024, 48),
                                   (512, 512, 16)])
def test_pairwise_fused_vs_oracle(orc, dev, n, m, d):
    """4 / 8 / 16 row blocks x 1 / 4 / 8 column tiles, the fused launch (engine="mesh"):
    plan, scalings, iteration count and the cost's max of the oracle; d = 48 and 16 give an
    odd number of 16-deep chunks and a single one (the prologue's X ring wraps / clamps)."""
    from otfuse import ops
    X, Y = _emb(n, m, d, n + m + d)
    P_r, u_r, v_r, info_r, mx = _oracle(orc, X, Y, 0.05, 40)
    res = ops.sinkhorn_pairwise(torch.from_numpy(X).to(dev), torch.from_numpy(Y).to(dev), 0.05,
                                max_iter=40, stop_thr=0.0, engine="mesh")
    info = res.info()
    assert info["engine_name"] == "mesh" and info["status_name"] == "max_iter" and info["fallback"] == 0
    assert info["niter"] == info_r["niter"]
    assert abs(float(res.cost_max) - mx) / mx < 1e-12
    assert nrel(res.plan.cpu().numpy(), P_r) < TOL64
    c = float(np.median(res.u.cpu().numpy() / u_r))
    np.testing.assert_allclose(res.u.cpu().numpy() / c, u_r, rtol=1e-10)
    np.testing.assert_allclose(res.v.cpu().numpy() * c, v_r, rtol=1e-10)


def test_pairwise_metric_shape_matches_unfused(dev):
    """The bench's headline step (N = 4096, d = 512, eps 0.1, 100 iterations): AUTO takes the
    fused launch, which agrees with the cost-then-solve path to float64 rounding (the
    products are summed in another order), and two runs are bitwise equal."""
    from otfuse import gw, ops
    from otfuse.synthetic import paired_embeddings
    Xn, Yn, _ = paired_embeddings(4096, 512, seed=1234)
    X, Y = torch.from_numpy(Xn).to(dev), torch.from_numpy(Yn).to(dev)
    r1 = ops.sinkhorn_pairwise(X, Y, 0.1, max_iter=100, stop_thr=0.0)
    r2 = ops.sinkhorn_pairwise(X, Y, 0.1, max_iter=100, stop_thr=0.0)
    C, cmax = gw.pairwise_cost_f64(X, Y, scale_max=False)
    a = torch.full((4096,), 1.0 / 4096, device=dev, dtype=torch.float64)
    ru = ops.sinkhorn(a, a, C, 0.1, max_iter=100, stop_thr=0.0, cost_scale=cmax)
    assert r1.info()["engine_name"] == "mesh" and ru.info()["engine_name"] == "mesh"
    assert torch.equal(r1.plan, r2.plan) and torch.equal(r1.u, r2.u) and torch.equal(r1.v, r2.v)
    assert abs(float(r1.cost_max) - float(cmax)) / float(cmax) < 1e-13
    assert nrel(r1.plan.cpu().numpy(), ru.plan.cpu().numpy()) < 1e-11


@pytest.fixture(scope="module")
def bench_shape_oracle(orc):
    """The bench's own inputs (bench.py: paired_embeddings(4096, 512, seed=1234)) through the
    oracle's float64 cost once; the POT solves per eps are computed on demand."""
    from otfuse.synthetic import paired_embeddings
    X, Y, _ = paired_embeddings(4096, 512, seed=1234)
    C, mx = orc.pairwise_cost(X, Y)
    a = np.full(4096, 1.0 / 4096)
    cache = {}

    def get(reg):
        if reg not in cache:
            cache[reg] = orc.sinkhorn_knopp(a, a, C, reg, 100, 0.0, cscale=1.0 / mx)
        return cache[reg]
    return X, Y, mx, get


@pytest.mark.parametrize("reg", [0.1, 5e-3])
def test_pairwise_bench_shape_vs_oracle(bench_shape_oracle, dev, reg):
    """The headline launch itself at the exact bench shape (N = 4096, d = 512, 100 iterations,
    stopThr = 0, the bench's seeded inputs): AUTO takes the fused float64 mesh launch, whose
    plan is within 1e-9 of the float64 oracle (cost + POT sinkhorn_knopp), with the oracle's
    iteration count, cost max and scalings (modulo the Sinkhorn scale mode) -- at the bench's
    eps = 0.1 and the reference's per-epoch eps = 5e-3 (MRI_PET_OT_OT_per_epoch_attn.py)."""
    from otfuse import ops
    X, Y, mx, get = bench_shape_oracle
    P_r, u_r, v_r, info_r = get(reg)
    res = ops.sinkhorn_pairwise(torch.from_numpy(X).to(dev), torch.from_numpy(Y).to(dev), reg,
                                max_iter=100, stop_thr=0.0)
    info = res.info()
    assert info["engine_name"] == "mesh" and info["fallback"] == 0
    assert info["status_name"] == "max_iter" and info["niter"] == info_r["niter"] == 99
    assert info["break_iter"] == info_r["break_iter"]
    assert abs(float(res.cost_max) - mx) / mx < 1e-12
    assert nrel(res.plan.cpu().numpy(), P_r) < TOL64
    u, v = res.u.cpu().numpy(), res.v.cpu().numpy()
    c = float(np.median(u / u_r))
    np.testing.assert_allclose(u / c, u_r, rtol=1e-9)
    np.testing.assert_allclose(v * c, v_r, rtol=1e-9)


def test_pairwise_euclidean_unscaled_vs_oracle(orc, dev):
    """The euclidean metric without the max scaling (cost in data units, reg to match)."""
    from otfuse import ops
    X, Y = _emb(1024, 1024, 64, 5)
    P_r, u_r, v_r, info_r, mx = _oracle(orc, X, Y, 2.0, 30, metric="euclidean", scale_max=False)
    res = ops.sinkhorn_pairwise(torch.from_numpy(X).to(dev), torch.from_numpy(Y).to(dev), 2.0,
                                metric="euclidean", scale_max=False, max_iter=30, stop_thr=0.0,
                                engine="mesh")
    assert res.info()["engine_name"] == "mesh"
    assert abs(float(res.cost_max) - mx) / mx < 1e-12
    assert nrel(res.plan.cpu().numpy(), P_r) < TOL64


def test_pairwise_converged_stop_and_float32_plan(orc, dev):
    """POT's stop (error every 10 iterations), non-uniform marginals and a float32 plan."""
    from otfuse import ops
    X, Y = _emb(1024, 2048, 64, 9)
    rng = np.random.default_rng(2)
    a = rng.random(1024) + 0.5
    a /= a.sum()
    b = rng.random(2048) + 0.5
    b /= b.sum()
    P_r, u_r, v_r, info_r, mx = _oracle(orc, X, Y, 0.05, 2000, a=a, b=b, stop=1e-7)
    res = ops.sinkhorn_pairwise(torch.from_numpy(X).to(dev), torch.from_numpy(Y).to(dev), 0.05,
                                a=torch.from_numpy(a).to(dev), b=torch.from_numpy(b).to(dev),
                                max_iter=2000, stop_thr=1e-7, engine="mesh", plan_dtype=torch.float32)
    info = res.info()
    assert info_r["niter"] < 1999
    assert info["status_name"] == "converged" and info["niter"] == info_r["niter"]
    np.testing.assert_allclose(info["err"], info_r["err"], rtol=1e-6, atol=1e-15)
    assert res.plan.dtype == torch.float32
    assert nrel(res.plan.cpu().numpy(), P_r) < 1e-6


@pytest.mark.parametrize("n,m,d", [(1000, 700, 50), (512, 512, 40), (256, 1024, 64)])
def test_pairwise_unfused_shapes_vs_oracle(orc, dev, n, m, d):
    """Shapes the fused launch does not take (ragged tiles, d not a multiple of 16, fewer
    than 4 row blocks): the cost, then the solve, same results."""
    from otfuse import ops
    X, Y = _emb(n, m, d, 3 * n + m)
    P_r, u_r, v_r, info_r, mx = _oracle(orc, X, Y, 0.05, 40)
    res = ops.sinkhorn_pairwise(torch.from_numpy(X).to(dev), torch.from_numpy(Y).to(dev), 0.05,
                                max_iter=40, stop_thr=0.0)
    assert res.info()["niter"] == info_r["niter"]
    assert abs(float(res.cost_max) - mx) / mx < 1e-12
    assert nrel(res.plan.cpu().numpy(), P_r) < TOL64


@pytest.mark.parametrize("xcc", ["1", "0"])
def test_pairwise_registration_fallback(orc, dev, monkeypatch, xcc):
    """A fused grid that cannot become co-resident (a persistent blocker on another stream,
    a 1-ms registration window) gives up; the fallback queued behind it builds the cost and
    solves, returning the oracle's plan (info fallback = 1).  OTF_MESH_XCC=0: blockIdx roles,
    no registration barrier -- the grid-max barrier of the cost build is the first
    device-wide wait and gives up as a registration give-up."""
    from otfuse import ops
    monkeypatch.setenv("OTF_REG_MS", "1")
    monkeypatch.setenv("OTF_MESH_XCC", xcc)
    # the whole-chip shape (256 workgroups): the blocker's CUs keep some of them out
    X, Y = _emb(4096, 4096, 64, 21)
    P_r, u_r, v_r, info_r, mx = _oracle(orc, X, Y, 0.05, 20)
    Xd, Yd = torch.from_numpy(X).to(dev), torch.from_numpy(Y).to(dev)
    g = torch.Generator(device=dev).manual_seed(3)
    Cg = torch.rand(512, 512, device=dev, generator=g, dtype=torch.float64)
    ag = torch.full((512,), 1.0 / 512, device=dev, dtype=torch.float64)
    s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    torch.cuda.synchronize()
    with torch.cuda.stream(s1):
        blocker = ops.sinkhorn(ag, ag, Cg, 0.1, max_iter=40000, stop_thr=0.0, engine="gather",
                               want_plan=False)
    with torch.cuda.stream(s2):
        torch.cuda._sleep(4_000_000)  # ~2 ms: the blocker holds its CUs before the fused grid starts
        res = ops.sinkhorn_pairwise(Xd, Yd, 0.05, max_iter=20, stop_thr=0.0, engine="mesh")
    torch.cuda.synchronize()
    info = res.info()
    assert blocker.info()["status_name"] == "max_iter"
    assert info["status_name"] == "max_iter" and info["niter"] == info_r["niter"]
    assert abs(float(res.cost_max) - mx) / mx < 1e-12
    assert nrel(res.plan.cpu().numpy(), P_r) < TOL64
    if info["fallback"] != 1:
        pytest.skip("the blocker finished before the fused launch: no contention to test")


def test_pairwise_fallback_bench_shape_vs_oracle(bench_shape_oracle, dev, monkeypatch):
    """The fused step's fallback at the bench shape (N = 4096, d = 512, 100 iterations): a
    registration give-up (forced, OTF_FORCE_REG_GIVEUP=1) hands the solve to the relay
    fallback -- the cost tiles, K and 101 streaming passes by a grid that needs no
    co-residency -- whose plan is within 1e-9 of the oracle, with the oracle's iteration
    count and cost max.  Its device time is printed (DESIGN.md records it)."""
    from otfuse import ops
    X, Y, mx, get = bench_shape_oracle
    P_r, u_r, v_r, info_r = get(0.1)
    Xd, Yd = torch.from_numpy(X).to(dev), torch.from_numpy(Y).to(dev)
    monkeypatch.setenv("OTF_FORCE_REG_GIVEUP", "1")
    ws = ops.sinkhorn_pairwise_workspace(4096, 4096, 100, dev)
    res = ops.sinkhorn_pairwise(Xd, Yd, 0.1, max_iter=100, stop_thr=0.0, workspace=ws)
    info = res.info()
    assert info["fallback"] == 1 and info["engine_name"] == "stream" and info["stalled"] == 0
    assert info["status_name"] == "max_iter" and info["niter"] == info_r["niter"]
    assert abs(float(res.cost_max) - mx) / mx < 1e-12
    assert nrel(res.plan.cpu().numpy(), P_r) < TOL64
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(3):
        e0.record()
        ops.sinkhorn_pairwise(Xd, Yd, 0.1, max_iter=100, stop_thr=0.0, workspace=ws, plan_out=res.plan)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    print(f"relay fallback at the bench shape: {sorted(ts)[1]:.3f} ms per call (median of 3)")
    assert sorted(ts)[1] < 20.0
