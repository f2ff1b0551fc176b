"""Mesh engine (csrc/otf_mesh.hip): the headline metric config (BASELINE.json configs[1]:
N = 4096, eps = 0.1, 100 iterations; MRI_PET_OT_nojax.py:143 -> POT sinkhorn_knopp,
perturbot/perturbot/match/utils.py:6-115) and every float32 problem of 4..64 row tiles x
1..8 column tiles, with both reductions exchanged as epoch-tagged granules (row hop,
column partials -> reducer -> sums) instead of atomics + barriers.  Checked against the
oracle's sinkhorn_knopp restatement and the other engines (needs an MI355X)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def nrel(x, ref):
    x = np.asarray(x, dtype=np.float64)
    ref = np.asarray(ref, dtype=np.float64)
    return np.abs(x - ref).max() / np.abs(ref).max()


def _t(x, dev, dt=None):
    return torch.as_tensor(np.asarray(x), device=dev, dtype=dt)


def test_metric_config_takes_mesh_and_matches_oracle(orc, dev):
    """AUTO picks the mesh engine for the metric config; plan within 1e-4 normwise of the
    float64 oracle, same as the tiled engine's plan to float32 rounding."""
    from otfuse import ops
    from otfuse.synthetic import paired_embeddings
    N, d = 4096, 512
    X, Y, _ = paired_embeddings(N, d, seed=77)
    C, cmax = ops.pairwise_cost(_t(X, dev), _t(Y, dev))
    a = torch.full((N,), 1.0 / N, device=dev)
    res = ops.sinkhorn(a, a, C, 0.1, max_iter=100, stop_thr=0.0, cost_scale=cmax)
    info = res.info()
    assert info["engine_name"] == "mesh" and info["status_name"] == "max_iter"
    assert info["niter"] == 99
    P = res.plan.cpu().numpy().astype(np.float64)
    np.testing.assert_allclose(P.sum(1), 1.0 / N, rtol=1e-4)
    Cr, _ = orc.pairwise_cost(X, Y, scale_max=True)
    Pr, *_ = orc.sinkhorn_knopp(np.full(N, 1.0 / N), np.full(N, 1.0 / N), Cr, 0.1, 100, 0.0)
    assert nrel(P, Pr) < 1e-4
    rt = ops.sinkhorn(a, a, C, 0.1, max_iter=100, stop_thr=0.0, cost_scale=cmax, engine="tiled")
    assert nrel(P, rt.plan.cpu().numpy()) < 1e-5


@pytest.mark.parametrize("n,m", [(512, 512), (640, 3000), (1000, 4096), (2048, 500),
                                 (4100, 1000), (4096, 4096), (8192, 2048), (3001, 2049),
                                 (513, 7), (8100, 100), (1024, 8192), (2048, 6000), (512, 4097)])
def test_mesh_grid_shapes_vs_oracle(orc, dev, n, m):
    """4..64 row tiles (powers of two and not: 8 reducer loads per lane), 1..16 column
    tiles (past 8 the row hop takes two members per lane and the roles are by blockIdx),
    ragged last row tile / column tile / chunk, non-uniform marginals."""
    from otfuse import ops
    rng = np.random.default_rng(n * 3 + m)
    C = rng.random((n, m))
    a = rng.random(n) + 0.5
    a /= a.sum()
    b = rng.random(m) + 0.5
    b /= b.sum()
    P_r, u_r, v_r, info_r = orc.sinkhorn_knopp(a, b, C, 0.1, 40, 0.0)
    res = ops.sinkhorn(_t(a, dev, torch.float32), _t(b, dev, torch.float32),
                       _t(C, dev, torch.float32), 0.1, max_iter=40, stop_thr=0.0, engine="mesh")
    info = res.info()
    assert info["engine_name"] == "mesh" and info["niter"] == info_r["niter"]
    assert nrel(res.plan.cpu().numpy(), P_r) < 1e-4
    np.testing.assert_allclose(res.u.cpu().numpy() * res.v.cpu().numpy().mean(),
                               u_r * v_r.mean(), rtol=1e-3)


def test_mesh_is_bitwise_reproducible(dev):
    """Every sum has one fixed order (no atomics): the same bits every run."""
    from otfuse import ops
    n = m = 4096
    g = torch.Generator(device=dev).manual_seed(5)
    C = torch.rand(n, m, device=dev, generator=g)
    a = torch.full((n,), 1.0 / n, device=dev)
    outs = [ops.sinkhorn(a, a, C, 0.05, max_iter=200, stop_thr=0.0, engine="mesh") for _ in range(3)]
    for r in outs:
        assert r.info()["engine_name"] == "mesh"
    assert torch.equal(outs[0].plan, outs[1].plan) and torch.equal(outs[0].plan, outs[2].plan)
    assert torch.equal(outs[0].u, outs[2].u) and torch.equal(outs[0].v, outs[2].v)


def test_mesh_converged_stop_and_error_log(orc, dev):
    """The marginal error travels reducer -> column tile -> row hop; it stops on the
    oracle's check and logs the same errors (float32 vs float64)."""
    from otfuse import ops
    rng = np.random.default_rng(31)
    n, m = 2048, 1536
    C = rng.random((n, m)).astype(np.float32)
    a = np.full(n, 1.0 / n)
    b = np.full(m, 1.0 / m)
    P_r, *_, info_r = orc.sinkhorn_knopp(a, b, C.astype(np.float64), 0.05, 2000, 1e-5)
    assert info_r["niter"] < 1999
    res = ops.sinkhorn(_t(a, dev, torch.float32), _t(b, dev, torch.float32), _t(C, dev), 0.05,
                       max_iter=2000, stop_thr=1e-5, engine="mesh")
    info = res.info()
    assert info["status_name"] == "converged"
    assert abs(info["niter"] - info_r["niter"]) <= 10
    k = min(len(info["err"]), len(info_r["err"])) - 1
    np.testing.assert_allclose(info["err"][:k], info_r["err"][:k], rtol=2e-3)
    assert nrel(res.plan.cpu().numpy(), P_r) < 1e-3
    # squared-error mode (vendored utils.py:88-89) stops on the same check
    _, _, _, info_s = orc.sinkhorn_knopp(a, b, C.astype(np.float64), 0.05, 2000, 1e-10,
                                         err_squared=True)
    rs = ops.sinkhorn(_t(a, dev, torch.float32), _t(b, dev, torch.float32), _t(C, dev), 0.05,
                      max_iter=2000, stop_thr=1e-10, err_squared=True, engine="mesh")
    assert abs(rs.info()["niter"] - info_s["niter"]) <= 10


def test_mesh_last_iteration_check(orc, dev):
    """max_iter - 1 on a check (91 iterations): the final error needs the extra exchange."""
    from otfuse import ops
    rng = np.random.default_rng(4)
    n, m = 1024, 2048
    # a 1-D transport (sorted points, squared distance) at reg 0.01: the errors decay
    # slowly and stay far above float32's floor over all 10 checks
    x = np.sort(rng.random(n))
    y = np.sort(rng.random(m)) ** 2
    C = (x[:, None] - y[None, :]) ** 2
    a = rng.random(n) + 0.2
    a /= a.sum()
    b = rng.random(m) + 0.2
    b /= b.sum()
    P_r, *_, info_r = orc.sinkhorn_knopp(a, b, C, 0.01, 91, 0.0)
    res = ops.sinkhorn(_t(a, dev, torch.float32), _t(b, dev, torch.float32),
                       _t(C, dev, torch.float32), 0.01, max_iter=91, stop_thr=0.0, engine="mesh")
    info = res.info()
    assert info["n_err"] == len(info_r["err"]) == 10
    np.testing.assert_allclose(info["err"], info_r["err"], rtol=5e-3)
    assert nrel(res.plan.cpu().numpy(), P_r) < 1e-4


def test_mesh_numerical_breaks_match_oracle(orc, dev):
    """A zero column of K (K^T u = 0 at iteration 0: v break) and u overflow mid-solve
    revert to the same iterate as POT / the oracle."""
    from otfuse import ops
    rng = np.random.default_rng(22)
    n, m = 1024, 1024
    a = np.full(n, 1.0 / n)
    b = np.full(m, 1.0 / m)
    C2 = rng.random((n, m)).astype(np.float32)
    C2[:, 700] = 1e3
    P2, *_, info2 = orc.sinkhorn_knopp(a, b, C2.astype(np.float64), 1.0, 100, 0.0)
    assert info2["break_iter"] == 0
    res = ops.sinkhorn(_t(a, dev, torch.float32), _t(b, dev, torch.float32), _t(C2, dev), 1.0,
                       max_iter=100, stop_thr=0.0, engine="mesh", shift=False)
    info = res.info()
    assert info["status_name"] == "numerical_break" and info["break_iter"] == 0
    assert info["niter"] == info2["niter"]
    assert nrel(res.plan.cpu().numpy(), P2) < 1e-5
    # u overflows in the plain float32 kernel after a few iterations at a small reg (the
    # shifted kernel, AUTO's choice here, does not: this pins the plain kernel's break)
    C3 = (rng.random((n, m)) * 3.0).astype(np.float32)
    ref = ops.sinkhorn(_t(a, dev, torch.float32), _t(b, dev, torch.float32), _t(C3, dev), 8e-3,
                       max_iter=300, stop_thr=0.0, engine="stream", shift=False)
    res = ops.sinkhorn(_t(a, dev, torch.float32), _t(b, dev, torch.float32), _t(C3, dev), 8e-3,
                       max_iter=300, stop_thr=0.0, engine="mesh", shift=False)
    ri, mi = ref.info(), res.info()
    assert mi["status_name"] == ri["status_name"]
    assert mi["niter"] == ri["niter"] and mi["break_iter"] == ri["break_iter"]
    if ri["status_name"] == "numerical_break":
        assert mi["break_iter"] >= 1
    assert nrel(res.plan.cpu().numpy(), ref.plan.cpu().numpy()) < 1e-3


def test_mesh_fp16_cost_storage(dev):
    """fp16 cost storage (BASELINE config 5 form) computed in float32: same plan as the
    streaming engine on the same fp16 cost."""
    from otfuse import ops
    n = m = 4096
    g = torch.Generator(device=dev).manual_seed(9)
    C = torch.rand(n, m, device=dev, generator=g).half()
    a = torch.full((n,), 1.0 / n, device=dev)
    ref = ops.sinkhorn(a, a, C, 0.1, max_iter=60, stop_thr=0.0, engine="stream")
    res = ops.sinkhorn(a, a, C, 0.1, max_iter=60, stop_thr=0.0)
    assert res.info()["engine_name"] == "mesh"
    assert (res.plan - ref.plan).abs().max() / ref.plan.abs().max() < 1e-5


def test_mesh_float64_plan_output(dev):
    from otfuse import ops
    n, m = 1024, 1024
    g = torch.Generator(device=dev).manual_seed(2)
    C = torch.rand(n, m, device=dev, generator=g)
    a = torch.full((n,), 1.0 / n, device=dev)
    r32 = ops.sinkhorn(a, a, C, 0.1, max_iter=30, stop_thr=0.0, engine="mesh")
    r64 = ops.sinkhorn(a, a, C, 0.1, max_iter=30, stop_thr=0.0, engine="mesh", plan_dtype=torch.float64)
    assert r64.plan.dtype == torch.float64
    assert (r64.plan.float() - r32.plan).abs().max() / r32.plan.abs().max() < 1e-6


def test_mesh_unsupported_shapes_are_refused(dev):
    from otfuse import ops
    for n, m, dt in [(300, 200, torch.float32), (1024, 8193, torch.float32),
                     (8193, 512, torch.float32), (1000, 1024, torch.float64),
                     (1024, 1000, torch.float64), (384, 512, torch.float64)]:
        C = torch.rand(n, m, device=dev, dtype=dt)
        a = torch.full((n,), 1.0 / n, device=dev, dtype=dt)
        b = torch.full((m,), 1.0 / m, device=dev, dtype=dt)
        with pytest.raises(Exception, match="unsupported"):
            ops.sinkhorn(a, b, C, 0.1, max_iter=10, engine="mesh")
        assert ops.sinkhorn(a, b, C, 0.1, max_iter=10).info()["engine_name"] != "mesh"


@pytest.mark.parametrize("n,m", [(4096, 4096), (1000, 1500)])
def test_mesh_xcc_local_and_write_through_paths_agree_bitwise(dev, monkeypatch, n, m):
    """Roles by XCC registration (column path inside one L2, plain stores; 8 x nrb
    workgroups launched, surplus leaves) and by blockIdx (every hop write-through) reduce
    in the same fixed order: identical bits."""
    from otfuse import ops
    g = torch.Generator(device=dev).manual_seed(11)
    C = torch.rand(n, m, device=dev, generator=g)
    a = torch.full((n,), 1.0 / n, device=dev)
    b = torch.full((m,), 1.0 / m, device=dev)
    r1 = ops.sinkhorn(a, b, C, 0.05, max_iter=120, stop_thr=0.0, engine="mesh")
    monkeypatch.setenv("OTF_MESH_XCC", "0")
    r0 = ops.sinkhorn(a, b, C, 0.05, max_iter=120, stop_thr=0.0, engine="mesh")
    assert r1.info()["engine_name"] == r0.info()["engine_name"] == "mesh"
    assert torch.equal(r0.plan, r1.plan) and torch.equal(r0.u, r1.u) and torch.equal(r0.v, r1.v)


def test_two_mesh_solves_on_two_streams(dev):
    """Two concurrent 64-workgroup grids: each registers its own XCC population (or falls
    back to write-through roles) and both finish with the streaming engine's plan."""
    from otfuse import ops
    n = m = 1024
    g = torch.Generator(device=dev).manual_seed(3)
    C = torch.rand(n, m, device=dev, generator=g)
    a = torch.full((n,), 1.0 / n, device=dev)
    ref = ops.sinkhorn(a, a, C, 0.05, max_iter=400, stop_thr=0.0, engine="stream").plan
    s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    torch.cuda.synchronize()
    outs = []
    for s in (s1, s2):
        with torch.cuda.stream(s):
            outs.append(ops.sinkhorn(a, a, C, 0.05, max_iter=400, stop_thr=0.0, engine="mesh"))
    torch.cuda.synchronize()
    for r in outs:
        assert r.info()["status_name"] == "max_iter"
        assert (r.plan - ref).abs().max() / ref.abs().max() < 1e-5
