"""Gather engine (csrc/otf_gather.hip): the per-batch feature plans of the training
loop (BASELINE config 2: 512 x 512 float64, MRI_PET_OT_nojax.py:143) and every other
problem of <= 16 row tiles x <= 512 columns, with the column sums exchanged as
epoch-tagged granules instead of atomics + a grid barrier.  Checked against the
oracle's sinkhorn_knopp restatement, the F2 golden vectors (made by the reference's own
get_feature_coupling_pot) and the other engines (needs an MI355X)."""
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


def test_config2_takes_gather_and_matches_golden(golden, orc, dev):
    """AUTO picks the gather engine for the config-2 feature plan; F2 golden (reference
    get_feature_coupling_pot, 2000 iterations at eps 1e-2) to 1e-9, and the same plan
    as the row-block resident engine to 1e-12."""
    from otfuse import ops
    from otfuse.pot import feature_coupling_pot_device
    f = golden("f2_feature_pot_b8_d512.npz")
    ts = torch.full((8,), 1 / 8, dtype=torch.float64, device=dev)
    res = feature_coupling_pot_device(_t(f["X"], dev), _t(f["Y"], dev), ts_diag=ts, eps=1e-2)
    info = res.info()
    assert info["engine_name"] == "gather"
    assert info["n_err"] == int(f["n_err"]) and info["status_name"] == "max_iter"
    np.testing.assert_allclose(info["err"], f["err"], rtol=1e-5)
    P = res.plan.cpu().numpy()
    idx = f["idx"]
    assert nrel(P[idx[:, 0], idx[:, 1]], f["plan_samples"]) < 1e-9
    assert nrel(P.sum(1), f["plan_rowsum"]) < 1e-9
    M = orc.feature_cost(f["X"], f["Y"], np.eye(8) / 8)
    u = torch.full((M.shape[0],), 1.0 / M.shape[0], dtype=torch.float64, device=dev)
    r2 = ops.sinkhorn(u, u, _t(M, dev), 1e-2, max_iter=2000, stop_thr=1e-9, engine="resident")
    assert nrel(P, r2.plan.cpu().numpy()) < 1e-12


@pytest.mark.parametrize("n,m,dt", [(1, 1, torch.float64), (65, 33, torch.float64),
                                    (960, 512, torch.float64), (1023, 511, torch.float64),
                                    (129, 64, torch.float32), (2047, 512, torch.float32),
                                    (256, 3, torch.float32), (5, 500, torch.float64)])
def test_gather_grid_sizes_vs_oracle(orc, dev, n, m, dt):
    """1..16 workgroups (ragged last tile), ragged last chunk, non-uniform marginals."""
    from otfuse import ops
    rng = np.random.default_rng(n * 7 + m)
    C = rng.random((n, m))
    a = rng.random(n) + 0.5
    a /= a.sum()
    b = rng.random(m) + 0.5
    b /= b.sum()
    P_r, u_r, v_r, info_r = orc.sinkhorn_knopp(a, b, C, 0.1, 60, 0.0)
    res = ops.sinkhorn(_t(a, dev, dt), _t(b, dev, dt), _t(C, dev, dt), 0.1, max_iter=60,
                       stop_thr=0.0, engine="gather")
    info = res.info()
    assert info["engine_name"] == "gather" and info["niter"] == info_r["niter"]
    tol = 1e-4 if dt == torch.float32 else 1e-10
    assert nrel(res.plan.cpu().numpy(), P_r) < tol


@pytest.mark.parametrize("n,m,dt", [(512, 512, torch.float64), (2048, 500, torch.float32)])
def test_gather_is_bitwise_reproducible(dev, n, m, dt):
    """Every workgroup adds the partials in workgroup order: same bits every run."""
    from otfuse import ops
    g = torch.Generator(device=dev).manual_seed(n)
    C = torch.rand(n, m, device=dev, generator=g, dtype=torch.float64).to(dt)
    a = torch.full((n,), 1.0 / n, device=dev, dtype=dt)
    b = torch.full((m,), 1.0 / m, device=dev, dtype=dt)
    outs = [ops.sinkhorn(a, b, C, 0.05, max_iter=300, stop_thr=0.0, engine="gather") for _ in range(3)]
    for r in outs:
        assert r.info()["engine_name"] == "gather"
    assert torch.equal(outs[0].plan, outs[1].plan) and torch.equal(outs[0].plan, outs[2].plan)
    assert torch.equal(outs[0].u, outs[2].u) and torch.equal(outs[0].v, outs[2].v)


def test_gather_break_mid_solve_matches_oracle(orc, dev):
    """A numerical break after some iterations (u overflows at a tiny reg) reverts to the
    same iterate as POT / the oracle."""
    from otfuse import ops
    rng = np.random.default_rng(5)
    n, m = 300, 200
    C = rng.random((n, m)) * 3.0
    a = np.full(n, 1.0 / n)
    b = np.full(m, 1.0 / m)
    P_r, *_, info_r = orc.sinkhorn_knopp(a, b, C, 4e-3, 500, 0.0)
    res = ops.sinkhorn(_t(a, dev), _t(b, dev), _t(C, dev), 4e-3, max_iter=500, stop_thr=0.0,
                       engine="gather")
    info = res.info()
    assert info["status_name"] == ("numerical_break" if info_r["break_iter"] >= 0 else "max_iter")
    assert info["niter"] == info_r["niter"] and info["break_iter"] == info_r["break_iter"]
    assert nrel(res.plan.cpu().numpy(), P_r) < 1e-9


def test_gather_unsupported_shapes_are_refused(dev):
    from otfuse import ops
    for n, m, dt in [(64, 513, torch.float64), (1025, 64, torch.float64), (2049, 64, torch.float32)]:
        C = torch.rand(n, m, device=dev, dtype=dt)
        a = torch.full((n,), 1.0 / n, device=dev, dtype=dt)
        b = torch.full((m,), 1.0 / m, device=dev, dtype=dt)
        with pytest.raises(Exception, match="unsupported"):
            ops.sinkhorn(a, b, C, 0.1, max_iter=10, engine="gather")
        # AUTO still solves it with another engine
        assert ops.sinkhorn(a, b, C, 0.1, max_iter=10).info()["engine_name"] != "gather"


def test_two_gather_solves_on_two_streams(dev):
    """Small grids: two concurrent solves are co-resident and both finish correctly."""
    from otfuse import ops
    n = m = 512
    g = torch.Generator(device=dev).manual_seed(3)
    C = torch.rand(n, m, device=dev, generator=g, dtype=torch.float64)
    a = torch.full((n,), 1.0 / n, device=dev, dtype=torch.float64)
    ref = ops.sinkhorn(a, a, C, 0.05, max_iter=400, stop_thr=0.0, engine="stream").plan
    s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    torch.cuda.synchronize()
    outs = []
    for s in (s1, s2):
        with torch.cuda.stream(s):
            outs.append(ops.sinkhorn(a, a, C, 0.05, max_iter=400, stop_thr=0.0, engine="gather"))
    torch.cuda.synchronize()
    for r in outs:
        assert r.info()["status_name"] == "max_iter"
        assert (r.plan - ref).abs().max() / ref.abs().max() < 1e-12


def test_gather_team_mode_agrees_bitwise(dev, monkeypatch):
    """XCC team mode (8 x nwg workgroups launched, the first complete XCC team solves with
    plain stores inside its L2) and the one-workgroup-per-tile write-through launch add
    the partials in the same order: identical bits, config-2 shape, float64."""
    from otfuse import ops
    n = m = 512
    g = torch.Generator(device=dev).manual_seed(21)
    C = torch.rand(n, m, device=dev, generator=g, dtype=torch.float64)
    a = torch.full((n,), 1.0 / n, device=dev, dtype=torch.float64)
    r1 = ops.sinkhorn(a, a, C, 0.02, max_iter=500, stop_thr=0.0, engine="gather")
    monkeypatch.setenv("OTF_GATHER_TEAM", "0")
    r0 = ops.sinkhorn(a, a, C, 0.02, max_iter=500, stop_thr=0.0, engine="gather")
    assert r1.info()["engine_name"] == r0.info()["engine_name"] == "gather"
    assert torch.equal(r0.plan, r1.plan) and torch.equal(r0.u, r1.u) and torch.equal(r0.v, r1.v)


@pytest.mark.parametrize("dt", [torch.float64, torch.float32])
def test_gather_zero_column_sum_breaks_like_pot(orc, dev, dt):
    """A column whose K underflows entirely (S_j = 0): POT reverts at iteration 0.  The
    float64 chunks carry their tag in the values' low mantissa bits -- an exact zero must
    come back as zero once the tag is cleared, or the break would be missed."""
    from otfuse import ops
    rng = np.random.default_rng(11)
    n, m = 512, 512
    C = rng.random((n, m))
    C[:, 37] = 2e3   # exp(-2e3 / 0.5) = 0 in float32 and float64
    a = np.full(n, 1.0 / n)
    b = np.full(m, 1.0 / m)
    P_r, *_, info_r = orc.sinkhorn_knopp(a, b, C, 0.5, 50, 0.0)
    res = ops.sinkhorn(_t(a, dev, dt), _t(b, dev, dt), _t(C, dev, dt), 0.5, max_iter=50,
                       stop_thr=0.0, engine="gather")
    info = res.info()
    assert info["engine_name"] == "gather"
    assert info["status_name"] == ("numerical_break" if info_r["break_iter"] >= 0 else "max_iter")
    assert info["niter"] == info_r["niter"] and info["break_iter"] == info_r["break_iter"]
    assert nrel(res.plan.cpu().numpy(), P_r) < (1e-5 if dt == torch.float32 else 1e-12)
