"""Mesh engine, float64 form (csrc/otf_mesh64.hip): POT's sinkhorn_knopp
(MRI_PET_OT_nojax.py:143 -> POT sinkhorn_knopp, perturbot/perturbot/match/utils.py:6-115)
in the reference's own precision with K = exp(-C/reg) held on chip (registers + LDS) for
the whole solve, on whole 128 x 512 tiles (4..32 row blocks x 1..8 column tiles; the
N = 4096 metric shape is bench.py's metric_f64 leg).  Checked against the float64 oracle
at 1e-9 and against the sweep engine (needs an MI355X)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

TOL64 = 1e-9  # normwise relative plan tolerance of the float64 paths


def nrel(x, ref):
    x = np.asarray(x, dtype=np.float64)
    ref = np.asarray(ref, dtype=np.float64)
    return np.abs(x - ref).max() / np.abs(ref).max()


def _t(x, dev):
    return torch.as_tensor(np.asarray(x, dtype=np.float64), device=dev)


@pytest.mark.parametrize("n,m", [(512, 1024), (1024, 4096), (2048, 512), (4096, 2048), (4096, 4096)])
def test_mesh64_shapes_vs_oracle(orc, dev, n, m):
    """4 / 8 / 16 / 32 row blocks, 1 (no row hop) / 2 / 4 / 8 column tiles, non-uniform
    marginals, 40 fixed iterations: plan, scalings and iteration count of the oracle."""
    from otfuse import ops
    rng = np.random.default_rng(n + 7 * m)
    C = rng.random((n, m))
    a = rng.random(n) + 0.5
    a /= a.sum()
    b = rng.random(m) + 0.5
    b /= b.sum()
    P_r, u_r, v_r, info_r = orc.sinkhorn_knopp(a, b, C, 0.05, 40, 0.0)
    res = ops.sinkhorn(_t(a, dev), _t(b, dev), _t(C, dev), 0.05, max_iter=40, stop_thr=0.0, engine="mesh")
    info = res.info()
    assert info["engine_name"] == "mesh" and info["status_name"] == "max_iter"
    assert info["niter"] == info_r["niter"] and res.u.dtype == torch.float64
    assert nrel(res.plan.cpu().numpy(), P_r) < TOL64
    c = float(np.median(res.u.cpu().numpy() / u_r))
    np.testing.assert_allclose(res.u.cpu().numpy() / c, u_r, rtol=1e-10)
    np.testing.assert_allclose(res.v.cpu().numpy() * c, v_r, rtol=1e-10)


def test_mesh64_is_auto_for_whole_tiles_and_matches_sweep(dev):
    """AUTO takes the float64 mesh for a whole-tile float64 cost; the sweep engine (K
    streamed from the workspace) agrees to float64 rounding; two runs are bitwise equal."""
    from otfuse import ops
    n = m = 4096
    g = torch.Generator(device=dev).manual_seed(17)
    C = torch.rand(n, m, device=dev, generator=g, dtype=torch.float64)
    a = torch.full((n,), 1.0 / n, device=dev, dtype=torch.float64)
    r1 = ops.sinkhorn(a, a, C, 0.05, max_iter=120, stop_thr=0.0)
    r2 = ops.sinkhorn(a, a, C, 0.05, max_iter=120, stop_thr=0.0)
    rs = ops.sinkhorn(a, a, C, 0.05, max_iter=120, stop_thr=0.0, engine="sweep")
    assert r1.info()["engine_name"] == "mesh" and rs.info()["engine_name"] == "sweep"
    assert torch.equal(r1.plan, r2.plan) and torch.equal(r1.u, r2.u) and torch.equal(r1.v, r2.v)
    assert (r1.plan - rs.plan).abs().max().item() / rs.plan.abs().max().item() < 1e-12


def test_mesh64_converged_stop_and_error_log(orc, dev):
    """POT's error check every 10 iterations travels reducer -> column tile -> row hop:
    the same stopping iteration and error log as the oracle (float64 both)."""
    from otfuse import ops
    rng = np.random.default_rng(41)
    n, m = 2048, 1536
    C = rng.random((n, m))
    a = np.full(n, 1.0 / n)
    b = np.full(m, 1.0 / m)
    P_r, *_, info_r = orc.sinkhorn_knopp(a, b, C, 0.05, 2000, 1e-9)
    assert info_r["niter"] < 1999
    res = ops.sinkhorn(_t(a, dev), _t(b, dev), _t(C, dev), 0.05, max_iter=2000, stop_thr=1e-9, engine="mesh")
    info = res.info()
    assert info["engine_name"] == "mesh" and info["status_name"] == "converged"
    assert info["niter"] == info_r["niter"]
    np.testing.assert_allclose(info["err"], info_r["err"], rtol=1e-6, atol=1e-15)
    assert nrel(res.plan.cpu().numpy(), P_r) < TOL64
    # squared-error mode (vendored utils.py:88-89)
    _, _, _, info_s = orc.sinkhorn_knopp(a, b, C, 0.05, 2000, 1e-16, err_squared=True)
    rs = ops.sinkhorn(_t(a, dev), _t(b, dev), _t(C, dev), 0.05, max_iter=2000, stop_thr=1e-16,
                      err_squared=True, engine="mesh")
    assert rs.info()["niter"] == info_s["niter"]


def test_mesh64_last_iteration_check(orc, dev):
    """max_iter - 1 on a check (91 iterations): the final error takes the extra exchange."""
    from otfuse import ops
    rng = np.random.default_rng(6)
    n, m = 1024, 2048
    x = np.sort(rng.random(n))
    y = np.sort(rng.random(m)) ** 2
    C = (x[:, None] - y[None, :]) ** 2
    a = np.full(n, 1.0 / n)
    b = np.full(m, 1.0 / m)
    P_r, *_, info_r = orc.sinkhorn_knopp(a, b, C, 0.01, 91, 0.0)
    res = ops.sinkhorn(_t(a, dev), _t(b, dev), _t(C, dev), 0.01, max_iter=91, stop_thr=0.0, engine="mesh")
    info = res.info()
    assert info["n_err"] == len(info_r["err"]) == 10
    np.testing.assert_allclose(info["err"], info_r["err"], rtol=1e-7)
    assert nrel(res.plan.cpu().numpy(), P_r) < TOL64


def test_mesh64_numerical_break_matches_oracle(orc, dev):
    """A column whose K underflows to zero in float64 (C / reg > 745): K^T u = 0 at
    iteration 0, POT's revert-and-break, the same plan as the oracle."""
    from otfuse import ops
    rng = np.random.default_rng(23)
    n, m = 1024, 1024
    a = np.full(n, 1.0 / n)
    b = np.full(m, 1.0 / m)
    C = rng.random((n, m))
    C[:, 300] = 1e3
    P_r, *_, info_r = orc.sinkhorn_knopp(a, b, C, 1.0, 100, 0.0)
    assert info_r["break_iter"] == 0
    res = ops.sinkhorn(_t(a, dev), _t(b, dev), _t(C, dev), 1.0, max_iter=100, stop_thr=0.0, engine="mesh")
    info = res.info()
    assert info["engine_name"] == "mesh" and info["status_name"] == "numerical_break"
    assert info["break_iter"] == 0 and info["niter"] == info_r["niter"]
    assert nrel(res.plan.cpu().numpy(), P_r) < TOL64


def test_mesh64_cost_scale_and_float32_plan(orc, dev):
    """scale_cost = "max_cost" through cost_scale (a device scalar) and a float32 plan."""
    from otfuse import ops
    rng = np.random.default_rng(8)
    n, m = 1024, 1024
    C = rng.random((n, m)) * 7.0
    a = np.full(n, 1.0 / n)
    P_r, *_ = orc.sinkhorn_knopp(a, a, C / C.max(), 0.1, 50, 0.0)
    Cd = _t(C, dev)
    cs = Cd.max().reshape(1)
    r64 = ops.sinkhorn(_t(a, dev), _t(a, dev), Cd, 0.1, max_iter=50, stop_thr=0.0, cost_scale=cs, engine="mesh")
    r32 = ops.sinkhorn(_t(a, dev), _t(a, dev), Cd, 0.1, max_iter=50, stop_thr=0.0, cost_scale=cs, engine="mesh",
                       plan_dtype=torch.float32)
    assert r64.info()["engine_name"] == r32.info()["engine_name"] == "mesh"
    assert nrel(r64.plan.cpu().numpy(), P_r) < TOL64
    assert r32.plan.dtype == torch.float32
    assert nrel(r32.plan.cpu().numpy(), P_r) < 1e-6


@pytest.mark.parametrize("n,m", [(4096, 4096), (1024, 2048)])
def test_mesh64_xcc_local_and_write_through_paths_agree_bitwise(dev, monkeypatch, n, m):
    """XCC-registration roles (plain stores inside one L2) and blockIdx roles (every hop
    write-through) reduce in the same fixed order: identical bits."""
    from otfuse import ops
    g = torch.Generator(device=dev).manual_seed(12)
    C = torch.rand(n, m, device=dev, generator=g, dtype=torch.float64)
    a = torch.full((n,), 1.0 / n, device=dev, dtype=torch.float64)
    b = torch.full((m,), 1.0 / m, device=dev, dtype=torch.float64)
    r1 = ops.sinkhorn(a, b, C, 0.05, max_iter=60, stop_thr=0.0, engine="mesh")
    monkeypatch.setenv("OTF_MESH_XCC", "0")
    r0 = ops.sinkhorn(a, b, C, 0.05, max_iter=60, stop_thr=0.0, engine="mesh")
    assert r1.info()["engine_name"] == r0.info()["engine_name"] == "mesh"
    assert torch.equal(r0.plan, r1.plan) and torch.equal(r0.u, r1.u) and torch.equal(r0.v, r1.v)
