"""Two-hop mesh (csrc/otf_mesh2.hip, OTF_MESH2=1): 256 x 256 register tiles, the column
side one all-gather of the column tile's 16 producers, the row side one hop, four
tag-in-mantissa floats per 16-B granule.  POT sinkhorn_knopp semantics
(MRI_PET_OT_nojax.py:143 -> perturbot/perturbot/match/utils.py:6-115) against the
float64 oracle and the three-hop mesh engine (needs an MI355X)."""
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


@pytest.fixture
def mesh2(monkeypatch):
    monkeypatch.setenv("OTF_MESH2", "1")


def test_mesh2_metric_config_vs_oracle_and_mesh(orc, dev, mesh2, monkeypatch):
    """N = 4096, d = 512, eps = 0.1, 100 iterations (BASELINE configs[1]): 1e-4 of the
    float64 oracle, 1e-5 of the three-hop engine."""
    from otfuse import ops
    from otfuse.synthetic import paired_embeddings
    N, d = 4096, 512
    X, Y, _ = paired_embeddings(N, d, seed=77)
    C, cmax = ops.pairwise_cost(_t(X, dev), _t(Y, dev))
    a = torch.full((N,), 1.0 / N, device=dev)
    res = ops.sinkhorn(a, a, C, 0.1, max_iter=100, stop_thr=0.0, cost_scale=cmax)
    info = res.info()
    assert info["engine_name"] == "mesh" and info["status_name"] == "max_iter" and info["niter"] == 99
    Cr, _ = orc.pairwise_cost(X, Y, scale_max=True)
    Pr, ur, vr, info_r = orc.sinkhorn_knopp(np.full(N, 1.0 / N), np.full(N, 1.0 / N), Cr, 0.1, 100, 0.0)
    P = res.plan.cpu().numpy()
    assert nrel(P, Pr) < 1e-4
    np.testing.assert_allclose(P.astype(np.float64).sum(1), 1.0 / N, rtol=1e-4)
    monkeypatch.setenv("OTF_MESH2", "0")
    r3 = ops.sinkhorn(a, a, C, 0.1, max_iter=100, stop_thr=0.0, cost_scale=cmax)
    assert nrel(P, r3.plan.cpu().numpy()) < 1e-5
    np.testing.assert_allclose(res.u.cpu().numpy() * res.v.cpu().numpy().mean(),
                               r3.u.cpu().numpy() * r3.v.cpu().numpy().mean(), rtol=1e-4)


@pytest.mark.parametrize("n,m", [(2048, 2048), (4096, 2048), (2048, 4096)])
def test_mesh2_shapes_vs_oracle(orc, dev, mesh2, n, m):
    """8 / 16 row blocks x 8 / 16 column tiles, non-uniform marginals."""
    from otfuse import ops
    rng = np.random.default_rng(n + 7 * m)
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


def test_mesh2_converged_stop_and_error_log(orc, dev, mesh2):
    """The marginal error of iterate it - 1 travels as one row-hop chunk per column tile:
    the oracle's checks, stop within a check of the oracle's iteration."""
    from otfuse import ops
    rng = np.random.default_rng(31)
    n = m = 2048
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


def test_mesh2_last_iteration_check(orc, dev, mesh2):
    """max_iter - 1 on a check (91 iterations): the final error needs the extra exchange."""
    from otfuse import ops
    rng = np.random.default_rng(4)
    n, m = 2048, 4096
    x = np.sort(rng.random(n))
    y = np.sort(rng.random(m)) ** 2
    C = (x[:, None] - y[None, :]) ** 2
    a = rng.random(n) + 0.2
    a /= a.sum()
    b = rng.random(m) + 0.2
    b /= b.sum()
    P_r, *_, info_r = orc.sinkhorn_knopp(a, b, C, 0.01, 91, 0.0)
    res = ops.sinkhorn(_t(a, dev, torch.float32), _t(b, dev, torch.float32),
                       _t(C, dev, torch.float32), 0.01, max_iter=91, stop_thr=0.0, engine="mesh",
                       shift=False)
    info = res.info()
    assert info["n_err"] == len(info_r["err"]) == 10
    np.testing.assert_allclose(info["err"], info_r["err"], rtol=5e-3)
    assert nrel(res.plan.cpu().numpy(), P_r) < 1e-4


def test_mesh2_numerical_breaks_match_oracle(orc, dev, mesh2):
    """A zero column of K (v break at iteration 0) and a u overflow mid-solve revert to the
    same iterate as POT / the streaming engine."""
    from otfuse import ops
    rng = np.random.default_rng(22)
    n = m = 2048
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
    C3 = (rng.random((n, m)) * 3.0).astype(np.float32)
    ref = ops.sinkhorn(_t(a, dev, torch.float32), _t(b, dev, torch.float32), _t(C3, dev), 8e-3,
                       max_iter=300, stop_thr=0.0, engine="stream", shift=False)
    res = ops.sinkhorn(_t(a, dev, torch.float32), _t(b, dev, torch.float32), _t(C3, dev), 8e-3,
                       max_iter=300, stop_thr=0.0, engine="mesh", shift=False)
    ri, mi = ref.info(), res.info()
    assert mi["status_name"] == ri["status_name"]
    assert mi["niter"] == ri["niter"] and mi["break_iter"] == ri["break_iter"]


def test_mesh2_bitwise_reproducible_and_roles_agree(dev, mesh2, monkeypatch):
    """Fixed-order sums: the same bits every run, and XCC-local roles (plain column
    stores) and blockIdx roles (every hop write-through) give identical bits."""
    from otfuse import ops
    n = m = 4096
    g = torch.Generator(device=dev).manual_seed(5)
    C = torch.rand(n, m, device=dev, generator=g)
    a = torch.full((n,), 1.0 / n, device=dev)
    outs = [ops.sinkhorn(a, a, C, 0.05, max_iter=200, stop_thr=0.0, engine="mesh") for _ in range(2)]
    monkeypatch.setenv("OTF_MESH_XCC", "0")
    outs.append(ops.sinkhorn(a, a, C, 0.05, max_iter=200, stop_thr=0.0, engine="mesh"))
    for r in outs:
        assert r.info()["engine_name"] == "mesh"
    assert torch.equal(outs[0].plan, outs[1].plan) and torch.equal(outs[0].plan, outs[2].plan)
    assert torch.equal(outs[0].u, outs[2].u) and torch.equal(outs[0].v, outs[2].v)


def test_mesh2_shifted_kernel_and_fp16_storage(orc, dev, mesh2):
    """The shifted kernel (reg = 0.01, AUTO's choice) and fp16 cost storage on the
    two-hop form: 1e-4 of the float64 oracle on the stored values."""
    from otfuse import ops
    from otfuse.synthetic import paired_embeddings
    N = 4096
    X, Y, _ = paired_embeddings(N, 256, seed=3)
    C, cmax = ops.pairwise_cost(_t(X, dev), _t(Y, dev))
    a = torch.full((N,), 1.0 / N, device=dev)
    res = ops.sinkhorn(a, a, C, 0.01, max_iter=60, stop_thr=0.0, cost_scale=cmax)
    assert res.shifted and res.info()["engine_name"] == "mesh"
    Cs = C.double().cpu().numpy() / float(cmax)
    Pr, *_ = orc.sinkhorn_knopp(np.full(N, 1.0 / N), np.full(N, 1.0 / N), Cs, 0.01, 60, 0.0)
    assert nrel(res.plan.cpu().numpy(), Pr) < 1e-4
    Ch = (C / cmax).half()
    r16 = ops.sinkhorn(a, a, Ch, 0.1, max_iter=60, stop_thr=0.0)
    assert r16.info()["engine_name"] == "mesh"
    P16, *_ = orc.sinkhorn_knopp(np.full(N, 1.0 / N), np.full(N, 1.0 / N),
                                 Ch.double().cpu().numpy(), 0.1, 60, 0.0)
    assert nrel(r16.plan.cpu().numpy(), P16) < 1e-4
