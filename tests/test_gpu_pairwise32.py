"""Fused pairwise cost + float32 Sinkhorn (otf_sinkhorn_pairwise_f32,
``ops.sinkhorn_pairwise(precision="fp32")``): the reference's ``M = euclidean_distances(X, Y,
squared=True); M /= M.max(); ot.sinkhorn(a, b, M, reg)`` (MRI_PET_OT_nojax.py:70-75, :143) in
float32 compute, with every workgroup of the float32 mesh building its 128 x 512 cost tile from
the split-fp16 images in its prologue.  Checked against the two calls it replaces
(``pairwise_cost`` + ``sinkhorn``: bitwise where the two-call cost runs the same 16x16x32
kernel, at the metric shape) and against the float64 oracle at the float32 path's 1e-4
(needs an MI355X).  The fused launch runs on request (engine="mesh"); AUTO runs the two calls,
measured faster at the metric shape."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

TOL32 = 1e-4  # normwise relative plan tolerance of the float32 paths against the float64 oracle


def nrel(x, ref):
    x = np.asarray(x, dtype=np.float64)
    ref = np.asarray(ref, dtype=np.float64)
    return np.abs(x - ref).max() / np.abs(ref).max()


def _emb(n, m, d, seed):
    rng = np.random.default_rng(seed)
    X = rng.standard_normal((n, d)).astype(np.float32)
    Y = (0.7 * X[np.arange(m) % n] + 0.5 * rng.standard_normal((m, d))).astype(np.float32)
    return X, Y


def _oracle(orc, X, Y, reg, iters, metric="sqeuclidean", stop=0.0, a=None, b=None):
    C, mx = orc.pairwise_cost(X, Y, metric=metric)
    n, m = C.shape
    a = np.full(n, 1.0 / n) if a is None else a
    b = np.full(m, 1.0 / m) if b is None else b
    P, u, v, info = orc.sinkhorn_knopp(a, b, C, reg, iters, stop, cscale=1.0 / mx)
    return P, info, mx


def _two_calls(X, Y, reg, iters, metric="sqeuclidean", engine="auto"):
    from otfuse import ops
    C, cmax = ops.pairwise_cost(X, Y, metric)
    n, m = C.shape
    a = torch.full((n,), 1.0 / n, device=X.device)
    b = torch.full((m,), 1.0 / m, device=X.device)
    return ops.sinkhorn(a, b, C, reg, max_iter=iters, stop_thr=0.0, cost_scale=cmax, engine=engine), cmax


def test_pairwise32_metric_shape_bitwise_two_calls(dev):
    """The float32 leg's shape (N = 4096, d = 512, eps 0.1, 100 iterations, the bench's inputs):
    the fused launch (engine="mesh") gives cost max, plan and scalings bitwise those of
    pairwise_cost + sinkhorn (the same 16x16x32 MFMA sequence per cost block, the same
    epilogue, the same K, the same mesh loop); two runs are bitwise equal; AUTO runs the two
    calls (measured faster), the same bits again."""
    from otfuse import ops
    from otfuse.synthetic import paired_embeddings
    Xn, Yn, _ = paired_embeddings(4096, 512, seed=1234)
    X, Y = torch.from_numpy(Xn).to(dev), torch.from_numpy(Yn).to(dev)
    r1 = ops.sinkhorn_pairwise(X, Y, 0.1, max_iter=100, stop_thr=0.0, precision="fp32", engine="mesh")
    r2 = ops.sinkhorn_pairwise(X, Y, 0.1, max_iter=100, stop_thr=0.0, precision="fp32", engine="mesh")
    ra = ops.sinkhorn_pairwise(X, Y, 0.1, max_iter=100, stop_thr=0.0, precision="fp32")
    ru, cmax = _two_calls(X, Y, 0.1, 100)
    i1 = r1.info()
    assert i1["engine_name"] == "mesh" and i1["fallback"] == 0 and i1["status_name"] == "max_iter"
    assert ru.info()["engine_name"] == "mesh"
    assert r1.plan.dtype == torch.float32 and r1.u.dtype == torch.float32
    assert torch.equal(r1.cost_max, cmax)
    assert torch.equal(r1.plan, ru.plan) and torch.equal(r1.u, ru.u) and torch.equal(r1.v, ru.v)
    assert torch.equal(r1.plan, r2.plan) and torch.equal(r1.u, r2.u)
    assert torch.equal(ra.plan, r1.plan) and torch.equal(ra.v, r1.v)


@pytest.mark.parametrize("reg", [0.1, 0.05])
def test_pairwise32_metric_shape_vs_oracle(orc, dev, reg):
    """The fused float32 step at the metric shape within 1e-4 of the float64 oracle (cost +
    POT sinkhorn_knopp) with its iteration count, at the bench's eps and at 0.05."""
    from otfuse import ops
    from otfuse.synthetic import paired_embeddings
    Xn, Yn, _ = paired_embeddings(4096, 512, seed=1234)
    P_r, info_r, mx = _oracle(orc, Xn, Yn, reg, 100)
    res = ops.sinkhorn_pairwise(torch.from_numpy(Xn).to(dev), torch.from_numpy(Yn).to(dev), reg, max_iter=100,
                                stop_thr=0.0, precision="fp32", engine="mesh")
    info = res.info()
    assert info["engine_name"] == "mesh" and info["niter"] == info_r["niter"]
    assert abs(float(res.cost_max) - mx) / mx < 1e-6
    assert nrel(res.plan.cpu().numpy(), P_r) < TOL32


@pytest.mark.parametrize("n,m,d", [(512, 512, 64), (1024, 2048, 128), (2048, 4096, 256), (512, 1024, 48),
                                   (1536, 512, 96)])
def test_pairwise32_fused_shapes(orc, dev, n, m, d):
    """4 / 8 / 16 / 12 row blocks x 1 / 2 / 4 / 8 column tiles, d not a multiple of the 64-deep
    image padding (48, 96): the fused launch (engine="mesh") against the float64 oracle at 1e-4
    and against the two calls to float32 rounding (their cost kernel may tile differently)."""
    from otfuse import ops
    X, Y = _emb(n, m, d, n + m + d)
    P_r, info_r, mx = _oracle(orc, X, Y, 0.05, 40)
    Xd, Yd = torch.from_numpy(X).to(dev), torch.from_numpy(Y).to(dev)
    res = ops.sinkhorn_pairwise(Xd, Yd, 0.05, max_iter=40, stop_thr=0.0, engine="mesh", precision="fp32")
    info = res.info()
    assert info["engine_name"] == "mesh" and info["status_name"] == "max_iter" and info["fallback"] == 0
    assert info["niter"] == info_r["niter"]
    assert abs(float(res.cost_max) - mx) / mx < 1e-6
    assert nrel(res.plan.cpu().numpy(), P_r) < TOL32
    ru, _ = _two_calls(Xd, Yd, 0.05, 40, engine="mesh")
    assert nrel(res.plan.cpu().numpy(), ru.plan.cpu().numpy()) < 1e-5


def test_pairwise32_euclidean_and_converged_stop(orc, dev):
    """The euclidean metric, POT's converged stop (error every 10 iterations)."""
    from otfuse import ops
    X, Y = _emb(1024, 1024, 64, 5)
    P_r, info_r, mx = _oracle(orc, X, Y, 0.05, 2000, metric="euclidean", stop=1e-5)
    res = ops.sinkhorn_pairwise(torch.from_numpy(X).to(dev), torch.from_numpy(Y).to(dev), 0.05,
                                metric="euclidean", max_iter=2000, stop_thr=1e-5, precision="fp32",
                                engine="mesh")
    info = res.info()
    assert info["engine_name"] == "mesh" and info["status_name"] == "converged"
    assert info["niter"] == info_r["niter"]
    assert abs(float(res.cost_max) - mx) / mx < 1e-6
    assert nrel(res.plan.cpu().numpy(), P_r) < TOL32


@pytest.mark.parametrize("reg", [5e-3, 0.01])
def test_pairwise32_shifted_eps_takes_two_calls(orc, dev, reg):
    """Below reg = 1/64 the float32 solve needs the shifted kernel (a pass over C): the two
    calls run it, within 1e-4 of the oracle at the reference's per-epoch eps."""
    from otfuse import ops
    X, Y = _emb(2048, 2048, 128, 17)
    P_r, info_r, mx = _oracle(orc, X, Y, reg, 60)
    res = ops.sinkhorn_pairwise(torch.from_numpy(X).to(dev), torch.from_numpy(Y).to(dev), reg, max_iter=60,
                                stop_thr=0.0, precision="fp32")
    assert res.shifted and res.info()["niter"] == info_r["niter"]
    assert nrel(res.plan.cpu().numpy(), P_r) < TOL32


@pytest.mark.parametrize("n,m,d", [(1000, 700, 50), (256, 1024, 64)])
def test_pairwise32_unfused_shapes(orc, dev, n, m, d):
    """Shapes the fused launch does not take (ragged tiles, fewer than 4 row blocks): the two
    calls, same results."""
    from otfuse import ops
    X, Y = _emb(n, m, d, 5 * n + m)
    P_r, info_r, mx = _oracle(orc, X, Y, 0.05, 40)
    res = ops.sinkhorn_pairwise(torch.from_numpy(X).to(dev), torch.from_numpy(Y).to(dev), 0.05, max_iter=40,
                                stop_thr=0.0, precision="fp32")
    assert res.info()["niter"] == info_r["niter"]
    assert nrel(res.plan.cpu().numpy(), P_r) < TOL32


def test_pairwise32_forced_fallback_vs_oracle(orc, dev, monkeypatch):
    """A registration give-up (forced, OTF_FORCE_REG_GIVEUP=1) hands the fused float32 solve to
    the relay fallback: it builds the float32 cost (on the float64 matrix cores, from the prep's
    norms), K over it and the streaming passes -- within 1e-4 of the oracle, info fallback = 1."""
    from otfuse import ops
    X, Y = _emb(2048, 2048, 128, 23)
    P_r, info_r, mx = _oracle(orc, X, Y, 0.05, 40)
    monkeypatch.setenv("OTF_FORCE_REG_GIVEUP", "1")
    res = ops.sinkhorn_pairwise(torch.from_numpy(X).to(dev), torch.from_numpy(Y).to(dev), 0.05, max_iter=40,
                                stop_thr=0.0, precision="fp32", engine="mesh")
    info = res.info()
    assert info["fallback"] == 1 and info["engine_name"] == "stream" and info["stalled"] == 0
    assert info["status_name"] == "max_iter" and info["niter"] == info_r["niter"]
    assert abs(float(res.cost_max) - mx) / mx < 1e-6
    assert nrel(res.plan.cpu().numpy(), P_r) < TOL32
