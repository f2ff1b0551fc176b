"""HIP path vs the oracle and the golden vectors (needs an MI355X).

Tolerances: the north star asks for plans within 1e-4 relative of the reference
CPU path.  "Relative" is normwise: max|P - P_ref| / max|P_ref| (entries of
exp(-M/reg) far below the plan's scale carry no information and exp() amplifies
last-bit cost differences in them).  float64 paths are held to 1e-9..1e-10.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def nrel(x, ref):
    x = np.asarray(x, dtype=np.float64)
    ref = np.asarray(ref, dtype=np.float64)
    return np.abs(x - ref).max() / np.abs(ref).max()


@pytest.fixture(scope="module")
def ops():
    from otfuse import ops as o
    return o


def _t(x, dev, dt=None):
    return torch.as_tensor(np.asarray(x), device=dev, dtype=dt)


# ----------------------------------------------------------------------------- cost
@pytest.mark.parametrize("algo", ["split16", "f32"])
@pytest.mark.parametrize("n,m,d", [(256, 256, 64), (130, 77, 40), (4096, 4096, 512), (1, 5, 3),
                                   (300, 129, 1000), (4100, 3999, 300)])
def test_pairwise_cost_vs_oracle(ops, orc, dev, n, m, d, algo):
    from otfuse.synthetic import paired_embeddings
    X, _, _ = paired_embeddings(n, d, seed=n)
    _, Y, _ = paired_embeddings(m, d, seed=m + 1)
    C, cmax = ops.pairwise_cost(_t(X, dev), _t(Y, dev), algo=algo)
    Cr, mr = orc.pairwise_cost(X, Y)
    assert nrel(C.cpu().numpy(), Cr) < 2e-6
    assert float(cmax) == pytest.approx(mr, rel=1e-5)


def test_split16_wide_dynamic_range(ops, orc, dev):
    """Rows with very different magnitudes and tiny entries (per-row power-of-two scale)."""
    rng = np.random.default_rng(17)
    X = (rng.standard_normal((200, 96)) * np.logspace(-3, 3, 200)[:, None]).astype(np.float32)
    Y = (rng.standard_normal((150, 96)) * np.logspace(2, -2, 150)[:, None]).astype(np.float32)
    X[5, :10] = 1e-7
    C, _ = ops.pairwise_cost(_t(X, dev), _t(Y, dev), algo="split16")
    Cr, _ = orc.pairwise_cost(X, Y)
    # per-element error relative to the entry's own scale |x|^2 + |y|^2
    scale = (X.astype(np.float64) ** 2).sum(1)[:, None] + (Y.astype(np.float64) ** 2).sum(1)[None]
    assert (np.abs(C.cpu().numpy() - Cr) / scale).max() < 1e-6


@pytest.mark.parametrize("n,m,d,in_dt,out_dt,metric", [
    (4096, 4096, 512, torch.float32, torch.float32, "sqeuclidean"),
    (4100, 3999, 300, torch.float32, torch.float32, "euclidean"),
    (8192, 8192, 256, torch.float16, torch.float16, "sqeuclidean"),
    (4096, 4096, 40, torch.float32, torch.float16, "sqeuclidean")])
def test_cost_kernel_forms_match_oracle(ops, orc, dev, n, m, d, in_dt, out_dt, metric):
    """The 256 x 256 cost kernels: the 16x16x32 form for float32 storage (float32 operands
    split in the kernel when the rows are whole aligned stages, the prep's fp16 images
    otherwise) and the 32x32x16 form for fp16 storage -- within the split-fp16 oracle
    tolerance on the first 300 and the last 40 rows, cmax alike."""
    g = torch.Generator(device=dev).manual_seed(n + d + 1)
    X = torch.randn(n, d, device=dev, generator=g).to(in_dt)
    Y = (torch.randn(m, d, device=dev, generator=g) * 0.7 + 0.2).to(in_dt)
    C1, mx1, u1 = ops.pairwise_cost_ex(X, Y, metric=metric, out_dtype=out_dt)
    torch.cuda.synchronize()
    tol = 2e-3 if out_dt == torch.float16 else 2e-6
    assert float(mx1) == float(C1.max())
    rows = torch.cat([torch.arange(0, 300, device=dev), torch.arange(n - 40, n, device=dev)])
    Cr, _ = orc.pairwise_cost(X[rows].double().cpu().numpy(), Y.double().cpu().numpy(), metric=metric)
    got = C1[rows].double().cpu().numpy() * float(u1)
    assert nrel(got, Cr) < tol


@pytest.mark.parametrize("n,m,d,out_dt,metric,same", [
    (4096, 4096, 512, torch.float32, "sqeuclidean", False),
    (4100, 3999, 256, torch.float32, "euclidean", False),
    (3000, 3000, 128, torch.float32, "sqeuclidean", True),
    (8192, 8192, 256, torch.float16, "sqeuclidean", False),
    (4096, 4096, 300, torch.float32, "sqeuclidean", False)])   # d % 64 != 0: image path
def test_cost_f32in_split_in_kernel_is_bit_identical(ops, dev, n, m, d, out_dt, metric, same):
    """The 16x16x32 kernel splitting the float32 operands into hi / lo fp16 in registers
    (rows that are whole 16-B aligned stages) builds the same images as
    split16_prep2_kernel: the same cost bits, cmax and unit as the prep-image path, which
    the same data takes from rows with a leading dimension of d + 1 -- ragged tiles, the
    Euclidean metric, X is Y (zero diagonal) and fp16 storage included."""
    g = torch.Generator(device=dev).manual_seed(n + d + 7)
    X = torch.randn(n, d, device=dev, generator=g) * torch.logspace(-2, 2, n, device=dev)[:, None]
    Y = X if same else (torch.randn(m, d, device=dev, generator=g) * 0.7 + 0.2)

    def padded(T):  # same values, leading dimension d + 1 (not a 16-B multiple)
        buf = torch.zeros((T.shape[0], d + 1), device=dev)
        buf[:, :d] = T
        return buf[:, :d]
    C1, mx1, u1 = ops.pairwise_cost_ex(X, Y, metric=metric, out_dtype=out_dt)
    Xp = padded(X)
    C0, mx0, u0 = ops.pairwise_cost_ex(Xp, Xp if same else padded(Y), metric=metric, out_dtype=out_dt)
    torch.cuda.synchronize()
    assert torch.equal(C0, C1) and torch.equal(mx0, mx1) and torch.equal(u0, u1)


def test_pairwise_cost_euclidean_same_input_zero_diag(ops, orc, dev):
    rng = np.random.default_rng(1)
    X = rng.random((70, 33)).astype(np.float32)
    Xd = _t(X, dev)
    C, _ = ops.pairwise_cost(Xd, metric="euclidean")
    Cr, _ = orc.pairwise_cost(X, X, metric="euclidean", zero_diag=True)
    Cg = C.cpu().numpy()
    assert np.all(np.diag(Cg) == 0)
    assert nrel(Cg, Cr) < 1e-5


def test_pairwise_cost_asymmetric_identity_check(ops, dev):
    """A = I against an asymmetric B catches a transposed C/D write."""
    d = 64
    X = torch.eye(d, device=dev)
    Y = torch.arange(d * d, dtype=torch.float32, device=dev).reshape(d, d) / (d * d)
    C, _ = ops.pairwise_cost(X, Y)
    ref = (X[:, None, :] - Y[None, :, :]).pow(2).sum(-1)
    assert torch.allclose(C, ref, rtol=1e-5, atol=1e-5)


# ----------------------------------------------------------------------------- Sinkhorn POT
def test_f1_sinkhorn_config1_golden(ops, golden, dev):
    f = golden("f1_sinkhorn_256.npz")
    X, Y = _t(f["X"], dev), _t(f["Y"], dev)
    C, cmax = ops.pairwise_cost(X, Y)
    a = torch.full((256,), 1 / 256, device=dev)
    res = ops.sinkhorn(a, a, C, float(f["reg"]), max_iter=int(f["iters"]), stop_thr=0.0,
                       cost_scale=cmax)
    info = res.info()
    assert info["status_name"] == "max_iter" and info["niter"] == 49
    P = res.plan.cpu().numpy()
    idx = f["idx"]
    assert nrel(P[idx[:, 0], idx[:, 1]], f["plan_samples"]) < 1e-4
    assert nrel(P.sum(0), f["plan_colsum"]) < 1e-4
    assert nrel(P.sum(1), f["plan_rowsum"]) < 1e-4


def test_f1_float64_path_is_tight(ops, golden, orc, dev):
    f = golden("f1_sinkhorn_256.npz")
    C, _ = orc.pairwise_cost(f["X"], f["Y"], scale_max=True)
    a = torch.full((256,), 1 / 256, device=dev, dtype=torch.float64)
    res = ops.sinkhorn(a, a, _t(C, dev), 0.1, max_iter=50, stop_thr=0.0)
    u, v = res.u.cpu().numpy(), res.v.cpu().numpy()
    s = np.linalg.norm(u) / np.linalg.norm(f["u"])
    np.testing.assert_allclose(u / s, f["u"], rtol=1e-11)
    np.testing.assert_allclose(v * s, f["v"], rtol=1e-11)


def test_f2_per_batch_feature_coupling_golden(ops, golden, dev):
    from otfuse.pot import feature_coupling_pot_device
    f = golden("f2_feature_pot_b8_d512.npz")
    ts = torch.full((8,), 1 / 8, dtype=torch.float64, device=dev)
    res = feature_coupling_pot_device(_t(f["X"], dev), _t(f["Y"], dev), ts_diag=ts, eps=1e-2)
    info = res.info()
    assert info["n_err"] == int(f["n_err"]) and info["status_name"] == "max_iter"
    np.testing.assert_allclose(info["err"], f["err"], rtol=1e-5)
    P = res.plan.cpu().numpy()
    idx = f["idx"]
    assert nrel(P[idx[:, 0], idx[:, 1]], f["plan_samples"]) < 1e-9
    assert nrel(P.sum(1), f["plan_rowsum"]) < 1e-9


def test_f2_drop_in_numpy_api(golden, dev):
    from otfuse.pot import get_feature_coupling_pot
    f = golden("f2_feature_pot_b8_d512.npz")
    Tv, log = get_feature_coupling_pot(({0: f["X"]}, {0: f["Y"]}), Ts={0: np.eye(8) / 8}, eps=1e-2)
    assert isinstance(Tv, np.ndarray) and Tv.dtype == np.float64 and log == {}
    idx = f["idx"]
    assert nrel(Tv[idx[:, 0], idx[:, 1]], f["plan_samples"]) < 1e-9


def test_f3_numerical_break_golden(ops, golden, dev):
    from otfuse.pot import feature_coupling_pot_device
    f = golden("f3_numerical_break.npz")
    ts = torch.full((8,), 1 / 8, dtype=torch.float64, device=dev)
    res = feature_coupling_pot_device(_t(f["X"], dev), _t(f["Y"], dev), ts_diag=ts, eps=1e-3)
    info = res.info()
    assert info["status_name"] == "numerical_break" and info["break_iter"] == 0
    assert info["last_good"] == -1
    P = res.plan.cpu().numpy()
    assert nrel(P, f["plan"]) < 1e-9
    assert np.array_equal(P == 0, f["plan"] == 0)


def test_f4_blockdiag_nonsquare_golden(golden, dev):
    from otfuse.pot import get_feature_coupling_pot
    f = golden("f4_feature_blockdiag.npz")
    data = ({1: f["X1"], 0: f["X0"]}, {1: f["Y1"], 0: f["Y0"]})   # insertion order != sorted
    Tv, _ = get_feature_coupling_pot(data, Ts={0: f["Ts0"], 1: f["Ts1"]}, eps=float(f["eps"]))
    assert Tv.shape == (64, 48)
    assert nrel(Tv, f["plan"]) < 1e-9


def test_feature_cost_dense_ts_vs_oracle(ops, orc, dev):
    rng = np.random.default_rng(4)
    X = rng.random((20, 70)).astype(np.float32)
    Y = rng.random((13, 50)).astype(np.float32)
    Ts = rng.random((20, 13))
    M = ops.feature_cost(_t(X, dev), _t(Y, dev), Ts=_t(Ts, dev)).cpu().numpy()
    assert nrel(M, orc.feature_cost(X, Y, Ts)) < 1e-13
    Tsq = rng.random((20, 20))
    Y2 = rng.random((20, 50)).astype(np.float32)
    M2 = ops.feature_cost(_t(X, dev), _t(Y2, dev), Ts=_t(Tsq, dev), weights="fot").cpu().numpy()
    assert nrel(M2, orc.feature_cost(X, Y2, Tsq, weights="fot")) < 1e-13


@pytest.mark.parametrize("engine", ["stream", "resident", "tiled", "sweep", "gather", "mesh"])
@pytest.mark.parametrize("n,m,dt", [(300, 200, torch.float32), (64, 4099, torch.float32),
                                    (1024, 512, torch.float64), (2048, 500, torch.float32),
                                    (1000, 8191, torch.float32), (513, 2049, torch.float64),
                                    (3, 7, torch.float64), (1, 1, torch.float32),
                                    (4100, 1000, torch.float32), (1200, 16383, torch.float32),
                                    (700, 8191, torch.float64), (200000, 5, torch.float32)])
def test_sinkhorn_ragged_shapes_vs_oracle(ops, orc, dev, n, m, dt, engine):
    rng = np.random.default_rng(n + m)
    C = rng.random((n, m))
    a = rng.random(n) + 0.5
    a /= a.sum()
    b = rng.random(m) + 0.5
    b /= b.sum()
    P_r, u_r, v_r, info_r = orc.sinkhorn_knopp(a, b, C, 0.1, 60, 0.0)
    try:
        res = ops.sinkhorn(_t(a, dev, dt), _t(b, dev, dt), _t(C, dev, dt), 0.1, max_iter=60,
                           stop_thr=0.0, engine=engine)
    except Exception as e:  # resident / tiled need one row block / tile per CU; tiled is fp32
        if engine in ("resident", "tiled", "sweep", "gather", "mesh") and "unsupported" in str(e):
            pytest.skip(f"problem does not fit the {engine} engine")
        raise
    tol = 1e-4 if dt == torch.float32 else 1e-10
    assert nrel(res.plan.cpu().numpy(), P_r) < tol
    info = res.info()
    assert info["niter"] == info_r["niter"]
    assert info["engine_name"] == engine
    np.testing.assert_allclose(res.u.cpu().numpy() * res.v.cpu().numpy().mean(),
                               u_r * v_r.mean(), rtol=tol * 10)


@pytest.mark.parametrize("engine", ["stream", "resident", "tiled", "sweep", "gather", "mesh"])
def test_float32_stop_and_break_all_engines(ops, orc, dev, engine):
    """float32 inputs: the convergence stop lands on the oracle's check (every 10) and a
    zero column of K (K^T u = 0 at iteration 0) reverts to (u0, v0) in every engine."""
    rng = np.random.default_rng(22)
    n, m = 700, 300
    C = rng.random((n, m)).astype(np.float32)
    a = np.full(n, 1.0 / n)
    b = np.full(m, 1.0 / m)
    P_r, *_, info_r = orc.sinkhorn_knopp(a, b, C.astype(np.float64), 0.05, 2000, 1e-5)
    assert info_r["niter"] < 1999
    res = ops.sinkhorn(_t(a, dev, torch.float32), _t(b, dev, torch.float32), _t(C, dev), 0.05,
                       max_iter=2000, stop_thr=1e-5, engine=engine)
    info = res.info()
    assert info["engine_name"] == engine
    assert info["status_name"] == "converged"
    assert abs(info["niter"] - info_r["niter"]) <= 10   # float32 error vs float64 at a check
    assert nrel(res.plan.cpu().numpy(), P_r) < 1e-3
    # a column of cost 1e3 at reg 1: exp(-1000) = 0 in float32 and float64
    C2 = rng.random((n, m)).astype(np.float32)
    C2[:, 17] = 1e3
    P2, *_, info2 = orc.sinkhorn_knopp(a, b, C2.astype(np.float64), 1.0, 100, 0.0)
    assert info2["break_iter"] == 0
    res = ops.sinkhorn(_t(a, dev, torch.float32), _t(b, dev, torch.float32), _t(C2, dev), 1.0,
                       max_iter=100, stop_thr=0.0, engine=engine)
    info = res.info()
    assert info["status_name"] == "numerical_break" and info["break_iter"] == 0
    assert info["niter"] == info2["niter"]
    assert nrel(res.plan.cpu().numpy(), P2) < 1e-5
    # a ROW of cost 1e3: K v = 0 there, u = inf at iteration 0 (the non-finite-u path:
    # the sweep engine's granule flags, the mesh engine's hop-A tags)
    C3 = rng.random((n, m)).astype(np.float32)
    C3[41, :] = 1e3
    P3, *_, info3 = orc.sinkhorn_knopp(a, b, C3.astype(np.float64), 1.0, 100, 0.0)
    assert info3["break_iter"] == 0
    res = ops.sinkhorn(_t(a, dev, torch.float32), _t(b, dev, torch.float32), _t(C3, dev), 1.0,
                       max_iter=100, stop_thr=0.0, engine=engine)
    info = res.info()
    assert info["status_name"] == "numerical_break" and info["break_iter"] == info3["break_iter"]
    assert info["niter"] == info3["niter"] and info["last_good"] == -1
    assert nrel(res.plan.cpu().numpy(), P3) < 1e-5


@pytest.mark.parametrize("engine", ["stream", "resident", "sweep", "gather"])   # float64 (tiled: fp32 test above)
def test_engines_agree_on_early_stop_and_break(ops, orc, golden, dev, engine):
    """Convergence stop and the numerical break behave identically in both engines."""
    rng = np.random.default_rng(21)
    C = rng.random((500, 300))
    a = np.ones(500) / 500
    b = np.ones(300) / 300
    P_r, *_, info_r = orc.sinkhorn_knopp(a, b, C, 0.05, 2000, 1e-9)
    res = ops.sinkhorn(_t(a, dev), _t(b, dev), _t(C, dev), 0.05, max_iter=2000, stop_thr=1e-9,
                       engine=engine, sync_every=25)
    info = res.info()
    assert info["status_name"] == "converged" and info["niter"] == info_r["niter"]
    np.testing.assert_allclose(info["err"], info_r["err"], rtol=1e-6, atol=1e-15)
    assert nrel(res.plan.cpu().numpy(), P_r) < 1e-10
    f = golden("f3_numerical_break.npz")
    M = orc.feature_cost(f["X"], f["Y"], np.eye(8) / 8)
    d = M.shape[0]
    u = torch.full((d,), 1.0 / d, dtype=torch.float64, device=dev)
    res = ops.sinkhorn(u, u, _t(M, dev), 1e-3, max_iter=2000, stop_thr=1e-9, engine=engine)
    info = res.info()
    assert info["status_name"] == "numerical_break" and info["break_iter"] == 0
    assert nrel(res.plan.cpu().numpy(), f["plan"]) < 1e-9


def test_converged_mode_stops_at_same_iteration(ops, orc, dev):
    rng = np.random.default_rng(8)
    C = rng.random((200, 150))
    a = np.ones(200) / 200
    b = np.ones(150) / 150
    P_r, *_, info_r = orc.sinkhorn_knopp(a, b, C, 0.05, 2000, 1e-9)
    res = ops.sinkhorn(_t(a, dev), _t(b, dev), _t(C, dev), 0.05, max_iter=2000, stop_thr=1e-9,
                       sync_every=20)
    info = res.info()
    assert info["status_name"] == "converged"
    assert info["niter"] == info_r["niter"]
    np.testing.assert_allclose(info["err"], info_r["err"], rtol=1e-6, atol=1e-15)
    assert nrel(res.plan.cpu().numpy(), P_r) < 1e-10


def test_vendored_squared_error_mode(ops, orc, dev):
    rng = np.random.default_rng(9)
    C = rng.random((64, 64))
    a = np.ones(64) / 64
    _, _, _, info_r = orc.sinkhorn_knopp(a, a, C, 0.05, 2000, 1e-12, err_squared=True)
    res = ops.sinkhorn(_t(a, dev), _t(a, dev), _t(C, dev), 0.05, max_iter=2000, stop_thr=1e-12,
                       err_squared=True)
    assert res.info()["niter"] == info_r["niter"]


# ----------------------------------------------------------------------------- full size
def test_metric_config_full_size_properties(ops, orc, dev):
    """BASELINE metric config at full size: N = 4096, d = 512, eps = 0.1, 100 iterations,
    against the float64 oracle (a few seconds on the host) and marginal properties."""
    from otfuse.synthetic import paired_embeddings
    N, d = 4096, 512
    X, Y, _ = paired_embeddings(N, d, seed=1234)
    C, cmax = ops.pairwise_cost(_t(X, dev), _t(Y, dev))
    a = torch.full((N,), 1.0 / N, device=dev)
    res = ops.sinkhorn(a, a, C, 0.1, max_iter=100, stop_thr=0.0, cost_scale=cmax)
    P = res.plan.cpu().numpy().astype(np.float64)
    # row marginals are exact after a u-update; column marginals carry the residual
    np.testing.assert_allclose(P.sum(1), 1.0 / N, rtol=1e-4)
    Cr, _ = orc.pairwise_cost(X, Y, scale_max=True)
    Pr, *_ = orc.sinkhorn_knopp(np.full(N, 1.0 / N), np.full(N, 1.0 / N), Cr, 0.1, 100, 0.0)
    assert nrel(P, Pr) < 1e-4
    assert np.linalg.norm(P - Pr) / np.linalg.norm(Pr) < 1e-4


# ----------------------------------------------------------------------------- OTT flavour
def test_ott_flavour_vs_log_restatement(ops, orc, dev):
    """OTT lse-mode semantics (parity unpinned: OTT absent); vs the oracle restatement."""
    rng = np.random.default_rng(12)
    C = rng.random((150, 120))
    a = np.ones(150) / 150
    b = np.ones(120) / 120
    P_r, f_r, g_r, info_r = orc.sinkhorn_log(a, b, C, 5e-3, max_iter=2000, threshold=1e-3,
                                             cscale=1.0 / C.max())
    M = _t(C, dev, torch.float64)
    from otfuse.perturbot import solve_ott
    res, _ = solve_ott(M, 5e-3)
    info = res.info()
    assert info["niter"] + 1 == info_r["n_iters"]
    assert nrel(res.plan.cpu().numpy(), P_r) < 1e-9
    assert abs(res.plan.sum().item() - 1.0) < 1e-6


def test_get_coupling_fot_blockdiag(golden, dev):
    from otfuse.perturbot import get_coupling_fot
    f = golden("f4_feature_blockdiag.npz")
    xd = {0: f["X0"][:12], 1: f["X1"][:12]}
    yd = {0: f["Y0"][:12], 1: f["Y1"][:12]}
    rng = np.random.default_rng(2)
    ts = {k: rng.random((12, 12)) for k in (0, 1)}
    Tv, log = get_coupling_fot((xd, yd), ts, eps=5e-3)
    assert Tv.shape == (64, 48) and len(log["cost"]) == 2
    # OTT: rows exact after the f-update; stop rule = L1 column-marginal error < 1e-3
    np.testing.assert_allclose(Tv.sum(1), 1 / 64, rtol=1e-6)
    assert np.abs(Tv.sum(0) - 1 / 48).sum() < 1e-3


# ----------------------------------------------------------------------------- plan use
def test_plan_postprocess_and_apply_golden(ops, golden, dev):
    from otfuse.fusion import ot_alignment_loss
    f = golden("f2_feature_pot_b8_d512.npz")
    X = _t(f["X"], dev).requires_grad_(True)
    Y = _t(f["Y"], dev).requires_grad_(True)
    loss, ot_mri, T = ot_alignment_loss(X, Y, eps=1e-2)
    idx = f["idx"]
    Tc = T.cpu().numpy()
    np.testing.assert_allclose(Tc[idx[:, 0], idx[:, 1]], f["Tn_samples"], rtol=1e-5, atol=1e-12)
    np.testing.assert_allclose(ot_mri.detach().cpu().numpy(), f["ot_mri_from_pet"], rtol=1e-5,
                               atol=1e-6)
    assert abs(float(loss) - float(f["ot_loss"])) < 1e-5
    loss.backward()
    # gradient through the HIP plan-apply matches torch's matmul
    Y2 = _t(f["Y"], dev).requires_grad_(True)
    from otfuse.fusion import cosine_loss
    cosine_loss(X.detach(), Y2 @ T.t()).backward()
    assert torch.allclose(Y.grad, Y2.grad, rtol=1e-4, atol=1e-7)


def test_plan_postprocess_nan_and_zero_rows(ops, dev):
    T = torch.rand(5, 7, dtype=torch.float64, device=dev)
    T[1, 3] = float("nan")
    T[2] = 0
    Tn = ops.plan_postprocess(T).cpu()
    Tr = T.cpu().float()
    Tr = torch.where(torch.isnan(Tr), torch.full_like(Tr, 1e-8), Tr)
    rs = Tr.sum(1, keepdim=True)
    rs = torch.where(rs == 0, torch.full_like(rs, 1e-8), rs)
    assert torch.allclose(Tn, Tr / rs, rtol=1e-6, atol=0)


def test_smoke_entry_point_runs(dev):
    import __graft_entry__ as g
    g.smoke()


@pytest.mark.parametrize("n,m,d,in_dt,metric,same", [
    (4096, 4096, 512, torch.float32, "sqeuclidean", False),
    (4000, 3900, 256, torch.float32, "euclidean", False),
    (3000, 3000, 128, torch.float32, "sqeuclidean", True),
    (4096, 4096, 300, torch.float32, "sqeuclidean", False),
    (4096, 4096, 40, torch.float32, "sqeuclidean", False),
    (4096, 4096, 512, torch.float16, "sqeuclidean", False),
    (4096, 4096, 48, torch.float16, "sqeuclidean", False),    # one 64-deep K-tile
    (4000, 3900, 192, torch.float16, "euclidean", False)])
def test_cost_8ph_kernel_is_bit_identical_to_register_staged(ops, dev, monkeypatch, n, m, d, in_dt, metric, same):
    """The 8-phase LDS-DMA cost kernel (cost_8ph_kernel, the default) gives every 16 x 16
    block cost_big16_kernel's MFMA sequence (split-fp16: hi.lo, lo.hi, hi.hi per 32-deep
    step; fp16 operands: one MFMA per 32-deep step, in k order) and its epilogue: float32
    costs, cmax and unit bitwise those of the register-staged kernel (OTF_COST_8PH=0) --
    ragged tiles, one or two K-tiles (d = 48 fp16, d = 40 split), d not a multiple of 64, X is Y (zero
    diagonal), the Euclidean metric, fp16 operands."""
    g = torch.Generator(device=dev).manual_seed(n + d + 11)
    X = (torch.randn(n, d, device=dev, generator=g) * torch.logspace(-1, 1, n, device=dev)[:, None]).to(in_dt)
    Y = X if same else (torch.randn(m, d, device=dev, generator=g) * 0.7 + 0.2).to(in_dt)
    C1, mx1, u1 = ops.pairwise_cost_ex(X, Y, metric=metric, out_dtype=torch.float32)
    monkeypatch.setenv("OTF_COST_8PH", "0")
    C0, mx0, u0 = ops.pairwise_cost_ex(X, Y, metric=metric, out_dtype=torch.float32)
    torch.cuda.synchronize()
    assert torch.equal(C0, C1) and torch.equal(mx0, mx1) and torch.equal(u0, u1)


@pytest.mark.parametrize("n,m,d,in_dt", [(8192, 8192, 1024, torch.float16), (4000, 3900, 256, torch.float32)])
def test_cost_8ph_fp16_storage_vs_register_staged_and_oracle(ops, orc, dev, monkeypatch, n, m, d, in_dt):
    """fp16 cost storage (config 5's form): the 8-phase kernel on 16x16x32 MFMAs against the
    32x32x16 register-staged kernel (OTF_COST_8PH=0; a different accumulation order, so
    within fp16 rounding: 1 ulp of the scaled cost) and the oracle on sampled rows; the same
    store scale (unit) and a cmax within one fp16 ulp."""
    g = torch.Generator(device=dev).manual_seed(n + d + 13)
    X = torch.randn(n, d, device=dev, generator=g).to(in_dt)
    Y = (torch.randn(m, d, device=dev, generator=g) * 0.7 + 0.2).to(in_dt)
    C1, mx1, u1 = ops.pairwise_cost_ex(X, Y, out_dtype=torch.float16)
    monkeypatch.setenv("OTF_COST_8PH", "0")
    C0, mx0, u0 = ops.pairwise_cost_ex(X, Y, out_dtype=torch.float16)
    torch.cuda.synchronize()
    assert torch.equal(u0, u1)
    diff = (C1.float() - C0.float()).abs()
    assert float((diff / C0.float().abs().clamp_min(2.0 ** -14)).max()) <= 2.0 ** -10
    assert abs(float(mx1) - float(mx0)) <= float(mx0) * 2.0 ** -10
    rows = torch.cat([torch.arange(0, 200, device=dev), torch.arange(n - 40, n, device=dev)])
    Cr, _ = orc.pairwise_cost(X[rows].double().cpu().numpy(), Y.double().cpu().numpy())
    assert nrel(C1[rows].double().cpu().numpy() * float(u1), Cr) < 2e-3


@pytest.mark.parametrize("n,m,d,in_dt", [(4096, 4096, 512, torch.float32), (4000, 3900, 192, torch.float16),
                                         (8192, 8192, 1024, torch.float16)])
def test_cost_8ph_kernel_race_screen_under_uneven_load(ops, dev, n, m, d, in_dt):
    """Race screen of the 8-phase kernel's DMA / barrier schedule (a misplaced read passes a
    single check whenever the DMA happens to land first): 24 launches, half of them beside a
    memory-bound copy stream and a GEMM on two other streams (uneven load), every result
    bitwise equal to the first launch alone."""
    g = torch.Generator(device=dev).manual_seed(n + d + 17)
    X = torch.randn(n, d, device=dev, generator=g).to(in_dt)
    Y = (torch.randn(m, d, device=dev, generator=g) * 0.7 + 0.2).to(in_dt)
    ref, mref, _ = ops.pairwise_cost_ex(X, Y, out_dtype=torch.float32)
    torch.cuda.synchronize()
    big = torch.empty(64 << 20, device=dev)
    dst = torch.empty_like(big)
    A = torch.randn(4096, 4096, device=dev)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    bad = 0
    for k in range(24):
        if k % 2:
            with torch.cuda.stream(s1):
                for _ in range(3):
                    dst.copy_(big)
            with torch.cuda.stream(s2):
                A @ A
        C, mx, _ = ops.pairwise_cost_ex(X, Y, out_dtype=torch.float32)
        torch.cuda.synchronize()
        bad += int(not (torch.equal(C, ref) and torch.equal(mx, mref)))
    assert bad == 0
