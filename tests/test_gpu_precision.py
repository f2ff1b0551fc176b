"""Precision coverage at the metric shape (N = 4096, d = 512, 100
iterations, max-normalised sq-Euclid cost) over the eps sweep {0.05, 0.01} and the
reference's per-epoch eps 5e-3 (MRI_PET_OT_nojax.py:94), where POT's float64
kernel-domain Sinkhorn (MRI_PET_OT_nojax.py:143 -> sinkhorn_knopp) runs on but a plain
float32 one does not: at eps = 0.01 float32 exp flushes the entries of K below 2^-126
(moving the plan by 2.2e-3 normwise), at 5e-3 whole columns of K vanish (a break at
iteration 0).  The float32 path therefore switches to the shifted kernel
K~ = 2^(C ks + A_i + B_j) (include/otfuse.h opts.shift) -- the same POT iterates --
below reg = 1/64, and holds the north star's 1e-4 at every eps here.  The oracle is the
float64 C restatement (pinned on the golden vectors, tests/test_oracle_golden.py)."""
import warnings

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

N, D = 4096, 512
TOL32 = 1e-4     # the north star's plan tolerance (normwise relative) for float32 compute


def nrel(x, ref):
    x = np.asarray(x, dtype=np.float64)
    ref = np.asarray(ref, dtype=np.float64)
    return np.abs(x - ref).max() / np.abs(ref).max()


@pytest.fixture(scope="module")
def metric_inputs(orc, dev):
    from otfuse import ops
    from otfuse.synthetic import paired_embeddings
    X, Y, _ = paired_embeddings(N, D, seed=1234)
    Xd = torch.as_tensor(X, device=dev)
    Yd = torch.as_tensor(Y, device=dev)
    C, cmax = ops.pairwise_cost(Xd, Yd)
    Cr, _ = orc.pairwise_cost(X, Y, scale_max=True)
    return X, Y, C, cmax, Cr


@pytest.fixture(scope="module")
def oracle_plans(orc, metric_inputs):
    cache = {}

    def get(eps):
        if eps not in cache:
            Cr = metric_inputs[4]
            cache[eps] = orc.sinkhorn_knopp(np.full(N, 1.0 / N), np.full(N, 1.0 / N), Cr, eps, 100, 0.0)
        return cache[eps]
    return get


@pytest.mark.parametrize("eps", [0.05, 0.01, 5e-3])
def test_metric_shape_float32_vs_float64_oracle(dev, metric_inputs, oracle_plans, eps):
    """The headline float32 path (split-fp16 cost, AUTO engine = mesh) against the float64
    oracle at 1e-4 for every eps of the sweep: plain kernel at 0.05, the shifted kernel
    (chosen automatically below reg = 1/64) at 0.01 and 5e-3 -- no float64 detour."""
    from otfuse import ops
    X, Y, C, cmax, Cr = metric_inputs
    a = torch.full((N,), 1.0 / N, device=dev)
    res = ops.sinkhorn(a, a, C, eps, max_iter=100, stop_thr=0.0, cost_scale=cmax)
    info = res.info()
    assert info["status_name"] == "max_iter" and info["niter"] == 99
    assert info["engine_name"] == "mesh" and res.u.dtype == torch.float32
    assert res.shifted == (eps < 1.0 / 64)
    Pr, _, _, info_r = oracle_plans(eps)
    assert info_r["break_iter"] == -1
    assert nrel(res.plan.cpu().numpy(), Pr) < TOL32
    # the marginal-error log: same checks as POT's, values to float32 accuracy
    assert info["n_err"] == len(info_r["err"])
    np.testing.assert_allclose(info["err"], info_r["err"], rtol=2e-3, atol=1e-9)


@pytest.mark.parametrize("eps", [0.04, 0.03, 0.02, 0.016, 0.0155])
def test_shift_threshold_metric_shape_vs_oracle(dev, metric_inputs, oracle_plans, eps):
    """Around the shift threshold (ops.SHIFT_RANGE = 64: max(C / cmax) / reg, i.e.
    reg = 1/64 = 0.015625 on a max-normalised cost): the plain float32 kernel at reg = 0.04,
    0.03, 0.02 and 0.016 (ratios 25 ... 62.5) and the shifted one just below 1/64
    (0.0155, ratio 64.5) -- all within the north star's 1e-4 of the float64 oracle with
    the oracle's error log."""
    from otfuse import ops
    X, Y, C, cmax, Cr = metric_inputs
    a = torch.full((N,), 1.0 / N, device=dev)
    res = ops.sinkhorn(a, a, C, eps, max_iter=100, stop_thr=0.0, cost_scale=cmax)
    info = res.info()
    assert info["engine_name"] == "mesh" and info["niter"] == 99
    assert res.shifted == (1.0 / eps > ops.SHIFT_RANGE)
    Pr, _, _, info_r = oracle_plans(eps)
    assert info_r["break_iter"] == -1
    assert nrel(res.plan.cpu().numpy(), Pr) < TOL32
    assert info["n_err"] == len(info_r["err"])
    np.testing.assert_allclose(info["err"], info_r["err"], rtol=2e-3, atol=1e-9)


def test_cost_scale_not_the_max_is_measured(dev, metric_inputs, oracle_plans):
    """A cost_scale that is not max(C) (here max / 2, an untagged tensor): the shift
    decision measures max(C / cost_scale) / reg (= 2 / 0.02 = 100 > 64, shifted) instead of
    assuming 1 / reg (= 50, plain), and the plan matches the oracle on C / (max / 2) =
    2 * Cr at reg 0.02, i.e. Cr at reg 0.01."""
    from otfuse import ops
    X, Y, C, cmax, Cr = metric_inputs
    half = cmax.clone() * 0.5
    assert ops.is_cost_max(cmax) and not ops.is_cost_max(half)
    a = torch.full((N,), 1.0 / N, device=dev)
    res = ops.sinkhorn(a, a, C, 0.02, max_iter=100, stop_thr=0.0, cost_scale=half)
    assert res.shifted and res.info()["niter"] == 99
    Pr, *_ = oracle_plans(0.01)
    assert nrel(res.plan.cpu().numpy(), Pr) < TOL32


def test_precision_auto_promotes_when_the_shift_cannot_apply(orc, dev, metric_inputs, oracle_plans):
    """precision='auto' on a float32 cost: float32 with the shifted kernel where it applies
    (reg = 0.01), float64 where float32 kernel-domain POT would lose the plan and the shift
    cannot run -- with shift=False at reg = 0.01, and past SHIFT_RANGE_F64 (reg = 1e-3,
    ratio 1000), where POT's own float64 K has exact zeros: there the float64 solve takes
    POT's decision (the oracle's status and iteration count)."""
    from otfuse import ops
    X, Y, C, cmax, Cr = metric_inputs
    a = torch.full((N,), 1.0 / N, device=dev)
    Pr, *_ = oracle_plans(0.01)
    r = ops.sinkhorn(a, a, C, 0.01, max_iter=100, stop_thr=0.0, cost_scale=cmax, precision="auto")
    assert r.shifted and r.u.dtype == torch.float32
    assert nrel(r.plan.cpu().numpy(), Pr) < TOL32
    r = ops.sinkhorn(a, a, C, 0.01, max_iter=100, stop_thr=0.0, cost_scale=cmax, precision="auto",
                     shift=False)
    assert r.u.dtype == torch.float64 and not r.shifted and r.info()["niter"] == 99
    assert nrel(r.plan.cpu().numpy(), Pr) < TOL32
    r = ops.sinkhorn(a, a, C, 1e-3, max_iter=100, stop_thr=0.0, cost_scale=cmax, precision="auto")
    assert r.u.dtype == torch.float64 and not r.shifted
    # the device scales in float64 (C * (-1 / (reg cmax))): the same float64 quotient here
    Cs = C.double().cpu().numpy() / float(cmax)
    Pr3, _, _, ir = orc.sinkhorn_knopp(np.full(N, 1.0 / N), np.full(N, 1.0 / N), Cs, 1e-3, 100, 0.0)
    i = r.info()
    assert (i["niter"], i["break_iter"]) == (ir["niter"], ir["break_iter"])
    assert nrel(r.plan.cpu().numpy(), Pr3) < 1e-9
    # an explicit shift=True on an engine without the shifted kernel (tiled; a 1024^2 block
    # of the metric cost, so that the float64 tiles fit the CUs): promoted to float64 like
    # shift=None, not rejected (the shift is a float32 form)
    Cb = C[:1024, :1024].contiguous()
    ab = torch.full((1024,), 1.0 / 1024, device=dev)
    r = ops.sinkhorn(ab, ab, Cb, 0.01, max_iter=100, stop_thr=0.0, cost_scale=cmax, precision="auto",
                     shift=True, engine="tiled")
    assert r.u.dtype == torch.float64 and not r.shifted and r.info()["engine_name"] == "tiled"
    u1 = np.full(1024, 1.0 / 1024)
    Prb, *_ = orc.sinkhorn_knopp(u1, u1, Cb.double().cpu().numpy() / float(cmax), 0.01, 100, 0.0)
    assert nrel(r.plan.cpu().numpy(), Prb) < 1e-9


def test_pot_sinkhorn_log_returns_pot_scalings_when_shifted(dev, metric_inputs, oracle_plans):
    """ot.sinkhorn drop-in (otfuse.pot.sinkhorn) with log=True on a max-normalised float32
    cost at reg = 0.01, where ops.sinkhorn takes the shifted kernel: log['u'], log['v'] are
    POT's scalings (2^A u~, 2^B v~, float64), equal to the oracle's up to POT's scale mode."""
    from otfuse import pot
    X, Y, C, cmax, Cr = metric_inputs
    M = C / cmax
    a = torch.full((N,), 1.0 / N, device=dev)
    P, log = pot.sinkhorn(a, a, M, 0.01, numItermax=100, stopThr=0.0, log=True)
    Pr, ur, vr, _ = oracle_plans(0.01)
    assert nrel(P.cpu().numpy(), Pr) < TOL32
    u, v = log["u"].cpu().numpy(), log["v"].cpu().numpy()
    assert log["u"].dtype == torch.float64
    c = np.median(u / ur)
    np.testing.assert_allclose(u / c, ur, rtol=5e-4)
    np.testing.assert_allclose(v * c, vr, rtol=5e-4)


@pytest.mark.parametrize("engine", ["mesh", "sweep", "stream"])
def test_shifted_kernel_every_engine_vs_oracle(dev, metric_inputs, oracle_plans, engine):
    """The shifted kernel on each engine that runs it (register-resident mesh, persistent
    sweep, per-iteration streaming pass) at reg = 0.01: 1e-4 of the float64 oracle, and
    POT's scalings recovered from (u~, v~, A, B) match the oracle's up to POT's scale
    mode (u c, v / c)."""
    from otfuse import ops
    X, Y, C, cmax, Cr = metric_inputs
    eps = 0.01
    a = torch.full((N,), 1.0 / N, device=dev)
    res = ops.sinkhorn(a, a, C, eps, max_iter=100, stop_thr=0.0, cost_scale=cmax, engine=engine,
                       shift=True)
    info = res.info()
    assert info["engine_name"] == engine and info["status_name"] == "max_iter" and info["niter"] == 99
    Pr, ur, vr, _ = oracle_plans(eps)
    assert nrel(res.plan.cpu().numpy(), Pr) < TOL32
    u, v = (t.cpu().numpy() for t in res.pot_scalings())
    c = np.median(u / ur)
    np.testing.assert_allclose(u / c, ur, rtol=5e-4)
    np.testing.assert_allclose(v * c, vr, rtol=5e-4)


def test_plain_float32_kernel_flushes_below_reg_one_over_64(dev, metric_inputs, oracle_plans):
    """Why the shift exists: the plain float32 kernel at reg = 0.01 is outside the north
    star's tolerance (K entries below 2^-126 are flushed by v_exp_f32; the CPU emulation of
    that flush gives the same 2.2e-3), and at 5e-3 it breaks at iteration 0 with a warning
    naming the remedy."""
    from otfuse import ops
    X, Y, C, cmax, Cr = metric_inputs
    a = torch.full((N,), 1.0 / N, device=dev)
    r = ops.sinkhorn(a, a, C, 0.01, max_iter=100, stop_thr=0.0, cost_scale=cmax, shift=False)
    assert r.info()["status_name"] == "max_iter" and not r.shifted
    Pr, *_ = oracle_plans(0.01)
    assert nrel(r.plan.cpu().numpy(), Pr) > 5 * TOL32
    r = ops.sinkhorn(a, a, C, 5e-3, max_iter=100, stop_thr=0.0, cost_scale=cmax, shift=False)
    with warnings.catch_warnings(record=True) as rec:
        warnings.simplefilter("always")
        i32 = r.info()
    assert i32["status_name"] == "numerical_break" and i32["break_iter"] <= 1
    assert any("shift=True" in str(w.message) for w in rec)


def test_shift_is_a_reparametrisation_in_the_plain_regime(dev, metric_inputs):
    """At reg = 0.1 (no float32 range issue) the shifted kernel reproduces the plain one:
    same iterates in exact arithmetic, plans within float32 rounding."""
    from otfuse import ops
    X, Y, C, cmax, Cr = metric_inputs
    a = torch.full((N,), 1.0 / N, device=dev)
    r0 = ops.sinkhorn(a, a, C, 0.1, max_iter=100, stop_thr=0.0, cost_scale=cmax)
    r1 = ops.sinkhorn(a, a, C, 0.1, max_iter=100, stop_thr=0.0, cost_scale=cmax, shift=True)
    assert not r0.shifted and r1.shifted
    assert r1.info()["niter"] == r0.info()["niter"] == 99
    assert nrel(r1.plan.cpu().numpy(), r0.plan.cpu().numpy()) < 1e-5


def test_shifted_fp16_storage_sweep_vs_oracle(orc, dev):
    """BASELINE config 5's storage (fp16 cost, power-of-two scaled, fp32 compute) at
    reg = 0.01 on the sweep engine with the shifted kernel, against the float64 oracle on
    the same stored values (4096 x 8192, 60 iterations)."""
    from otfuse import ops
    from otfuse.synthetic import paired_embeddings
    X, Y, _ = paired_embeddings(8192, 256, seed=77)
    Xd = torch.as_tensor(X[:4096], device=dev).half()
    Yd = torch.as_tensor(Y, device=dev).half()
    C, cmax, unit = ops.pairwise_cost_ex(Xd, Yd, out_dtype=torch.float16)
    a = torch.full((4096,), 1.0 / 4096, device=dev)
    b = torch.full((8192,), 1.0 / 8192, device=dev)
    res = ops.sinkhorn(a, b, C, 0.01, max_iter=60, stop_thr=0.0, cost_scale=cmax, engine="sweep")
    info = res.info()
    assert res.shifted and info["engine_name"] == "sweep" and info["niter"] == 59
    Cs = C.float().cpu().numpy().astype(np.float64)
    assert float(cmax) == Cs.max()       # stored values <= 1, cmax = their max
    Pr, *_ = orc.sinkhorn_knopp(np.full(4096, 1.0 / 4096), np.full(8192, 1.0 / 8192),
                                Cs / float(cmax), 0.01, 60, 0.0)
    assert nrel(res.plan.cpu().numpy(), Pr) < TOL32


@pytest.mark.parametrize("n,m,eps", [(4096, 4096, 0.1), (4000, 3001, 0.05), (1500, 8190, 2e-2)])
def test_float64_sweep_k_stream_is_bit_identical(dev, monkeypatch, n, m, eps):
    """The float64 sweep engine streams K = exp(-C / reg) written once by its prologue
    sweep (POT's own K, ot.bregman) instead of recomputing the float64 exp per element per
    sweep: the same exp of the same values, so the same plan, scalings, iteration count and
    error log bit for bit as the recomputing form (OTF_SWEEP_KSTREAM=0) in the
    deterministic mode (the default flush adds float64 partials with atomics, whose order
    varies run to run); ragged shapes and LDS-resident blocks included, every shape past the
    64 MiB from which the workspace holds K."""
    from otfuse import ops
    g = torch.Generator(device=dev).manual_seed(n + m)
    C = torch.rand(n, m, device=dev, generator=g, dtype=torch.float64)
    a = torch.full((n,), 1.0 / n, device=dev, dtype=torch.float64)
    b = torch.full((m,), 1.0 / m, device=dev, dtype=torch.float64)
    # deterministic mode: fixed-order column sums, so the two forms can be compared bitwise
    r1 = ops.sinkhorn(a, b, C, eps, max_iter=60, stop_thr=1e-12, engine="sweep", deterministic=True)
    monkeypatch.setenv("OTF_SWEEP_KSTREAM", "0")
    r0 = ops.sinkhorn(a, b, C, eps, max_iter=60, stop_thr=1e-12, engine="sweep", deterministic=True)
    i0, i1 = r0.info(), r1.info()
    assert i0["engine_name"] == i1["engine_name"] == "sweep"
    assert (i0["niter"], i0["status"], i0["err"]) == (i1["niter"], i1["status"], i1["err"])
    assert torch.equal(r0.plan, r1.plan) and torch.equal(r0.u, r1.u) and torch.equal(r0.v, r1.v)


def test_metric_shape_float64_leg_vs_oracle(orc, dev, metric_inputs, oracle_plans):
    """The float64 leg of the metric config (bench.py metric_f64): float64 cost from the
    embeddings and a float64 solve, held to 1e-9 of the float64 oracle -- at the bench's
    reg = 0.1 and at the reference's per-epoch reg = 5e-3."""
    from otfuse import gw, ops
    X, Y, _, _, Cr = metric_inputs
    Xd = torch.as_tensor(X, device=dev)
    Yd = torch.as_tensor(Y, device=dev)
    C64, _ = gw.pairwise_cost_f64(Xd, Yd, scale_max=True)
    assert nrel(C64.cpu().numpy(), Cr) < 1e-12
    a = torch.full((N,), 1.0 / N, device=dev, dtype=torch.float64)
    for eps in (0.1, 5e-3):
        res = ops.sinkhorn(a, a, C64, eps, max_iter=100, stop_thr=0.0)
        assert res.info()["status_name"] == "max_iter" and not res.shifted
        Pr, *_ = oracle_plans(eps) if eps != 0.1 else orc.sinkhorn_knopp(
            np.full(N, 1.0 / N), np.full(N, 1.0 / N), Cr, 0.1, 100, 0.0)
        assert nrel(res.plan.cpu().numpy(), Pr) < 1e-9
    # the bench form: unscaled float64 cost, the max applied inside the solve (cost_scale)
    C64u, cmax = gw.pairwise_cost_f64(Xd, Yd, scale_max=False)
    assert float(cmax) == float(C64u.max())
    res = ops.sinkhorn(a, a, C64u, 0.1, max_iter=100, stop_thr=0.0, cost_scale=cmax)
    Pr, *_ = orc.sinkhorn_knopp(np.full(N, 1.0 / N), np.full(N, 1.0 / N), Cr, 0.1, 100, 0.0)
    assert nrel(res.plan.cpu().numpy(), Pr) < 1e-9
