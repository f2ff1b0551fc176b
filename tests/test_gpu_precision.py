"""Precision coverage at the metric shape (N = 4096, d = 512, 100
iterations, max-normalised sq-Euclid cost) for the harder eps sweep {0.05, 0.01}, the
float64 form, and the regime where POT's float64 kernel-domain Sinkhorn
(MRI_PET_OT_nojax.py:143 -> sinkhorn_knopp) does not break but a float32 one would:
eps = 5e-3 (the reference's per-epoch eps, MRI_PET_OT_nojax.py:94).  The oracle is the
float64 C restatement (pinned on the golden vectors, tests/test_oracle_golden.py)."""
import warnings

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

N, D = 4096, 512


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


# Normwise plan error of the float32 path (split-fp16 cost, float32 kernel-domain solve)
# against the float64 oracle, measured on MI355X (r03): eps 0.1 -> < 1e-5, 0.05 -> < 1e-4,
# 0.01 -> 2.2e-3.  Kernel-domain Sinkhorn at small eps amplifies float32 rounding over
# the iterations; the float64 path (float64 cost + float64 solve) holds 1e-9 there.
@pytest.mark.parametrize("eps,tol32", [(0.05, 1e-4), (0.01, 5e-3)])
def test_metric_shape_harder_eps_float32_vs_float64_oracle(orc, dev, metric_inputs, eps, tol32):
    """The headline fp32 path (split-fp16 cost, mesh engine) at the harder eps of the
    sweep against the float64 oracle, and the float64 path at the same eps."""
    from otfuse import gw, ops
    X, Y, C, cmax, Cr = metric_inputs
    a = torch.full((N,), 1.0 / N, device=dev)
    res = ops.sinkhorn(a, a, C, eps, max_iter=100, stop_thr=0.0, cost_scale=cmax)
    info = res.info()
    assert info["status_name"] == "max_iter" and info["niter"] == 99
    Pr, _, _, info_r = orc.sinkhorn_knopp(np.full(N, 1.0 / N), np.full(N, 1.0 / N), Cr, eps, 100, 0.0)
    assert info_r["break_iter"] == -1
    assert nrel(res.plan.cpu().numpy(), Pr) < tol32
    C64, _ = gw.pairwise_cost_f64(torch.as_tensor(X, device=dev), torch.as_tensor(Y, device=dev),
                                  scale_max=True)
    a64 = a.double()
    r64 = ops.sinkhorn(a64, a64, C64, eps, max_iter=100, stop_thr=0.0)
    assert r64.info()["niter"] == 99
    assert nrel(r64.plan.cpu().numpy(), Pr) < 1e-9


def test_metric_shape_float64_leg_vs_oracle(orc, dev, metric_inputs):
    """The float64 leg of the metric config (bench.py metric_f64): float64 cost from the
    embeddings and a float64 solve, held to 1e-9 of the float64 oracle."""
    from otfuse import ops
    X, Y, _, _, Cr = metric_inputs
    Xd = torch.as_tensor(X, device=dev)
    Yd = torch.as_tensor(Y, device=dev)
    from otfuse import gw
    C64, _ = gw.pairwise_cost_f64(Xd, Yd, scale_max=True)
    assert nrel(C64.cpu().numpy(), Cr) < 1e-12
    a = torch.full((N,), 1.0 / N, device=dev, dtype=torch.float64)
    res = ops.sinkhorn(a, a, C64, 0.1, max_iter=100, stop_thr=0.0)
    assert res.info()["status_name"] == "max_iter"
    Pr, *_ = orc.sinkhorn_knopp(np.full(N, 1.0 / N), np.full(N, 1.0 / N), Cr, 0.1, 100, 0.0)
    assert nrel(res.plan.cpu().numpy(), Pr) < 1e-9


def test_float32_underflow_regime_auto_takes_float64(orc, dev, metric_inputs):
    """eps = 5e-3 on the max-normalised cost: some column's smallest C / eps exceeds
    float32's exp range, so a float32 kernel-domain solve breaks at iteration 0 (and
    warns), while POT's float64 solve runs on; precision='auto' detects it and solves in
    float64: same iteration count, plan within the north star's 1e-4 (the float32 cost's
    rounding, amplified by C / eps ~ 200, bounds it: 1.2e-5 measured); from a float64
    cost the float64 solve holds 1e-9."""
    from otfuse import gw, ops
    X, Y, C, cmax, Cr = metric_inputs
    eps = 5e-3
    Pr, _, _, info_r = orc.sinkhorn_knopp(np.full(N, 1.0 / N), np.full(N, 1.0 / N), Cr, eps, 100, 0.0)
    a = torch.full((N,), 1.0 / N, device=dev)
    r32 = ops.sinkhorn(a, a, C, eps, max_iter=100, stop_thr=0.0, cost_scale=cmax)
    with warnings.catch_warnings(record=True) as rec:
        warnings.simplefilter("always")
        i32 = r32.info()
    if info_r["break_iter"] == -1 and i32["status_name"] == "numerical_break":
        assert any("float32 POT Sinkhorn broke" in str(w.message) for w in rec)
    res = ops.sinkhorn(a, a, C, eps, max_iter=100, stop_thr=0.0, cost_scale=cmax, precision="auto")
    info = res.info()
    if i32["status_name"] == "numerical_break" and info_r["break_iter"] == -1:
        assert res.u.dtype == torch.float64      # the detector routed it to float64
    assert info["niter"] == info_r["niter"]
    assert nrel(res.plan.cpu().numpy(), Pr) < 1e-4
    C64, _ = gw.pairwise_cost_f64(torch.as_tensor(X, device=dev), torch.as_tensor(Y, device=dev),
                                  scale_max=True)
    a64 = a.double()
    r64 = ops.sinkhorn(a64, a64, C64, eps, max_iter=100, stop_thr=0.0)
    assert r64.info()["niter"] == info_r["niter"]
    assert nrel(r64.plan.cpu().numpy(), Pr) < 1e-9
