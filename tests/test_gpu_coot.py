"""COOT-L on the device (perturbot cot_labels.py) vs the oracle restatement.

OTT is absent, so parity is with the oracle's log-domain Sinkhorn restatement
(UNPINNED against the reference's own outputs); the EMD variant is pinned on
scipy's HiGHS LP (POT's network simplex is absent too).  Bars: coupled costs to 1e-12 relative
(float64 from float32 squares); the BCD loop must take the same number of iterations
and reach couplings within 1e-6 normwise."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def nrel(x, ref):
    return np.abs(np.asarray(x) - ref).max() / np.abs(ref).max()


@pytest.mark.parametrize("p,q,r,s", [(13, 11, 7, 5), (200, 150, 64, 48), (1, 3, 2, 1)])
def test_coupled_cost_vs_oracle(orc, dev, p, q, r, s):
    from otfuse import ops
    rng = np.random.default_rng(p + q)
    X = rng.standard_normal((p, r)).astype(np.float32)
    Y = rng.standard_normal((q, s)).astype(np.float32)
    T = rng.random((r, s))
    w1 = rng.random(r)
    w2 = rng.random(s)
    M = ops.coupled_cost(torch.as_tensor(X, device=dev), torch.as_tensor(Y, device=dev),
                         torch.as_tensor(T, device=dev), torch.as_tensor(w1, device=dev),
                         torch.as_tensor(w2, device=dev)).cpu().numpy()
    assert nrel(M, orc.coupled_cost_np(X, Y, T, w1, w2)) < 1e-12
    # transposed views (the feature-side cost): no copies, strides only
    Tt = rng.random((p, q))
    u1 = rng.random(p)
    u2 = rng.random(q)
    Xt = torch.as_tensor(X, device=dev).T
    Yt = torch.as_tensor(Y, device=dev).T
    Mt = ops.coupled_cost(Xt, Yt, torch.as_tensor(Tt, device=dev), torch.as_tensor(u1, device=dev),
                          torch.as_tensor(u2, device=dev)).cpu().numpy()
    assert nrel(Mt, orc.coupled_cost_np(X.T, Y.T, Tt, u1, u2)) < 1e-12


def test_cotl_sinkhorn_dropin_vs_oracle(orc, dev):
    from otfuse import perturbot
    rng = np.random.default_rng(0)
    Xd = {0: rng.random((20, 12)).astype(np.float32), 1: rng.random((25, 12)).astype(np.float32)}
    Yd = {0: rng.random((22, 9)).astype(np.float32), 1: rng.random((18, 9)).astype(np.float32)}
    Ts, log = perturbot.get_coupling_cotl_sinkhorn((Xd, Yd), eps=5e-2)
    Tr, Tvr, cost_r, log_r = orc.cotl_sinkhorn_np(Xd, Yd, 5e-2, niter=2000)
    assert len(log["cost"]) == len(log_r["cost"]) and "time" in log
    np.testing.assert_allclose(log["cost"], log_r["cost"], rtol=1e-6)
    for k in Xd:
        assert nrel(Ts[k], Tr[k]) < 1e-6


def test_cotl_emd_dropin_vs_oracle(orc, dev):
    """get_coupling_cotl: exact EMD (device network simplex) on general feature
    marginals, vs the BCD loop over HiGHS LP solves: same iterations, same plans."""
    from otfuse import perturbot
    rng = np.random.default_rng(1)
    Xd = {0: rng.random((20, 12)).astype(np.float32), 1: rng.random((25, 12)).astype(np.float32)}
    Yd = {0: rng.random((22, 9)).astype(np.float32), 1: rng.random((18, 9)).astype(np.float32)}
    Ts, log = perturbot.get_coupling_cotl((Xd, Yd))
    Tr, Tvr, cost_r, log_r = orc.cotl_emd_np(Xd, Yd, niter=2000)
    assert len(log["cost"]) == len(log_r["cost"]) and "time" in log
    np.testing.assert_allclose(log["cost"], log_r["cost"], rtol=1e-9)
    for k in Xd:
        assert np.abs(Ts[k] - Tr[k]).max() < 1e-9
