"""COOT-L oracle (CPU).  OTT and POT are absent, so the COOT-L restatement is parity
UNPINNED against the reference's outputs; what is checked here: the coupled cost
against the literal init_matrix_np construction (perturbot utils.py:125-184), and the
BCD loop's invariants (unit-mass couplings, monotone stop rule)."""
import numpy as np


def test_coupled_cost_matches_init_matrix_construction(orc):
    rng = np.random.default_rng(1)
    X = rng.random((13, 7)).astype(np.float32)
    Y = rng.random((11, 5)).astype(np.float32)
    v1 = rng.random(7)
    v2 = rng.random(5)
    Tv = rng.random((7, 5))
    # utils.py:173-184: constC = f1(X) v1 1^T + 1 v2^T f2(Y)^T, hX1 = X, hX2 = 2 Y
    constC = (X ** 2).astype(np.float64) @ v1.reshape(-1, 1) @ np.ones((1, 11)) + \
        np.ones((13, 1)) @ (v2.reshape(1, -1) @ (Y ** 2).astype(np.float64).T)
    ref = constC - (X.astype(np.float64) @ Tv) @ (2 * Y.astype(np.float64)).T
    M = orc.coupled_cost_np(X, Y, Tv, v1, v2)
    assert np.abs(M - ref).max() < 1e-12 * np.abs(ref).max()
    # the feature-side cost is the same construction on the transposed data
    Ts = rng.random((13, 11))
    w1 = np.ones(13) / 13
    w2 = np.ones(11) / 11
    Mf = orc.coupled_cost_np(X.T, Y.T, Ts, w1, w2)
    assert Mf.shape == (7, 5)


def test_cotl_sinkhorn_oracle_invariants(orc):
    rng = np.random.default_rng(0)
    Xd = {0: rng.random((20, 12)).astype(np.float32), 1: rng.random((25, 12)).astype(np.float32)}
    Yd = {0: rng.random((22, 9)).astype(np.float32), 1: rng.random((18, 9)).astype(np.float32)}
    Ts, Tv, cost, log = orc.cotl_sinkhorn_np(Xd, Yd, 5e-2, niter=2000)
    assert set(Ts) == {0, 1} and Ts[0].shape == (20, 22) and Tv.shape == (12, 9)
    assert abs(Tv.sum() - 1.0) < 1e-8
    for T in Ts.values():
        assert abs(T.sum() - 1.0) < 1e-6
    c = log["cost"]
    assert len(c) < 2000 and abs(c[-1] - c[-2]) < 1e-7 and cost == c[-1]
