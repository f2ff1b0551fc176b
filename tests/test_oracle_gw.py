"""GW oracle self-consistency (CPU).  POT / OTT are absent from the container, so the
GW restatements are parity-UNPINNED against the reference's own outputs; what is pinned
here is the exact-EMD inner solve (the C LAP vs scipy's independent
``linear_sum_assignment``) and the C CG-GW vs a NumPy restatement built on scipy."""
import numpy as np
import pytest


def _costs(n, d, seed, metric="euclidean"):
    from oracle import oracle as o
    from otfuse.synthetic import paired_embeddings
    X, Y, _ = paired_embeddings(n, d, seed=seed)
    C1, _ = o.pairwise_cost(X, X, metric=metric, zero_diag=metric == "euclidean", scale_max=True)
    C2, _ = o.pairwise_cost(Y, Y, metric=metric, zero_diag=metric == "euclidean", scale_max=True)
    return C1, C2


@pytest.mark.parametrize("n", [1, 2, 3, 17, 64, 200])
def test_lap_matches_scipy(orc, n):
    from scipy.optimize import linear_sum_assignment
    rng = np.random.default_rng(n)
    for _ in range(5):
        A = rng.standard_normal((n, n))
        _, cols = linear_sum_assignment(A)
        assert (orc.lap(A) == cols).all()


def test_lap_integer_ties_reach_the_optimum(orc):
    from scipy.optimize import linear_sum_assignment
    rng = np.random.default_rng(3)
    A = rng.integers(0, 3, (40, 40)).astype(np.float64)
    s = orc.lap(A)
    r, c = linear_sum_assignment(A)
    assert sorted(s.tolist()) == list(range(40))
    assert A[np.arange(40), s].sum() == A[r, c].sum()


def test_lap_rejects_nan(orc):
    A = np.ones((4, 4))
    A[:, 2] = np.nan
    with pytest.raises(FloatingPointError):
        orc.lap(A)


@pytest.mark.parametrize("n,seed", [(2, 1), (16, 2), (64, 3), (100, 4)])
def test_gw_cg_c_matches_numpy_scipy(orc, n, seed):
    C1, C2 = _costs(n, 24, seed)
    G, info = orc.gw_cg(C1, C2)
    G2, info2 = orc.gw_cg_np(C1, C2)
    assert info["n_iter"] == info2["n_iter"]
    assert np.abs(G - G2).max() < 1e-12
    assert info["gw_dist"] == pytest.approx(info2["gw_dist"], rel=1e-10, abs=1e-14)
    np.testing.assert_allclose(G.sum(1), 1.0 / n, rtol=1e-12)
    np.testing.assert_allclose(G.sum(0), 1.0 / n, rtol=1e-12)


def test_gw_cg_recovers_an_isometry(orc):
    """GW between a point cloud and a permuted copy of itself is zero at the permutation."""
    rng = np.random.default_rng(5)
    X = rng.standard_normal((30, 5))
    perm = rng.permutation(30)
    C1, _ = orc.pairwise_cost(X, X, metric="euclidean", zero_diag=True, scale_max=True)
    C2 = C1[np.ix_(perm, perm)]
    G, info = orc.gw_cg(C1, C2)
    assert info["gw_dist"] == pytest.approx(0.0, abs=1e-12)
    assert (G.argmax(1) == np.argsort(perm)).all()


@pytest.mark.parametrize("n,m", [(40, 40), (30, 50)])
def test_gw_entropic_marginals_and_log(orc, n, m):
    C1, _ = _costs(n, 16, 7, "sqeuclidean")
    _, C2 = _costs(m, 16, 8, "sqeuclidean")
    P, info = orc.gw_entropic(C1, C2, 5e-3)
    assert info["status"] == 1 and info["converged"]
    assert info["n_iters"] >= 5
    assert np.abs(P.sum(1) - 1.0 / n).max() < 1e-12     # f-update last: rows exact
    assert np.abs(P.sum(0) - 1.0 / m).sum() < 1e-3      # OTT threshold on the L1 column error
    c = info["costs"]
    assert abs(c[-2] - c[-1]) <= 1e-8 + 1e-3 * abs(c[-1])


def test_gw_entropic_labels_block_structure(orc):
    C1, C2 = _costs(40, 16, 9, "sqeuclidean")
    la = np.array([0] * 25 + [1] * 15, np.int32)
    lb = np.array([1] * 15 + [0] * 25, np.int32)
    P, info = orc.gw_entropic(C1, C2, 1e-2, labels_a=la, labels_b=lb)
    assert info["status"] == 1
    assert P[np.not_equal.outer(la, lb)].max() == 0.0
    np.testing.assert_allclose(P[la == 0].sum(), 25 / 40, rtol=1e-6)


@pytest.mark.parametrize("n,m,eps", [(20, 20, 5e-2), (30, 45, 1e-2), (40, 40, 5e-3)])
def test_gw_pgd_c_matches_numpy(orc, n, m, eps):
    """POT entropic GW (solver='PGD'): the C restatement against the NumPy one, which
    follows POT's code line by line on top of ``sinkhorn_knopp_np``."""
    C1, _ = _costs(n, 16, 11)
    _, C2 = _costs(m, 16, 12)
    T, info = orc.gw_pgd(C1, C2, eps)
    T2, info2 = orc.gw_pgd_np(C1, C2, eps)
    assert info["n_iter"] == info2["n_iter"]
    assert np.abs(T - T2).max() < 1e-12 * np.abs(T2).max()
    np.testing.assert_allclose(info["err"], info2["err"], rtol=1e-6, atol=1e-14)
    assert info["gw_dist"] == pytest.approx(info2["gw_dist"], rel=1e-10)
    assert info["converged"] and abs(T.sum() - 1.0) < 1e-9


def test_gw_pgd_weighted_marginals(orc):
    """Non-uniform p, q: the plan's marginals are the histograms (inner Sinkhorn)."""
    rng = np.random.default_rng(3)
    C1, _ = _costs(25, 8, 21)
    _, C2 = _costs(35, 8, 22)
    p = rng.random(25) + 0.5
    p /= p.sum()
    q = rng.random(35) + 0.5
    q /= q.sum()
    T, info = orc.gw_pgd(C1, C2, 2e-2, a=p, b=q)
    T2, info2 = orc.gw_pgd_np(C1, C2, 2e-2, p=p, q=q)
    assert info["n_iter"] == info2["n_iter"]
    assert np.abs(T - T2).max() < 1e-12 * np.abs(T2).max()
    np.testing.assert_allclose(T.sum(1), p, rtol=1e-9)
    np.testing.assert_allclose(T.sum(0), q, atol=1e-8)
