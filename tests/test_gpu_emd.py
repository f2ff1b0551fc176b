"""Exact EMD (otf_emd_solve, the device network simplex) vs the transportation LP.

POT is absent from the image, so ``pot.emd`` is pinned on scipy's HiGHS LP
(oracle.emd_lp): with generic costs the optimal plan is unique, so plans must agree
entry-wise (1e-9 absolute on unit mass) and costs to 1e-10 relative.  Degenerate
problems (uniform masses, zero masses, 1 x m) may have several optimal plans: there
the cost must match and the plan must be feasible and basic (<= n + m - 1 nonzeros).
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _problem(rng, n, m, zeros=0, uniform=False, scale=1.0):
    a = np.ones(n) / n if uniform else rng.random(n) + 0.05
    b = np.ones(m) / m if uniform else rng.random(m) + 0.05
    for _ in range(zeros):
        a[rng.integers(n)] = 0.0
    a /= a.sum()
    b /= b.sum()
    M = rng.random((n, m)) * scale
    return a, b, M


def _check_feasible(T, a, b, tol=1e-12):
    assert (T >= -tol).all()
    np.testing.assert_allclose(T.sum(1), a, atol=tol * 10)
    np.testing.assert_allclose(T.sum(0), b * a.sum() / b.sum(), atol=tol * 10)
    assert (np.abs(T) > 1e-15).sum() <= T.shape[0] + T.shape[1] - 1


@pytest.mark.parametrize("n,m", [(1, 1), (1, 7), (9, 1), (13, 11), (40, 70), (120, 90), (300, 250)])
def test_emd_vs_lp(orc, dev, n, m):
    from otfuse import pot
    rng = np.random.default_rng(n * 1000 + m)
    a, b, M = _problem(rng, n, m)
    T, log = pot.emd(a, b, M, log=True)
    Tr, cr = orc.emd_lp(a, b, M)
    _check_feasible(T, a, b)
    assert abs(log["cost"] - cr) <= 1e-10 * max(abs(cr), 1e-300) + 1e-15
    assert np.abs(T - Tr).max() < 1e-9
    assert log["result_code"] == 1 and log["warning"] is None


@pytest.mark.parametrize("case", ["uniform", "zeros", "wide_costs"])
def test_emd_degenerate_and_scaled(orc, dev, case):
    from otfuse import pot
    rng = np.random.default_rng(7)
    if case == "uniform":
        a, b, M = _problem(rng, 30, 30, uniform=True)
    elif case == "zeros":
        a, b, M = _problem(rng, 25, 35, zeros=5)
    else:
        a, b, M = _problem(rng, 50, 40, scale=1e6)
        M[::3] *= 1e-6
    T, log = pot.emd(a, b, M, log=True)
    Tr, cr = orc.emd_lp(a, b, M)
    _check_feasible(T, a, b)
    assert abs(log["cost"] - cr) <= 1e-9 * abs(cr) + 1e-12
    if case == "zeros":
        assert np.abs(T[a == 0]).max() == 0.0


def test_emd_batch_equals_single_solves(orc, dev):
    from otfuse import pot
    rng = np.random.default_rng(3)
    probs = [_problem(rng, int(rng.integers(2, 60)), int(rng.integers(2, 60))) for _ in range(70)]
    outs = pot.emd_batch(probs)     # 70 problems: two launches of <= 64 workgroups
    for (a, b, M), T in zip(probs, outs):
        assert np.array_equal(T, pot.emd(a, b, M))
    for (a, b, M), T in list(zip(probs, outs))[:5]:
        assert np.abs(T - orc.emd_lp(a, b, M)[0]).max() < 1e-9


def test_emd_pot_conventions(dev):
    from otfuse import pot
    rng = np.random.default_rng(5)
    M = rng.random((6, 8))
    T = pot.emd([], [], M)                       # empty -> uniform
    np.testing.assert_allclose(T.sum(1), np.ones(6) / 6, atol=1e-14)
    a = np.ones(6) / 6
    b = np.ones(8) / 8 * (1 + 1e-8)              # rescaled to a's mass
    T2 = pot.emd(a, b, M)
    np.testing.assert_allclose(T2.sum(0), np.ones(8) / 8, atol=1e-14)
    with pytest.raises(AssertionError):
        pot.emd(a, np.ones(8) / 4, M)            # masses differ: POT's check_marginals
    with pytest.warns(UserWarning, match="numItermax"):
        _, log = pot.emd(a, np.ones(8) / 8, M, numItermax=2, log=True)
    assert log["result_code"] == 3
    Md = torch.as_tensor(M, device=dev)          # device in, device out
    Td = pot.emd(torch.as_tensor(a, device=dev), torch.full((8,), 1 / 8, device=dev, dtype=torch.float64), Md)
    assert isinstance(Td, torch.Tensor) and Td.is_cuda
    assert np.abs(Td.cpu().numpy() - pot.emd(a, np.ones(8) / 8, M)).max() == 0.0


def test_emd_largest_size_is_feasible_and_optimal_vs_product(dev):
    """n + m + 1 at the LDS bound: feasible, basic, and no worse than the product
    plan or a north-west-corner plan."""
    from otfuse import ops, pot
    n = ops.emd_lds_nodes() // 2 - 1
    m = ops.emd_lds_nodes() - n - 1
    rng = np.random.default_rng(11)
    a, b, M = _problem(rng, n, m)
    T, log = pot.emd(a, b, M, log=True)
    _check_feasible(T, a, b, tol=1e-11)
    assert log["cost"] <= float((np.outer(a, b) * M).sum())
    assert log["result_code"] == 1


def _dual_certificate(T, M, a, b, tol):
    """Optimality of a feasible basic plan: potentials from the positive arcs (a spanning
    tree of the bipartite graph for non-degenerate masses), then every reduced cost
    M_ij - u_i - v_j >= -tol."""
    n, m = M.shape
    ii, jj = np.nonzero(T > 1e-15)
    assert len(ii) == n + m - 1                        # non-degenerate: a spanning tree
    adj_r = [[] for _ in range(n)]
    adj_c = [[] for _ in range(m)]
    for i, j in zip(ii, jj):
        adj_r[i].append(j)
        adj_c[j].append(i)
    u = np.full(n, np.nan)
    v = np.full(m, np.nan)
    u[0] = 0.0
    stack = [("r", 0)]
    while stack:
        kind, k = stack.pop()
        if kind == "r":
            for j in adj_r[k]:
                if np.isnan(v[j]):
                    v[j] = M[k, j] - u[k]
                    stack.append(("c", j))
        else:
            for i in adj_c[k]:
                if np.isnan(u[i]):
                    u[i] = M[i, k] - v[k]
                    stack.append(("r", i))
    assert not np.isnan(u).any() and not np.isnan(v).any()
    red = M - u[:, None] - v[None, :]
    assert red.min() >= -tol, red.min()


@pytest.mark.parametrize("n,m", [(13, 11), (120, 90), (300, 250)])
def test_emd_global_tree_matches_lds_tree(orc, dev, monkeypatch, n, m):
    """The global-memory tree (problems past the LDS) runs the same pivots: forced on
    problems that fit the LDS, the plans and pivot counts are bit-identical."""
    from otfuse import ops
    rng = np.random.default_rng(n + 7 * m)
    a, b, M = _problem(rng, n, m)
    args = [(torch.as_tensor(a, device=dev), torch.as_tensor(b, device=dev), torch.as_tensor(M, device=dev))]
    r0 = ops.emd_batched(args)
    T0, i0 = r0.plans[0].cpu().numpy(), r0.infos()[0]
    monkeypatch.setenv("OTF_EMD_TREE", "global")
    r1 = ops.emd_batched(args)
    T1, i1 = r1.plans[0].cpu().numpy(), r1.infos()[0]
    assert np.array_equal(T0, T1) and i0["n_pivots"] == i1["n_pivots"] and i0["cost"] == i1["cost"]
    Tr, cr = orc.emd_lp(a, b, M)
    assert np.abs(T1 - Tr).max() < 1e-9


def test_emd_past_the_lds_ceiling_is_optimal(dev):
    """n + m + 1 = 5201 > the LDS bound (4800), where POT's emd has no ceiling: the
    global-tree network simplex returns a feasible basic plan with a dual certificate
    (every reduced cost >= 0 for the potentials of its tree)."""
    from otfuse import ops, pot
    n, m = 2700, 2500
    assert n + m + 1 > ops.emd_lds_nodes()
    rng = np.random.default_rng(21)
    a, b, M = _problem(rng, n, m)
    T, log = pot.emd(a, b, M, log=True, numItermax=10 ** 7)
    assert log["result_code"] == 1
    _check_feasible(T, a, b, tol=1e-11)
    _dual_certificate(T, M, a, b, tol=1e-9)
    assert log["cost"] == pytest.approx(float((T * M).sum()), rel=1e-12)
