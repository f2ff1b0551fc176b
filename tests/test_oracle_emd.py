"""The EMD checker (oracle.emd_lp, HiGHS LP) against closed forms — CPU only.

POT's network simplex is absent, so ``pot.emd`` parity rests on this LP; it is pinned
here on the 1-D case, where the optimal cost with |x - y| is the L1 distance of the
two CDFs, and on the assignment case (uniform masses, n = m) against scipy's LAP.
"""
import ctypes

import numpy as np
import pytest


def _cdf_l1(x, a, y, b):
    pts = np.concatenate([x, y])
    order = np.argsort(pts, kind="stable")
    w = np.concatenate([a, -b])[order]
    p = pts[order]
    F = np.cumsum(w)[:-1]
    return float(np.sum(np.abs(F) * np.diff(p)))


@pytest.mark.parametrize("n,m,seed", [(5, 7, 0), (30, 20, 1), (1, 9, 2), (40, 40, 3)])
def test_emd_lp_1d_closed_form(n, m, seed):
    from oracle import oracle
    rng = np.random.default_rng(seed)
    x, y = rng.random(n), rng.random(m)
    a, b = rng.random(n) + 0.1, rng.random(m) + 0.1
    a /= a.sum()
    b /= b.sum()
    T, cost = oracle.emd_lp(a, b, np.abs(x[:, None] - y[None, :]))
    assert cost == pytest.approx(_cdf_l1(x, a, y, b), rel=1e-9, abs=1e-12)
    np.testing.assert_allclose(T.sum(1), a, atol=1e-9)
    np.testing.assert_allclose(T.sum(0), b, atol=1e-9)


def test_emd_lp_uniform_square_is_assignment():
    from scipy.optimize import linear_sum_assignment
    from oracle import oracle
    rng = np.random.default_rng(9)
    M = rng.random((25, 25))
    T, cost = oracle.emd_lp(np.full(25, 1 / 25), np.full(25, 1 / 25), M)
    r, c = linear_sum_assignment(M)
    assert cost == pytest.approx(M[r, c].sum() / 25, rel=1e-12)
    assert np.abs(T[r, c] - 1 / 25).max() < 1e-9


def test_emd_abi_layout():
    from otfuse import _lib as L
    import re
    assert ctypes.sizeof(L.EmdProblem) == 56
    src = open(L.HEADER_PATH).read()
    for name, val in [("OTF_EMD_OPTIMAL", 0), ("OTF_EMD_MAX_ITER", 1), ("OTF_EMD_INFEASIBLE", 2),
                      ("OTF_EMD_UNBOUNDED", 3)]:
        m = re.search(rf"\b{name}\s*=\s*(-?\d+)", src)
        assert m and int(m.group(1)) == val, name
    lib = L.lib()
    assert lib.otf_emd_max_nodes() >= 4096 and lib.otf_emd_lds_nodes() == 4800
    probs = (L.EmdProblem * 1)()
    assert lib.otf_emd_solve(0, probs, 10, None, None) == L.OTF_EINVAL
    probs[0] = L.EmdProblem(None, None, None, 1, None, 1, 1, 1)
    assert lib.otf_emd_solve(1, probs, 10, None, None) == L.OTF_EINVAL
