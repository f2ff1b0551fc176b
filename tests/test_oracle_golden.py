"""The CPU oracle against the golden vectors produced by the reference's own code
(tests/golden/make_golden.py).  CPU only."""
import numpy as np
import pytest


def _plan_from(u, v, C, reg):
    return u[:, None] * np.exp(C / (-reg)) * v[None, :]


def _scale_free(u, v):
    """u, v are defined up to u*c, v/c; drift along that mode is rounding, not error."""
    s = np.linalg.norm(u)
    return u / s, v * s


def test_f1_sinkhorn_fixed_iters(golden, orc):
    f = golden("f1_sinkhorn_256.npz")
    C, _ = orc.pairwise_cost(f["X"], f["Y"], scale_max=True)
    a = np.ones(256) / 256
    P, u, v, info = orc.sinkhorn_knopp(a, a, C, float(f["reg"]), int(f["iters"]), 0.0)
    assert info["n_updates"] == 50 and info["break_iter"] == -1
    ur, vr = _scale_free(f["u"], f["v"])
    uo, vo = _scale_free(u, v)
    np.testing.assert_allclose(uo, ur, rtol=1e-10)
    np.testing.assert_allclose(vo, vr, rtol=1e-10)
    idx = f["idx"]
    np.testing.assert_allclose(P[idx[:, 0], idx[:, 1]], f["plan_samples"], rtol=1e-10)
    np.testing.assert_allclose(P.sum(0), f["plan_colsum"], rtol=1e-10, atol=1e-18)


def test_f2_feature_coupling_converged_mode(golden, orc):
    f = golden("f2_feature_pot_b8_d512.npz")
    M = orc.feature_cost(f["X"], f["Y"], np.eye(8) / 8)
    idx = f["idx"]
    np.testing.assert_allclose(M[idx[:, 0], idx[:, 1]], f["M_samples"], rtol=1e-12, atol=1e-14)
    np.testing.assert_allclose(M.sum(1), f["M_rowsum"], rtol=1e-12)
    d = M.shape[0]
    a = np.ones(d) / d
    P, u, v, info = orc.sinkhorn_knopp(a, a, M, float(f["eps"]), int(f["numItermax"]),
                                       float(f["stopThr"]))
    assert len(info["err"]) == int(f["n_err"])
    np.testing.assert_allclose(info["err"], f["err"], rtol=1e-6)
    # not converged after 2000 iterations (slow map): entries agree normwise; the
    # relative error of individual tiny entries is amplified rounding
    ps = P[idx[:, 0], idx[:, 1]]
    assert np.abs(ps - f["plan_samples"]).max() <= 1e-9 * np.abs(f["plan_samples"]).max()
    np.testing.assert_allclose(P.sum(1), f["plan_rowsum"], rtol=1e-8)


def test_f3_numerical_break_reverts(golden, orc):
    f = golden("f3_numerical_break.npz")
    M = orc.feature_cost(f["X"], f["Y"], np.eye(8) / 8)
    d = M.shape[0]
    a = np.ones(d) / d
    P, u, v, info = orc.sinkhorn_knopp(a, a, M, float(f["eps"]), 2000, 1e-9)
    assert info["break_iter"] == 0 and info["n_updates"] == 0
    np.testing.assert_allclose(u, 1.0 / d)
    # K/(n m) with M/eps ~ 1e3: exp() amplifies last-bit differences in M, so compare
    # normwise (max |dP| / max |P|)
    assert np.abs(P - f["plan"]).max() <= 1e-9 * np.abs(f["plan"]).max()
    assert np.array_equal(P == 0, f["plan"] == 0)


def test_f4_blockdiag_ts_and_nonsquare(golden, orc):
    f = golden("f4_feature_blockdiag.npz")
    xd = {0: f["X0"], 1: f["X1"]}
    yd = {0: f["Y0"], 1: f["Y1"]}
    Ts = orc.block_diag_ts({0: f["Ts0"], 1: f["Ts1"]}, xd, yd)
    np.testing.assert_array_equal(Ts, f["Ts"])
    M = orc.feature_cost(f["Xcat"], f["Ycat"], Ts)
    np.testing.assert_allclose(M, f["M"], rtol=1e-12, atol=1e-13)
    d, d2 = M.shape
    P, u, v, info = orc.sinkhorn_knopp(np.ones(d) / d, np.ones(d2) / d2, M, float(f["eps"]), 2000,
                                       1e-9)
    assert len(info["err"]) == int(f["n_err"])
    np.testing.assert_allclose(P, f["plan"], rtol=1e-9, atol=1e-300)


def test_numpy_and_c_restatements_agree(orc):
    rng = np.random.default_rng(3)
    X = rng.random((37, 11))
    Y = rng.random((29, 11))
    Cn = orc.pairwise_cost_np(X, Y)
    Cc, mx = orc.pairwise_cost(X, Y)
    np.testing.assert_allclose(Cc, Cn, rtol=1e-12, atol=1e-12)
    assert mx == pytest.approx(Cn.max())
    Ts = rng.random((37, 29))
    np.testing.assert_allclose(orc.feature_cost(X, Y, Ts), orc.feature_cost_np(X, Y, Ts),
                               rtol=1e-11, atol=1e-11)
    a = np.ones(37) / 37
    b = np.ones(29) / 29
    Pn, un, vn, inf_n = orc.sinkhorn_knopp_np(a, b, Cn / Cn.max(), 0.05, 300, 1e-9)
    Pc, uc, vc, inf_c = orc.sinkhorn_knopp(a, b, Cn / Cn.max(), 0.05, 300, 1e-9)
    assert inf_n["niter"] == inf_c["niter"]
    np.testing.assert_allclose(Pc, Pn, rtol=1e-10, atol=1e-16)


def test_euclidean_zero_diag_and_max_iter_zero(orc):
    rng = np.random.default_rng(5)
    X = rng.random((9, 4))
    C, _ = orc.pairwise_cost(X, X, metric="euclidean", zero_diag=True)
    assert np.all(np.diag(C) == 0)
    np.testing.assert_allclose(C, orc.pairwise_cost_np(X, X, "euclidean", zero_diag=True), rtol=1e-12)
    a = np.ones(9) / 9
    P, u, v, info = orc.sinkhorn_knopp(a, a, C, 0.1, 0, 1e-9)
    np.testing.assert_allclose(P, np.exp(-C / 0.1) / 81, rtol=1e-14)


def test_log_domain_restatement_matches_kernel_domain(orc):
    """OTT-flavour restatement (unpinned) agrees with POT's at convergence."""
    rng = np.random.default_rng(11)
    C = rng.random((40, 30))
    a = np.ones(40) / 40
    b = np.ones(30) / 30
    P1, f, g, info = orc.sinkhorn_log(a, b, C, 0.05, max_iter=2000, threshold=1e-12)
    P2, *_ = orc.sinkhorn_knopp(a, b, C, 0.05, 5000, 1e-14)
    np.testing.assert_allclose(P1, P2, rtol=1e-7, atol=1e-14)
    np.testing.assert_allclose(P1.sum(1), a, rtol=1e-9)


def test_plan_apply_matches_fixture(golden, orc):
    f = golden("f2_feature_pot_b8_d512.npz")
    M = orc.feature_cost(f["X"], f["Y"], np.eye(8) / 8)
    d = M.shape[0]
    P, *_ = orc.sinkhorn_knopp(np.ones(d) / d, np.ones(d) / d, M, 1e-2, 2000, 1e-9)
    Tn, out = orc.plan_apply(P, f["Y"])
    idx = f["idx"]
    np.testing.assert_allclose(Tn[idx[:, 0], idx[:, 1]], f["Tn_samples"], rtol=2e-5)
    np.testing.assert_allclose(out, f["ot_mri_from_pet"], rtol=2e-5, atol=1e-6)


def test_random_gamma_init_matches_reference_draw_and_scaling(golden, orc):
    """F5: the oracle's random_gamma_init (utils.py:118-122) draws the same Beta(0.1,
    0.1) matrix from NumPy's global generator and scales it like the reference's own
    sinkhorn_scaling."""
    f = golden("f5_random_gamma_init.npz")
    for tag in ("a", "b"):
        np.random.seed(int(f[f"seed_{tag}"]))
        P = orc.random_gamma_init_np(f[f"p_{tag}"], f[f"q_{tag}"])
        np.testing.assert_allclose(P, f[f"plan_{tag}"], rtol=1e-12, atol=1e-300)

