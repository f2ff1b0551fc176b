"""Device GW solvers (csrc/otf_gw.hip) vs the oracle's GW restatements.

POT / OTT are absent, so the oracle itself is parity-UNPINNED against the reference's
outputs (its exact-EMD step is pinned to scipy in tests/test_oracle_gw.py).  Bars:
CG-GW is a vertex / short convex path — plans must agree to 1e-12 absolute and the
iteration counts exactly; entropic GW in float64 — plans within 1e-4 normwise relative
(the north star's tolerance), identical outer iteration counts.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def nrel(x, ref):
    return np.abs(np.asarray(x) - ref).max() / np.abs(ref).max()


def _emb(n, d, seed):
    from otfuse.synthetic import paired_embeddings
    return paired_embeddings(n, d, seed=seed)


@pytest.mark.parametrize("metric,zero_diag,n,m,d", [("euclidean", True, 64, 64, 512),
                                                    ("sqeuclidean", False, 130, 77, 33),
                                                    ("euclidean", False, 1, 5, 3),
                                                    # 128 x 128 float64 tiles, fused epilogue
                                                    ("euclidean", True, 1000, 1000, 64),
                                                    ("sqeuclidean", False, 1030, 777, 300),
                                                    ("sqeuclidean", False, 2048, 300, 1027)])
def test_pairwise_cost_f64_vs_oracle(orc, dev, metric, zero_diag, n, m, d):
    """Past 16384 outputs the 128 x 128 tile kernel on float64 MFMA, to 1e-12 of the
    oracle."""
    from otfuse import gw
    X, _, _ = _emb(n, d, 1)
    _, Y, _ = _emb(m, d, 2)
    same = n == m and zero_diag
    Xd = torch.as_tensor(X, device=dev)
    Yd = Xd if same else torch.as_tensor(Y, device=dev)
    C, cmax = gw.pairwise_cost_f64(Xd, None if same else Yd, metric=metric, zero_diag=zero_diag,
                                   scale_max=True)
    Cr, mr = orc.pairwise_cost(X, X if same else Y, metric=metric, zero_diag=zero_diag,
                               scale_max=True)
    assert float(cmax) == pytest.approx(mr, rel=1e-12)
    assert np.abs(C.cpu().numpy() - Cr).max() < 1e-12


def _label_costs(orc, sizes, d, seed, metric="euclidean"):
    out = []
    for k, n in enumerate(sizes):
        X, Y, _ = _emb(n, d, seed + k)
        zd = metric == "euclidean"
        C1, _ = orc.pairwise_cost(X, X, metric=metric, zero_diag=zd, scale_max=True)
        C2, _ = orc.pairwise_cost(Y, Y, metric=metric, zero_diag=zd, scale_max=True)
        out.append((C1, C2))
    return out


def test_gw_cg_batched_vs_oracle(orc, dev):
    """Every label problem of one launch (sizes 1..200) against the C restatement."""
    from otfuse import gw
    sizes = [1, 2, 3, 17, 64, 64, 100, 130, 200]
    probs = _label_costs(orc, sizes, 48, 10)
    res = gw.solve_batched([torch.as_tensor(c1, device=dev) for c1, _ in probs],
                           [torch.as_tensor(c2, device=dev) for _, c2 in probs], gw.GW_CG,
                           max_iter=10000, log_len=64)
    infos = res.infos()
    for (C1, C2), T, info in zip(probs, res.plans, infos):
        G, ref = orc.gw_cg(C1, C2)
        assert info["status"] == "converged", info
        assert info["n_iter"] == ref["n_iter"]
        assert np.abs(T.cpu().numpy() - G).max() < 1e-12
        assert info["cost"] == pytest.approx(ref["gw_dist"], rel=1e-9, abs=1e-13)
        np.testing.assert_allclose(info["costs"], ref["loss"], rtol=1e-9, atol=1e-13)


def test_gw_cg_random_metric_spaces_many_seeds(orc, dev):
    """Random point clouds (not the structured embeddings): 16 problems in one launch,
    each checked against the NumPy + scipy restatement (independent LAP)."""
    from otfuse import gw
    rng = np.random.default_rng(123)
    C1s, C2s = [], []
    for k in range(16):
        n = int(rng.integers(5, 90))
        A = rng.standard_normal((n, 3))
        B = rng.standard_normal((n, 4))
        C1s.append(orc.pairwise_cost(A, A, metric="euclidean", zero_diag=True, scale_max=True)[0])
        C2s.append(orc.pairwise_cost(B, B, metric="euclidean", zero_diag=True, scale_max=True)[0])
    res = gw.solve_batched([torch.as_tensor(c, device=dev) for c in C1s],
                           [torch.as_tensor(c, device=dev) for c in C2s], gw.GW_CG, max_iter=10000)
    for C1, C2, T, info in zip(C1s, C2s, res.plans, res.infos()):
        G, ref = orc.gw_cg_np(C1, C2)
        assert info["n_iter"] == ref["n_iter"]
        assert np.abs(T.cpu().numpy() - G).max() < 1e-12
        assert info["cost"] == pytest.approx(ref["gw_dist"], rel=1e-9, abs=1e-13)


def test_gw_cg_unequal_and_weighted_vs_oracle(orc, dev):
    """CG-GW on unequal groups and non-uniform marginals (POT's call with general p, q):
    the linear step is the device network simplex; the oracle runs the same CG with the
    HiGHS LP as EMD.  Generic costs -> unique vertices -> same path."""
    from otfuse import gw
    rng = np.random.default_rng(77)
    C1s, C2s, ps, qs = [], [], [], []
    for k in range(6):
        n, m = int(rng.integers(3, 60)), int(rng.integers(3, 60))
        A = rng.standard_normal((n, 3))
        B = rng.standard_normal((m, 4))
        C1s.append(orc.pairwise_cost(A, A, metric="euclidean", zero_diag=True, scale_max=True)[0])
        C2s.append(orc.pairwise_cost(B, B, metric="euclidean", zero_diag=True, scale_max=True)[0])
        if k % 2:
            p = rng.random(n) + 0.1
            q = rng.random(m) + 0.1
            ps.append(p / p.sum())
            qs.append(q / q.sum())
        else:
            ps.append(None)
            qs.append(None)
    res = gw.solve_batched([torch.as_tensor(c, device=dev) for c in C1s],
                           [torch.as_tensor(c, device=dev) for c in C2s], gw.GW_CG,
                           ps=[None if p is None else torch.as_tensor(p, device=dev) for p in ps],
                           qs=[None if q is None else torch.as_tensor(q, device=dev) for q in qs],
                           max_iter=10000, log_len=64)
    for C1, C2, p, q, T, info in zip(C1s, C2s, ps, qs, res.plans, res.infos()):
        G, ref = orc.gw_cg_np(C1, C2, p=p, q=q)
        assert info["status"] == "converged", info
        assert info["n_iter"] == ref["n_iter"]
        assert np.abs(T.cpu().numpy() - G).max() < 1e-9
        assert info["cost"] == pytest.approx(ref["gw_dist"], rel=1e-8, abs=1e-12)
    # the POT-form wrapper with weights and the unequal-group drop-in
    from otfuse import pot
    G1, log1 = gw.gromov_wasserstein(torch.as_tensor(C1s[1], device=dev), torch.as_tensor(C2s[1], device=dev),
                                     p=ps[1], q=qs[1], log=True)
    Gr, ref = orc.gw_cg_np(C1s[1], C2s[1], p=ps[1], q=qs[1])
    assert np.abs(G1.cpu().numpy() - Gr).max() < 1e-9
    Xd = {0: rng.standard_normal((12, 6)).astype(np.float32), 1: rng.standard_normal((20, 6)).astype(np.float32)}
    Yd = {0: rng.standard_normal((15, 6)).astype(np.float32), 1: rng.standard_normal((9, 6)).astype(np.float32)}
    Ts, _ = pot.get_coupling_gromov_pot((Xd, Yd))
    for k in Xd:
        assert Ts[k].shape == (len(Xd[k]), len(Yd[k]))
        np.testing.assert_allclose(Ts[k].sum(1), np.full(len(Xd[k]), 1.0 / len(Xd[k])), atol=1e-12)


def test_gw_cg_isometry(orc, dev):
    from otfuse import gw
    rng = np.random.default_rng(5)
    X = rng.standard_normal((50, 5))
    perm = rng.permutation(50)
    C1, _ = orc.pairwise_cost(X, X, metric="euclidean", zero_diag=True, scale_max=True)
    C2 = np.ascontiguousarray(C1[np.ix_(perm, perm)])
    G, log = gw.gromov_wasserstein(torch.as_tensor(C1, device=dev), torch.as_tensor(C2, device=dev),
                                   log=True)
    assert log["gw_dist"] == pytest.approx(0.0, abs=1e-12)
    assert (G.cpu().numpy().argmax(1) == np.argsort(perm)).all()


@pytest.mark.parametrize("n,m,eps", [(64, 64, 5e-3), (30, 50, 5e-3), (128, 100, 1e-2), (1, 4, 5e-3)])
def test_gw_entropic_vs_oracle(orc, dev, n, m, eps):
    from otfuse import gw
    (C1, _), = _label_costs(orc, [n], 24, 30, "sqeuclidean")
    (_, C2), = _label_costs(orc, [m], 24, 40, "sqeuclidean")
    P, info = gw.entropic_gromov_wasserstein_ott(torch.as_tensor(C1, device=dev),
                                                 torch.as_tensor(C2, device=dev), eps,
                                                 max_iterations=2000)
    Pr, ref = orc.gw_entropic(C1, C2, eps)
    assert info["n_iter"] == ref["n_iters"]
    assert info["converged"] == ref["converged"]
    assert info["converged_inner"] == ref["converged_inner"]
    assert nrel(P.cpu().numpy(), Pr) < 1e-4
    assert info["cost"] == pytest.approx(ref["reg_gw_cost"], rel=1e-6, abs=1e-9)


def test_gw_entropic_labelled_vs_oracle(orc, dev):
    from otfuse import gw
    (C1, C2), = _label_costs(orc, [60], 24, 50, "sqeuclidean")
    la = np.array([0] * 35 + [1] * 25, np.int32)
    lb = np.array([1] * 25 + [0] * 35, np.int32)
    P, info = gw.entropic_gromov_wasserstein_ott(torch.as_tensor(C1, device=dev),
                                                 torch.as_tensor(C2, device=dev), 1e-2,
                                                 labels_a=la, labels_b=lb, max_iterations=2000)
    Pr, ref = orc.gw_entropic(C1, C2, 1e-2, labels_a=la, labels_b=lb)
    Pn = P.cpu().numpy()
    assert Pn[np.not_equal.outer(la, lb)].max() == 0.0
    assert info["n_iter"] == ref["n_iters"]
    assert nrel(Pn, Pr) < 1e-4


def test_get_coupling_gromov_pot_dropin(orc, dev):
    """nojax per-epoch flow: grouped features -> GW per label -> feature coupling."""
    from otfuse import pot
    from otfuse.fusion import group_features_by_label
    X, Y, lab = _emb(120, 64, 77)
    gm = group_features_by_label(lab, X, max_samples_per_label=48)
    gp = group_features_by_label(lab, Y, max_samples_per_label=48)
    Ts, log = pot.get_coupling_gromov_pot((gp, gm))
    assert list(Ts) == list(gp)
    for l in gp:
        C1, _ = orc.pairwise_cost(gp[l], gp[l], metric="euclidean", zero_diag=True, scale_max=True)
        C2, _ = orc.pairwise_cost(gm[l], gm[l], metric="euclidean", zero_diag=True, scale_max=True)
        G, _ = orc.gw_cg(C1, C2)
        assert Ts[l].dtype == np.float32 and "time" in log[l]
        assert np.abs(Ts[l] - G).max() < 1e-7
    Tf, _ = pot.get_feature_coupling_pot((gp, gm), Ts)
    assert Tf.shape == (64, 64) and np.isfinite(Tf).all()


def test_get_coupling_egw_ott_fixed_dropin(orc, dev):
    from otfuse import perturbot
    from otfuse.fusion import group_features_by_label
    X, Y, lab = _emb(100, 32, 78)
    gm = group_features_by_label(lab, X, max_samples_per_label=40)
    gp = group_features_by_label(lab, Y, max_samples_per_label=40)
    T, log = perturbot.get_coupling_egw_ott_fixed((gp, gm), eps=5e-3)
    for l in gp:
        C1, _ = orc.pairwise_cost(gp[l], gp[l], scale_max=True)
        C2, _ = orc.pairwise_cost(gm[l], gm[l], scale_max=True)
        Pr, ref = orc.gw_entropic(C1, C2, 5e-3)
        assert log[l]["n_iters_outer"] == ref["n_iters"]
        assert set(log[l]) >= {"n_iters_outer", "converged_inner", "converged_outer", "GW cost",
                               "time", "cost_time"}
        assert nrel(T[l], Pr) < 1e-4
    Tf, flog = perturbot.get_coupling_fot((gp, gm), T, eps=5e-3)
    assert Tf.shape == (32, 32) and np.isfinite(Tf).all()


def test_egw_labels_and_all_dropins(dev):
    from otfuse import perturbot
    X, Y, lab = _emb(80, 16, 79)
    Xd = {0: X[lab == 0][:30], 1: X[lab == 1][:30]}
    Yd = {0: Y[lab == 0][:30], 1: Y[lab == 1][:30]}
    T_dict, log = perturbot.get_coupling_egw_labels_ott((Xd, Yd), eps=1e-2)
    assert set(T_dict) == {0, 1} and T_dict[0].shape == (30, 30)
    assert abs(sum(t.sum() for t in T_dict.values()) - 1.0) < 1e-6
    T, log2 = perturbot.get_coupling_egw_all_ott((Xd, Yd), eps=1e-2)
    assert T.shape == (60, 60) and abs(T.sum() - 1.0) < 1e-6


@pytest.mark.parametrize("n,m,eps", [(64, 64, 5e-3), (30, 45, 1e-2), (1, 4, 5e-2), (100, 90, 2e-2)])
def test_gw_pgd_vs_oracle(orc, dev, n, m, eps):
    """POT entropic GW, solver='PGD' (perturbot match/gw.py:47-57): float64 device solve
    against the C restatement -- same outer iteration count and err log, plans to 1e-9."""
    from otfuse import gw
    (C1, _), = _label_costs(orc, [n], 24, 60)
    (_, C2), = _label_costs(orc, [m], 24, 70)
    T, log = gw.entropic_gromov_wasserstein(torch.as_tensor(C1, device=dev),
                                            torch.as_tensor(C2, device=dev), epsilon=eps,
                                            log=True)
    Tr, ref = orc.gw_pgd(C1, C2, eps)
    assert log["n_iter"] == ref["n_iter"]
    assert log["inner_iters"] == ref["inner_iters"]
    np.testing.assert_allclose(log["err"], ref["err"], rtol=1e-6, atol=1e-14)
    assert nrel(T.cpu().numpy(), Tr) < 1e-9
    assert log["gw_dist"] == pytest.approx(ref["gw_dist"], rel=1e-9, abs=1e-14)


def test_gw_pgd_batched_weighted(orc, dev):
    """Several problems in one launch, with non-uniform marginals."""
    from otfuse import gw
    rng = np.random.default_rng(9)
    probs = _label_costs(orc, [20, 33, 48], 16, 80)
    ps = [rng.random(c1.shape[0]) + 0.5 for c1, _ in probs]
    qs = [rng.random(c2.shape[0]) + 0.5 for _, c2 in probs]
    ps = [p / p.sum() for p in ps]
    qs = [q / q.sum() for q in qs]
    res = gw.solve_batched([torch.as_tensor(c1, device=dev) for c1, _ in probs],
                           [torch.as_tensor(c2, device=dev) for _, c2 in probs], gw.GW_PGD,
                           ps=[torch.as_tensor(p, device=dev) for p in ps],
                           qs=[torch.as_tensor(q, device=dev) for q in qs], max_iter=1000,
                           tol_abs=1e-9, eps=2e-2, sk_max_iter=1000, sk_inner=10,
                           sk_threshold=1e-9, log_len=128)
    for (C1, C2), p, q, T, info in zip(probs, ps, qs, res.plans, res.infos()):
        Tr, ref = orc.gw_pgd(C1, C2, 2e-2, a=p, b=q)
        assert info["n_iter"] == ref["n_iter"]
        assert nrel(T.cpu().numpy(), Tr) < 1e-9


def test_perturbot_pot_gw_dropins(orc, dev):
    """perturbot match/gw.py: get_coupling_gw_cg / get_coupling_egw per label, and the
    all-to-all forms (labels ignored), against the oracle on cdist / max costs."""
    from otfuse import perturbot
    X, Y, lab = _emb(90, 24, 81)
    Xd = {0: X[lab == 0][:30], 1: X[lab == 1][:30]}
    Yd = {0: Y[lab == 0][:30], 1: Y[lab == 1][:30]}
    Ts, log = perturbot.get_coupling_gw_cg((Xd, Yd))
    Te, loge = perturbot.get_coupling_egw((Xd, Yd), eps=1e-2)
    assert set(log) >= {"cost_time", "time", 0, 1} and set(loge) >= {"cost_time", "time", 0, 1}
    for l in (0, 1):
        C1, _ = orc.pairwise_cost(Xd[l], Xd[l], metric="euclidean", zero_diag=True, scale_max=True)
        C2, _ = orc.pairwise_cost(Yd[l], Yd[l], metric="euclidean", zero_diag=True, scale_max=True)
        G, ref = orc.gw_cg(C1, C2)
        assert np.abs(Ts[l] - G).max() < 1e-12
        assert log[l]["gw_dist"] == pytest.approx(ref["gw_dist"], rel=1e-9, abs=1e-13)
        Tr, refe = orc.gw_pgd(C1, C2, 1e-2)
        assert nrel(Te[l], Tr) < 1e-9
        assert len(loge[l]["err"]) == len(refe["err"])
    T, loga = perturbot.get_coupling_gw_all((Xd, Yd))
    assert T.shape == (60, 60) and abs(T.sum() - 1.0) < 1e-9 and "time" in loga
    T2, loga2 = perturbot.get_coupling_egw_all((Xd, Yd), eps=1e-2)
    assert T2.shape == (60, 60) and abs(T2.sum() - 1.0) < 1e-6 and "gw_dist" in loga2


@pytest.mark.parametrize("n,m,eps", [(40, 50, 1e-4), (64, 17, 2e-3)])
def test_gw_pgd_small_inner_break_vs_oracle(orc, dev, n, m, eps):
    """The <= 64-point inner solve (two-barrier small_sinkhorn_knopp) on problems whose
    kernel underflows (eps = 1e-4: zero columns of K^T u -> POT's revert-and-break) and on
    a ragged n != m shape: same outer / inner counts as the oracle, plans to 1e-9."""
    from otfuse import gw
    (C1, _), = _label_costs(orc, [n], 16, 90)
    (_, C2), = _label_costs(orc, [m], 16, 91)
    T, log = gw.entropic_gromov_wasserstein(torch.as_tensor(C1, device=dev),
                                            torch.as_tensor(C2, device=dev), epsilon=eps,
                                            log=True)
    Tr, ref = orc.gw_pgd(C1, C2, eps)
    assert log["n_iter"] == ref["n_iter"]
    assert log["inner_iters"] == ref["inner_iters"]
    Td = T.cpu().numpy()
    assert np.array_equal(np.isfinite(Td), np.isfinite(Tr))
    fin = np.isfinite(Tr)
    if fin.any() and np.abs(Tr[fin]).max() > 0:
        assert np.abs(Td[fin] - Tr[fin]).max() / np.abs(Tr[fin]).max() < 1e-9


def test_gw_past_1024_points_vs_oracle(orc, dev):
    """Groups past the former 1024-point cap (POT's GW has none): GwHuge keeps its
    vectors and the simplex tree in the workspace.  CG on 1030 x 40 (linear step: the
    network simplex) and the OTT entropic solver on 1040 x 60, against the oracle."""
    from otfuse import gw
    rng = np.random.default_rng(1030)
    A = rng.standard_normal((1030, 3))
    B = rng.standard_normal((40, 4))
    C1 = orc.pairwise_cost(A, A, metric="euclidean", zero_diag=True, scale_max=True)[0]
    C2 = orc.pairwise_cost(B, B, metric="euclidean", zero_diag=True, scale_max=True)[0]
    res = gw.solve_batched([torch.as_tensor(C1, device=dev)], [torch.as_tensor(C2, device=dev)],
                           gw.GW_CG, max_iter=10000, log_len=64)
    info = res.infos()[0]
    G, ref = orc.gw_cg_np(C1, C2)
    assert info["status"] == "converged", info
    assert info["n_iter"] == ref["n_iter"]
    assert np.abs(res.plans[0].cpu().numpy() - G).max() < 1e-9
    assert info["cost"] == pytest.approx(ref["gw_dist"], rel=1e-8, abs=1e-12)
    A = rng.standard_normal((1040, 3))
    B = rng.standard_normal((60, 3))
    C1 = orc.pairwise_cost(A, A, scale_max=True)[0]
    C2 = orc.pairwise_cost(B, B, scale_max=True)[0]
    P, info = gw.entropic_gromov_wasserstein_ott(torch.as_tensor(C1, device=dev),
                                                 torch.as_tensor(C2, device=dev), 1e-2,
                                                 max_iterations=2000)
    Pr, ref = orc.gw_entropic(C1, C2, 1e-2)
    assert info["n_iter"] == ref["n_iters"]
    assert info["converged"] == ref["converged"]
    assert nrel(P.cpu().numpy(), Pr) < 1e-4
    assert info["cost"] == pytest.approx(ref["reg_gw_cost"], rel=1e-6, abs=1e-9)
