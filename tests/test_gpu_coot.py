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


def _coot_data(seed):
    rng = np.random.default_rng(seed)
    Xd = {0: rng.random((14, 10)).astype(np.float32), 1: rng.random((17, 10)).astype(np.float32)}
    Yd = {0: rng.random((15, 7)).astype(np.float32), 1: rng.random((12, 7)).astype(np.float32)}
    return Xd, Yd


@pytest.mark.parametrize("algo,algo2", [("emd", "sinkhorn"), ("sinkhorn", "emd")])
def test_cotl_mixed_solvers_vs_oracle(orc, dev, algo, algo2):
    """cotl_numpy with algo != algo2 (cot_labels.py:177-199): each stage on its own
    solver, same BCD iterations and plans as the oracle."""
    from otfuse import perturbot
    Xd, Yd = _coot_data(2)
    Ts, Tv, cost, log = perturbot.cotl_numpy(Xd, Yd, niter=200, algo=algo, algo2=algo2, reg=5e-2,
                                             log=True)
    Tr, Tvr, cost_r, log_r = orc.cotl_np(Xd, Yd, eps=5e-2, niter=200, algo=algo, algo2=algo2)
    assert len(log["cost"]) == len(log_r["cost"])
    np.testing.assert_allclose(log["cost"], log_r["cost"], rtol=1e-6)
    assert nrel(Tv, Tvr) < 1e-6
    for k in Xd:
        assert nrel(Ts[k], Tr[k]) < 1e-6


def test_cotl_sample_cost_prior_vs_oracle(orc, dev):
    """C_lin (cot_labels.py:175-176) added to every label's sample cost."""
    from otfuse import perturbot
    Xd = {0: np.random.default_rng(3).random((12, 8)).astype(np.float32),
          1: np.random.default_rng(4).random((12, 8)).astype(np.float32)}
    Yd = {0: np.random.default_rng(5).random((12, 6)).astype(np.float32),
          1: np.random.default_rng(6).random((12, 6)).astype(np.float32)}
    C_lin = np.random.default_rng(7).random((12, 12)) * 0.5
    Ts, Tv, cost, log = perturbot.cotl_numpy(Xd, Yd, niter=200, algo="emd", algo2="emd",
                                             C_lin=C_lin, log=True)
    Tr, Tvr, cost_r, log_r = orc.cotl_np(Xd, Yd, niter=200, algo="emd", algo2="emd", C_lin=C_lin)
    np.testing.assert_allclose(log["cost"], log_r["cost"], rtol=1e-9)
    for k in Xd:
        assert np.abs(Ts[k] - Tr[k]).max() < 1e-9


def test_random_gamma_init_device_vs_golden(golden, dev):
    """random_gamma_init (utils.py:118-122): the reference's Beta draw from NumPy's
    generator + the reference's own scaling loop (F5) -- the device scaling of the same
    draw matches it."""
    from otfuse import perturbot
    f = golden("f5_random_gamma_init.npz")
    for tag in ("a", "b"):
        np.random.seed(int(f[f"seed_{tag}"]))
        P = perturbot.random_gamma_init(f[f"p_{tag}"], f[f"q_{tag}"])
        assert nrel(P, f[f"plan_{tag}"]) < 1e-10


def test_cotl_random_init_vs_oracle(orc, dev):
    """cotl_numpy(random_init=True): the Ts / Tv initial couplings drawn in the
    reference's order (labels, then Tv) change the first sample costs; same BCD."""
    from otfuse import perturbot
    Xd, Yd = _coot_data(8)
    np.random.seed(21)
    Ts, Tv, cost, log = perturbot.cotl_numpy(Xd, Yd, niter=200, algo="emd", algo2="emd",
                                             random_init=True, log=True)
    np.random.seed(21)
    Tr, Tvr, cost_r, log_r = orc.cotl_np(Xd, Yd, niter=200, algo="emd", algo2="emd",
                                         random_init=True)
    np.testing.assert_allclose(log["cost"], log_r["cost"], rtol=1e-8)
    assert np.abs(Tv - Tvr).max() < 1e-8


def test_fot_numpy_random_init(dev):
    """fot_numpy(random_init=True) (fot.py:115-116): only the first delta changes; the
    feature plan is the one of the uniform start."""
    from otfuse import perturbot
    rng = np.random.default_rng(9)
    X = rng.random((20, 12)).astype(np.float32)
    Y = rng.random((20, 9)).astype(np.float32)
    Ts = np.eye(20) / 20
    T0, c0 = perturbot.fot_numpy(X, Y, Ts, reg2=5e-2, verbose=False)
    np.random.seed(4)
    T1, c1 = perturbot.fot_numpy(X, Y, Ts, reg2=5e-2, verbose=False, random_init=True)
    assert np.abs(T1 - T0).max() < 1e-14 and c1 == c0
