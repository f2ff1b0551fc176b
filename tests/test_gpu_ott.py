"""OTT-flavour Sinkhorn (perturbot fot.py:124-148 -> OTT 0.6 lse-mode solver, restated):
the resident engine's scaling form (engine="resident", float64) against the log-domain
streaming passes and the oracle restatement (needs an MI355X).  Parity of the OTT flavour
itself is unpinned (OTT is absent); these tests pin the two device forms to each other."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def nrel(x, ref):
    x = np.asarray(x, dtype=np.float64)
    ref = np.asarray(ref, dtype=np.float64)
    return np.abs(x - ref).max() / np.abs(ref).max()


@pytest.mark.parametrize("n,m,eps,thr,iters", [(2048, 2048, 5e-3, 1e-3, 2000), (1000, 700, 0.05, 1e-6, 500),
                                              (300, 512, 0.01, 0.0, 95), (2048, 1500, 0.02, 1e-4, 300)])
def test_ott_resident_scaling_form_matches_log_passes(dev, n, m, eps, thr, iters):
    from otfuse import ops
    g = torch.Generator(device=dev).manual_seed(n + m)
    C = torch.rand(n, m, device=dev, generator=g, dtype=torch.float64) ** 2
    a = torch.rand(n, device=dev, generator=g, dtype=torch.float64) + 0.5
    a /= a.sum()
    b = torch.rand(m, device=dev, generator=g, dtype=torch.float64) + 0.5
    b /= b.sum()
    scale = C.max().reshape(1)
    kw = dict(max_iter=iters, stop_thr=thr, flavor="ott", cost_scale=scale, check_every=10)
    r0 = ops.sinkhorn(a, b, C, eps, engine="stream", **kw)
    r1 = ops.sinkhorn(a, b, C, eps, engine="resident", **kw)
    i0, i1 = r0.info(), r1.info()
    assert i1["engine_name"] == "resident"
    for k in ("niter", "status_name", "n_err", "last_good"):
        assert i0[k] == i1[k], k
    np.testing.assert_allclose(i1["err"], i0["err"], rtol=1e-7, atol=1e-12 * max(i0["err"] + [1.0]))
    assert nrel(r1.plan.cpu().numpy(), r0.plan.cpu().numpy()) < 1e-10
    # potentials f, g (units of the scaled cost)
    assert (r1.u - r0.u).abs().max().item() < 1e-9
    assert (r1.v - r0.v).abs().max().item() < 1e-9


def test_solve_ott_takes_the_resident_form_and_matches_oracle(orc, dev):
    """perturbot.solve_ott picks the scaling form for float64 max_cost solves; the plan
    and the iteration count match the oracle's lse-mode restatement."""
    from otfuse import perturbot
    rng = np.random.default_rng(3)
    M = rng.random((256, 200)) ** 2
    res, _ = perturbot.solve_ott(torch.as_tensor(M, device=dev), 5e-3)
    info = res.info()
    assert info["engine_name"] == "resident"
    n, m = M.shape
    Pr, _, _, info_r = orc.sinkhorn_log(np.full(n, 1.0 / n), np.full(m, 1.0 / m), M, 5e-3,
                                        max_iter=2000, threshold=1e-3, cscale=1.0 / M.max())
    assert info["niter"] + 1 == info_r["n_iters"]
    assert nrel(res.plan.cpu().numpy(), Pr) < 1e-9


def test_solve_ott_falls_back_to_log_passes_when_the_grid_is_not_co_resident(dev, monkeypatch):
    """The scaling form has no relay fallback (that one is POT-flavour): a resident
    OTT grid that cannot register (8 CUs held by a long gather solve on another stream,
    1-ms registration window) ends in OTF_SK_TIMEOUT, and solve_ott re-solves with the
    log-domain passes -- the same plan as an uncontended solve."""
    from otfuse import ops, perturbot
    g = torch.Generator(device=dev).manual_seed(5)
    M = torch.rand(2048, 2048, device=dev, generator=g, dtype=torch.float64) ** 2
    ref, _ = perturbot.solve_ott(M, 5e-3)
    assert ref.info()["engine_name"] == "resident"
    Cg = torch.rand(512, 512, device=dev, generator=g, dtype=torch.float64)
    ag = torch.full((512,), 1.0 / 512, device=dev, dtype=torch.float64)
    monkeypatch.setenv("OTF_REG_MS", "1")
    s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    torch.cuda.synchronize()
    with torch.cuda.stream(s1):
        blocker = ops.sinkhorn(ag, ag, Cg, 0.1, max_iter=40000, stop_thr=0.0, engine="gather",
                               want_plan=False)
    with torch.cuda.stream(s2):
        res, _ = perturbot.solve_ott(M, 5e-3)
    torch.cuda.synchronize()
    info = res.info()
    assert info["status_name"] in ("converged", "max_iter") and info["stalled"] == 0
    assert info["niter"] == ref.info()["niter"]
    assert nrel(res.plan.cpu().numpy(), ref.plan.cpu().numpy()) < 1e-9
    assert blocker.info()["status_name"] == "max_iter"
    if info["engine_name"] == "resident":
        pytest.skip("the blocker finished before the OTT launch: no contention to test")
