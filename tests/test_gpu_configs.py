"""BASELINE configs 3 and 4 at their real sizes against the oracle, plus the boundary
pieces added for them (needs an MI355X).

* Config 3 -- the per-epoch chain of MRI_PET_OT_OT_per_epoch_attn.py:940-960: 2 labels x
  64 samples of d = 2048 backbone features (depth >= 50: 512 x 4), per-label entropic GW
  (get_coupling_egw_ott_fixed), then get_coupling_fot on the 2048 x 2048 float64
  feature cost at eps = 5e-3; and the POT form of the same chain (get_feature_coupling_pot
  with the block-diagonal GW plans, MRI_PET_OT_nojax.py:1110-1111).  OTT is absent, so
  the OTT-flavour steps are checked against the oracle's restatements (parity unpinned);
  the POT step is pinned like F2/F4 (float64, 1e-9).
* Config 4 -- MRI_T1_T2_OT.py:708-745 with bf16 encoder outputs: the bf16 embeddings go
  through ot_alignment_loss natively (otf_feature_cost_ex reads bf16); the reference
  is the oracle on the bf16-rounded values upcast to float32 (what the reference's
  float32 NumPy arrays would hold).
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def nrel(x, ref):
    x = np.asarray(x, dtype=np.float64)
    ref = np.asarray(ref, dtype=np.float64)
    return np.abs(x - ref).max() / np.abs(ref).max()


def _emb(n, d, seed):
    from otfuse.synthetic import paired_embeddings
    return paired_embeddings(n, d, seed=seed)


@pytest.fixture(scope="module")
def config3(dev):
    """2 labels x 64 paired samples, d = 2048, and the device EGW plans."""
    from otfuse import perturbot
    pet, mri = {}, {}
    for k in range(2):
        X, Y, _ = _emb(64, 2048, 900 + k)
        mri[k], pet[k] = X, Y
    Ts, log = perturbot.get_coupling_egw_ott_fixed((pet, mri), eps=5e-3)
    return pet, mri, Ts, log


def test_config3_egw_per_label_vs_oracle(config3, orc):
    pet, mri, Ts, log = config3
    for k in pet:
        C1, _ = orc.pairwise_cost(pet[k], pet[k], scale_max=True)
        C2, _ = orc.pairwise_cost(mri[k], mri[k], scale_max=True)
        Pr, ref = orc.gw_entropic(C1, C2, 5e-3)
        assert log[k]["n_iters_outer"] == ref["n_iters"]
        assert nrel(Ts[k], Pr) < 1e-4


def test_config3_get_coupling_fot_2048_vs_oracle(config3, orc):
    """get_coupling_fot on the 2048^2 float64 feature cost (fot.py:108-134): normalised
    block-diagonal Ts, column-sum w1, OTT max-cost Sinkhorn at eps = 5e-3."""
    from otfuse import perturbot
    pet, mri, Ts, _ = config3
    Tv, log = perturbot.get_coupling_fot((pet, mri), Ts, eps=5e-3)
    assert Tv.shape == (2048, 2048) and np.isfinite(Tv).all()
    X = np.concatenate([pet[k] for k in pet])
    Y = np.concatenate([mri[k] for k in pet])
    Tfull = perturbot.mdict_to_matrix(Ts, np.repeat([0, 1], 64), np.repeat([0, 1], 64))
    Tfull = Tfull / Tfull.sum()
    M = orc.feature_cost(X, Y, Tfull, weights="fot")
    orc.set_threads(16)
    u = np.full(2048, 1.0 / 2048)
    Pr, _, _, info = orc.sinkhorn_log(u, u, M, 5e-3, max_iter=2000, threshold=1e-3,
                                      cscale=1.0 / M.max())
    assert nrel(Tv, Pr) < 1e-8
    np.testing.assert_allclose(Tv.sum(1), 1.0 / 2048, rtol=1e-6)


def test_config3_device_chain_matches_dropins(config3, dev):
    """per_epoch_coupling_device (compute_pet_to_mri_coupling on device tensors, e.g. the
    all-gathered shards) equals the NumPy drop-in chain get_coupling_egw_ott_fixed +
    get_coupling_fot on the same rows: interleaved labels are grouped in np.unique order,
    the first 64 of each kept."""
    from otfuse import perturbot
    pet, mri, Ts, _ = config3
    Tv_ref, _ = perturbot.get_coupling_fot((pet, mri), Ts, eps=5e-3)
    # interleave the two labels' rows and add rows beyond the 64-per-label cut
    rng = np.random.default_rng(3)
    extra = 10
    lab = np.concatenate([np.zeros(64 + extra, np.int64), np.ones(64 + extra, np.int64)])
    P = np.concatenate([pet[0], rng.random((extra, 2048), np.float32), pet[1],
                        rng.random((extra, 2048), np.float32)])
    Mr = np.concatenate([mri[0], rng.random((extra, 2048), np.float32), mri[1],
                         rng.random((extra, 2048), np.float32)])
    # rows of label 0 at even positions, label 1 at odd ones, each label's order kept
    perm = np.empty(len(lab), np.int64)
    perm[0::2] = np.arange(64 + extra)
    perm[1::2] = 64 + extra + np.arange(64 + extra)
    Tv, info = perturbot.per_epoch_coupling_device(
        torch.as_tensor(Mr[perm], device=dev), torch.as_tensor(P[perm], device=dev),
        torch.as_tensor(lab[perm], device=dev), eps=5e-3, max_per_label=64)
    assert Tv.is_cuda and tuple(Tv.shape) == (2048, 2048)
    assert nrel(Tv.cpu().numpy(), Tv_ref) < 1e-9
    assert info()["labels"] == [0, 1]


class _PairComm:
    """Two ranks of a world-2 communicator simulated in one process (one device): rank 1's
    all_reduce contribution is recorded, rank 0's call adds it -- the all-reduce(SUM) of
    otfuse.distributed.split_label_plans without a second process."""

    def __init__(self, rank, store):
        self.rank, self.nranks, self.store = rank, 2, store

    def all_reduce(self, t, op="sum"):
        if self.rank == 1:
            self.store.append(t.clone())
        else:
            t += self.store[0]
        return t


def test_config3_label_split_matches_unsplit(config3, dev):
    """Config 3's per-epoch chain with the per-label entropic GW split over two ranks
    (labels dealt round-robin, one all-reduce of the padded plan stack,
    otfuse.distributed.split_label_plans): every label's plan bit-identical to the
    single-rank solve, the PET->MRI feature plan to 1e-12."""
    from otfuse import distributed, perturbot
    pet, mri, _, _ = config3
    lab = np.repeat([0, 1], 64)
    P = torch.as_tensor(np.concatenate([pet[0], pet[1]]), device=dev)
    M = torch.as_tensor(np.concatenate([mri[0], mri[1]]), device=dev)
    L = torch.as_tensor(lab, device=dev)
    Tv1, info1 = perturbot.per_epoch_coupling_device(M, P, L, eps=5e-3)
    pets = [P[:64].float(), P[64:].float()]
    mris = [M[:64].float(), M[64:].float()]
    ref, _ = perturbot.egw_label_plans(pets, mris, 5e-3)
    store = []
    solve = lambda p, m: perturbot.egw_label_plans(p, m, 5e-3)  # noqa: E731
    distributed.split_label_plans(pets, mris, _PairComm(1, store), solve)
    plans, _ = distributed.split_label_plans(pets, mris, _PairComm(0, store), solve)
    for T, R in zip(plans, ref):
        assert torch.equal(T, R)
    # the whole chain at rank 0, rank 1's share (label 1) as its all-reduce contribution
    other = torch.zeros((2, 64, 64), dtype=torch.float64, device=dev)
    other[1] = ref[1]
    Tv2, _ = distributed.per_epoch_coupling_split(M, P, L, _PairComm(0, [other]), eps=5e-3)
    # the same plans feed the same OTT solve (its column sums use float atomics, so two
    # runs agree to rounding, not bitwise)
    assert nrel(Tv1.cpu().numpy(), Tv2.cpu().numpy()) < 1e-12


def test_config3_pot_form_2048_vs_oracle(config3, orc):
    """POT form of the per-epoch chain: get_feature_coupling_pot with the block-diagonal
    GW plans (MRI_PET_OT_nojax.py:91-145), 2048^2 float64, eps = 5e-3, 2000 iterations,
    stopThr 1e-9 -- against the oracle at 1e-9 with the same iteration count."""
    from otfuse import pot
    pet, mri, Ts, _ = config3
    Tf, _ = pot.get_feature_coupling_pot((pet, mri), Ts, eps=5e-3)
    X = np.concatenate([pet[k] for k in sorted(pet)])
    Y = np.concatenate([mri[k] for k in sorted(pet)])
    Tbd = orc.block_diag_ts(Ts, pet, mri)
    M = orc.feature_cost(X, Y, Tbd)
    orc.set_threads(16)
    u = np.full(2048, 1.0 / 2048)
    Pr, *_ = orc.sinkhorn_knopp(u, u, M, 5e-3, 2000, 1e-9)
    assert Tf.shape == (2048, 2048)
    assert nrel(Tf, Pr) < 1e-9


@pytest.mark.parametrize("d", [512, 2048])
def test_config4_bf16_embeddings_through_ot_alignment_loss(orc, dev, d):
    from otfuse import ops
    from otfuse.fusion import cosine_loss, ot_alignment_loss
    X, Y, _ = _emb(8, d, 40 + d)
    mri = torch.as_tensor(X, device=dev).to(torch.bfloat16).requires_grad_(True)
    pet = torch.as_tensor(Y, device=dev).to(torch.bfloat16).requires_grad_(True)
    loss, ot_mri, T = ot_alignment_loss(mri, pet, eps=1e-2)
    # native bf16 read == the same kernels on the upcast values, bit for bit
    ts = torch.full((8,), 1.0 / 8, dtype=torch.float64, device=dev)
    assert torch.equal(ops.feature_cost(mri.detach(), pet.detach(), ts_diag=ts),
                       ops.feature_cost(mri.detach().float(), pet.detach().float(), ts_diag=ts))
    # oracle: the reference's chain on the bf16-rounded float32 arrays
    Xr = mri.detach().float().cpu().numpy()
    Yr = pet.detach().float().cpu().numpy()
    M = orc.feature_cost(Xr, Yr, np.eye(8) / 8)
    u = np.full(d, 1.0 / d)
    P, *_ = orc.sinkhorn_knopp(u, u, M, 1e-2, 2000, 1e-9)
    Tn = np.nan_to_num(P.astype(np.float32), nan=1e-8)
    rs = Tn.sum(1, keepdims=True)
    Tn = Tn / np.where(rs == 0, 1e-8, rs)
    np.testing.assert_allclose(T.cpu().numpy(), Tn, rtol=1e-4, atol=1e-9)
    Zr = Yr @ Tn.T
    np.testing.assert_allclose(ot_mri.detach().cpu().numpy(), Zr, rtol=1e-4, atol=1e-6)
    lr = float(cosine_loss(torch.from_numpy(Xr), torch.from_numpy(Zr)))
    assert abs(float(loss) - lr) < 1e-4
    loss.backward()
    assert mri.grad.dtype == torch.bfloat16 and pet.grad.dtype == torch.bfloat16
    assert torch.isfinite(mri.grad.float()).all() and torch.isfinite(pet.grad.float()).all()


# ------------------------------------------------------------------ boundary pieces
def test_fused_postprocess_apply_vs_torch(dev):
    from otfuse import ops
    g = torch.Generator(device=dev).manual_seed(5)
    T = torch.rand(300, 200, dtype=torch.float64, device=dev, generator=g)
    T[3, 7] = float("nan")
    T[10] = 0
    Z = torch.randn(20, 200, device=dev, generator=g)          # B = 20 > one 16-row block
    out, Tn = ops.plan_postprocess_apply(T, Z)
    Tr = T.float()
    Tr = torch.where(torch.isnan(Tr), torch.full_like(Tr, 1e-8), Tr)
    rs = Tr.sum(1, keepdim=True)
    Tr = Tr / torch.where(rs == 0, torch.full_like(rs, 1e-8), rs)
    assert torch.allclose(Tn, Tr, rtol=1e-6, atol=0)
    assert torch.allclose(out, Z @ Tr.t(), rtol=1e-4, atol=1e-5)
    # autograd: d/dZ of sum(out * G) = G @ Tn
    Zg = Z.clone().requires_grad_(True)
    o, _ = ops.PostprocessApply.apply(Zg, T)
    G = torch.randn_like(o)
    (o * G).sum().backward()
    assert torch.allclose(Zg.grad, G @ Tr, rtol=1e-4, atol=1e-5)


def test_nan_loss_contributes_no_gradient(dev):
    """MRI_PET_OT_nojax.py:724-725: a NaN OT loss is replaced by a constant 0."""
    from otfuse.fusion import ot_alignment_loss
    X, Y, _ = _emb(8, 64, 3)
    mri = torch.as_tensor(X, device=dev).requires_grad_(True)
    pet = torch.as_tensor(Y, device=dev).requires_grad_(True)
    T = torch.full((64, 64), float("nan"), device=dev)        # a given (bad) plan
    loss, _, _ = ot_alignment_loss(mri, pet, T_feature_pet2mri=T)
    assert float(loss) == 0.0
    loss.backward()
    assert torch.equal(mri.grad, torch.zeros_like(mri)) and torch.equal(pet.grad, torch.zeros_like(pet))


@pytest.mark.parametrize("dt,n,m", [(torch.float32, 2000, 3000), (torch.float64, 700, 450),
                                    (torch.float32, 37, 5), (torch.float32, 200, 9000)])
def test_deterministic_mode_is_bitwise_reproducible(orc, dev, dt, n, m):
    from otfuse import ops
    rng = np.random.default_rng(n)
    C = rng.random((n, m))
    a = np.full(n, 1.0 / n)
    b = np.full(m, 1.0 / m)
    Ct, at, bt = (torch.as_tensor(x, device=dev, dtype=dt) for x in (C, a, b))
    plans = []
    # engines that are fixed-order by construction: gather (small problems), mesh (float32,
    # 4..64 row tiles x <= 8 column tiles); the sweep engine's deterministic mode otherwise
    want = ("gather" if m <= 512 else "mesh" if dt == torch.float32 and n >= 385 and m <= 4096
            else "sweep")
    for _ in range(3):
        res = ops.sinkhorn(at, bt, Ct, 0.05, max_iter=80, stop_thr=0.0, deterministic=True)
        assert res.info()["engine_name"] == want
        plans.append(res.plan.clone())
    assert torch.equal(plans[0], plans[1]) and torch.equal(plans[0], plans[2])
    Pr, *_ = orc.sinkhorn_knopp(a, b, C, 0.05, 80, 0.0)
    assert nrel(plans[0].cpu().numpy(), Pr) < (1e-4 if dt == torch.float32 else 1e-10)
    with pytest.raises(Exception):
        ops.sinkhorn(at, bt, Ct, 0.05, max_iter=80, deterministic=True, engine="tiled")


def test_eot_and_leot_dropins_vs_oracle(orc, dev):
    """get_coupling_eot_ott / get_coupling_leot_ott (perturbot ott_egwl.py:299-454):
    PointCloud(x, y, scale_cost="max_cost") + OTT Sinkhorn, against the oracle's lse
    restatement on the same max-scaled cost (parity unpinned: OTT absent)."""
    from otfuse import ops, perturbot
    X, Y, lab = _emb(96, 48, 61)
    xd = {0: X[lab == 0][:40], 1: X[lab == 1][:40]}
    yd = {0: Y[lab == 0][:40], 1: Y[lab == 1][:40]}

    def ref(Xs, Xt):
        C, cmax = ops.pairwise_cost(torch.as_tensor(Xs, device=dev), torch.as_tensor(Xt, device=dev))
        Cs = ops.scale_inplace(C.double(), cmax).cpu().numpy()
        n, m = Cs.shape
        P, f, g, info = orc.sinkhorn_log(np.full(n, 1.0 / n), np.full(m, 1.0 / m), Cs, 5e-3)
        return P, info

    T, log = perturbot.get_coupling_eot_ott((xd, yd), eps=5e-3)
    Xs = np.concatenate([xd[k] for k in xd])
    Xt = np.concatenate([yd[k] for k in xd])
    Pr, info = ref(Xs, Xt)
    assert T.shape == (len(Xs), len(Xt)) and log["n_iters_outer"] == info["n_iters"]
    assert nrel(T, Pr) < 1e-9
    Td, logs = perturbot.get_coupling_leot_ott((xd, yd), eps=5e-3)
    for k in xd:
        Pr, info = ref(xd[k], yd[k])
        assert logs[k]["n_iters_outer"] == info["n_iters"]
        assert nrel(Td[k], Pr) < 1e-9


@pytest.mark.parametrize("engine,n,dt", [("tiled", 4096, torch.float32), ("mesh", 4096, torch.float32),
                                         ("gather", 512, torch.float64), ("mesh", 1024, torch.float64)])
def test_persistent_engine_beside_a_concurrent_persistent_grid(dev, monkeypatch, engine, n, dt):
    """A persistent solve launched together with a full-grid persistent solve on another
    stream (the r02 stall scenario: e.g. RCCL kernels holding CUs) cannot always become
    co-resident.  It must never hang, never return a silently wrong plan and -- with the
    relay fallback queued behind every persistent launch -- never lose the
    answer: each solve ends max_iter with the reference plan, either from its engine or
    from the fallback (info fallback = 1, counted in otf_sinkhorn_fallback_count)."""
    from otfuse import _lib as L, ops
    monkeypatch.setenv("OTF_STALL_MS", "300")
    g = torch.Generator(device=dev).manual_seed(9)
    Cb = torch.rand(4096, 4096, device=dev, generator=g)
    ab = torch.full((4096,), 1.0 / 4096, device=dev)
    C = Cb[:n, :n].to(dt).contiguous()
    a = torch.full((n,), 1.0 / n, device=dev, dtype=dt)
    ref = ops.sinkhorn(a, a, C, 0.1, max_iter=30, stop_thr=0.0, engine="stream").plan
    refb = ops.sinkhorn(ab, ab, Cb, 0.1, max_iter=30, stop_thr=0.0, engine="stream").plan
    s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    torch.cuda.synchronize()
    blocker_engine = "mesh" if engine == "gather" else engine
    with torch.cuda.stream(s1):
        blk = ops.sinkhorn(ab, ab, Cb, 0.1, max_iter=30, stop_thr=0.0, engine=blocker_engine)
    with torch.cuda.stream(s2):
        res = ops.sinkhorn(a, a, C, 0.1, max_iter=30, stop_thr=0.0, engine=engine)
    torch.cuda.synchronize()
    for r, rp in ((blk, refb), (res, ref)):
        info = r.info()                       # no OtfError: the fallback finished it
        assert info["status_name"] == "max_iter" and info["stalled"] == 0
        assert (r.plan - rp).abs().max() / rp.abs().max() < 1e-5
    import ctypes
    cnt = ctypes.c_uint64()
    L.check(L.lib().otf_sinkhorn_fallback_count(ctypes.byref(cnt)), "fallback_count")
    assert cnt.value >= int(blk.info()["fallback"]) + int(res.info()["fallback"])
    # the device is healthy afterwards
    r = ops.sinkhorn(a, a, C, 0.1, max_iter=30, stop_thr=0.0, engine=engine)
    assert r.info()["status_name"] == "max_iter" and r.info()["fallback"] == 0
    assert (r.plan - ref).abs().max() / ref.abs().max() < 1e-5


@pytest.mark.parametrize("dt", [torch.float32, torch.float64])
def test_solo_fallback_when_registration_cannot_complete(dev, monkeypatch, dt):
    """Force the fallback: a long gather solve (its XCC team holds 8 CUs for ~0.1 s) on
    one stream, then a mesh solve (a whole grid, one workgroup per CU) on another with a
    1-ms registration window: 8 of its workgroups cannot start, its registration gives
    up, the late workgroups see the give-up word and leave, and the relay fallback
    queued behind it returns the right plan (info fallback = 1)."""
    from otfuse import ops
    monkeypatch.setenv("OTF_REG_MS", "1")
    g = torch.Generator(device=dev).manual_seed(3)
    C = torch.rand(4096, 4096, device=dev, generator=g).to(dt)
    a = torch.full((4096,), 1.0 / 4096, device=dev, dtype=dt)
    Cg = torch.rand(512, 512, device=dev, generator=g, dtype=torch.float64)
    ag = torch.full((512,), 1.0 / 512, device=dev, dtype=torch.float64)
    ref = ops.sinkhorn(a, a, C, 0.1, max_iter=20, stop_thr=0.0, engine="stream").plan
    s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    torch.cuda.synchronize()
    with torch.cuda.stream(s1):
        blocker = ops.sinkhorn(ag, ag, Cg, 0.1, max_iter=40000, stop_thr=0.0, engine="gather",
                               want_plan=False)
    with torch.cuda.stream(s2):
        res = ops.sinkhorn(a, a, C, 0.1, max_iter=20, stop_thr=0.0, engine="mesh")
    torch.cuda.synchronize()
    info = res.info()
    assert info["status_name"] == "max_iter" and info["niter"] == 19 and info["stalled"] == 0
    assert (res.plan - ref).abs().max() / ref.abs().max() < 1e-5
    assert blocker.info()["status_name"] == "max_iter"
    if info["fallback"] != 1:
        pytest.skip("the blocker finished before the mesh launch: no contention to test")


@pytest.mark.parametrize("engine,n,m,dt,iters", [("tiled", 4096, 4096, torch.float32, 20000),
                                                 ("mesh", 4096, 4096, torch.float32, 40000),
                                                 ("mesh", 4096, 4096, torch.float64, 12000),
                                                 ("mesh", 4096, 4096, torch.float64, 30000),
                                                 ("resident", 512, 512, torch.float64, 30000),
                                                 ("gather", 512, 512, torch.float64, 60000),
                                                 ("sweep", 1024, 8192, torch.float32, 20000)])
def test_long_persistent_solve_outlives_the_stall_limit(dev, monkeypatch, engine, n, m, dt, iters):
    """The stall deadline is re-armed at every completed barrier: a solve that runs far
    longer than OTF_STALL_MS but keeps making progress finishes normally."""
    import time
    from otfuse import ops
    monkeypatch.setenv("OTF_STALL_MS", "40")
    g = torch.Generator(device=dev).manual_seed(4)
    C = torch.rand(n, m, device=dev, generator=g).to(dt)
    a = torch.full((n,), 1.0 / n, device=dev, dtype=dt)
    b = torch.full((m,), 1.0 / m, device=dev, dtype=dt)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    res = ops.sinkhorn(a, b, C, 0.5, max_iter=iters, stop_thr=0.0, engine=engine, want_plan=False)
    info = res.info()
    elapsed = time.perf_counter() - t0
    assert info["engine_name"] == engine
    assert info["status_name"] == "max_iter" and not info["stalled"]
    assert elapsed > 0.04 * 1.5     # the solve really outlived the stall limit


@pytest.mark.parametrize("engine,n,dt,reg,shift,tol", [
    ("mesh", 2048, torch.float32, 0.1, False, 1e-5),
    ("mesh", 2048, torch.float32, 5e-3, True, 1e-4),     # the shifted kernel's relay
    ("sweep", 4096, torch.float16, 0.1, False, 1e-4),    # fp16 cost storage, float32 compute
    ("tiled", 4096, torch.float32, 0.1, False, 1e-5),
    ("gather", 512, torch.float64, 0.05, False, 1e-9),
    ("resident", 512, torch.float64, 0.05, False, 1e-9),
    ("mesh", 4096, torch.float64, 0.1, False, 1e-9)])
def test_forced_relay_fallback_matches_the_engine(dev, monkeypatch, engine, n, dt, reg, shift, tol):
    """Every persistent engine's registration give-up (forced, OTF_FORCE_REG_GIVEUP=1: the
    launch is replaced by the give-up) hands the whole solve to the relay fallback, whose
    ticketed streaming passes must give the engine's own POT result: the plan within the
    compute precision's tolerance, the same status and iteration count (float64: POT's
    converged stop), info fallback = 1 -- for the float32 mesh (plain and
    shifted kernel), the sweep engine on an fp16 cost, the tiled, gather and resident
    engines and the float64 mesh on a float64 cost."""
    from otfuse import ops
    g = torch.Generator(device=dev).manual_seed(n + 31)
    X = torch.randn(n, 48, device=dev, generator=g, dtype=torch.float64)
    C = torch.cdist(X, X * 0.9 + 0.1) ** 2
    C = (C / C.max()).to(dt)
    cdt = torch.float64 if dt == torch.float64 else torch.float32
    a = torch.full((n,), 1.0 / n, device=dev, dtype=cdt)
    # float64: POT's converged stop (checked every 10 iterations); float32: a fixed count (its
    # error near a threshold may round either way between two summation orders)
    kw = dict(max_iter=300, stop_thr=1e-7, engine=engine) if dt == torch.float64 else \
        dict(max_iter=100, stop_thr=0.0, engine=engine)
    if shift:
        kw["shift"] = True
    r0 = ops.sinkhorn(a, a, C, reg, **kw)
    i0 = r0.info()
    assert i0["fallback"] == 0
    monkeypatch.setenv("OTF_FORCE_REG_GIVEUP", "1")
    r1 = ops.sinkhorn(a, a, C, reg, **kw)
    i1 = r1.info()
    assert i1["fallback"] == 1 and i1["engine_name"] == "stream" and i1["stalled"] == 0
    assert i1["status_name"] == i0["status_name"] and i1["niter"] == i0["niter"]
    assert ((r1.plan.double() - r0.plan.double()).abs().max() / r0.plan.double().abs().max()).item() < tol
