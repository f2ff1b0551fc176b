"""Drop-ins for the perturbot.match transport-plan API (OTT-flavour Sinkhorn).

Mirrors (names, arguments, return conventions):

* ``fot_numpy`` / ``get_coupling_fot`` -> perturbot/perturbot/match/fot.py:14-220
  (called per batch at MRI_PET_OT.py:677-681 and per epoch at
  MRI_PET_OT_OT_per_epoch_attn.py:959, baseline_models_fusion.py:167);
* ``get_coupling_eot_ott`` / ``get_coupling_leot_ott`` -> perturbot/perturbot/match/ott_egwl.py:299-454;
* ``gw_cg`` / ``egw_pgd`` / ``gw_all`` / ``egw_all`` and their ``get_coupling_gw_cg`` /
  ``get_coupling_egw`` / ``get_coupling_gw_all`` / ``get_coupling_egw_all`` wrappers ->
  perturbot/perturbot/match/gw.py:7-137 (POT GW: exact CG and entropic PGD; the costs
  are cdist / max, every label problem of a call in one device launch);
* ``mdict_to_matrix`` -> semantics of baseline_models_fusion.py:233-239 (the module
  ``perturbot.utils`` it stands in for is missing from the reference tree).

The linear solves are OTT-jax 0.6.0 ``linear.solve(Geometry(M, epsilon=eps,
scale_cost="max_cost"))`` semantics — lse-mode Sinkhorn, f = g = 0 start, g-update
then f-update, L1 marginal error after every 10 updates against threshold 1e-3,
max 2000 iterations — run by the HIP solver in float64 (the reference enables
JAX x64, MRI_PET_OT.py:23).  OTT is not installed in the build container, so this
flavour's parity is UNPINNED (tests check marginals and agreement with the oracle's
log-domain restatement).
"""
from __future__ import annotations

import time
import warnings
from typing import Dict, Tuple, Union
from numbers import Number

import numpy as np
import torch

from . import ops
from .pot import _device

OTT_THRESHOLD = 1e-3
OTT_MAX_ITER = 2000
OTT_INNER = 10


def mdict_to_matrix(M_dict, source_labels, target_labels):
    """Per-label blocks -> full matrix over label masks (baseline_models_fusion.py:233-239)."""
    source_labels = np.asarray(source_labels)
    target_labels = np.asarray(target_labels)
    Mtot = np.zeros((len(source_labels), len(target_labels)))
    for l, M in M_dict.items():
        Mtot[np.ix_(np.where(source_labels == l)[0], np.where(target_labels == l)[0])] = M
    return Mtot


# float64 OTT solves with scale_cost="max_cost" run in the resident engine's scaling form
# (one persistent launch: U = exp(f / eps), V = exp(g / eps)) when 1 / eps keeps
# K = exp(-C / (eps max C)) and the scalings far inside float64's range; else (and when
# that engine does not take the shape) the log-domain streaming passes.
OTT_SCALING_MAX = 300.0


def solve_ott(M: torch.Tensor, eps: float, scale_cost: str | None = "max_cost",
              a: torch.Tensor | None = None, b: torch.Tensor | None = None,
              threshold: float = OTT_THRESHOLD, max_iterations: int = OTT_MAX_ITER,
              sync_every: int = 50):
    """``ott.solvers.linear.solve(Geometry(cost_matrix=M, epsilon=eps, scale_cost=...))``
    on the device.  Returns ``(SinkhornResult, cost_scale or None)``."""
    n, m = M.shape
    dt = M.dtype
    if a is None:
        a = ops.uniform(n, dt, M.device)
    if b is None:
        b = ops.uniform(m, dt, M.device)
    scale = None
    if scale_cost == "max_cost":
        scale = M.max().reshape(1)
    elif scale_cost not in (None, 1.0):
        raise NotImplementedError(f"scale_cost={scale_cost!r}")
    kw = dict(max_iter=max_iterations, stop_thr=threshold, flavor="ott", cost_scale=scale,
              check_every=OTT_INNER, sync_every=sync_every, want_plan=True)
    if dt == torch.float64 and scale_cost == "max_cost" and 1.0 / float(eps) <= OTT_SCALING_MAX:
        # the scaling form's range contract holds for 0 <= M / max M <= 1 only: a cost with
        # negative entries (COOT-L with a user C_lin) or max M <= 0 takes the passes
        mn, mx = (float(t) for t in torch.aminmax(M))
        if mn >= 0.0 and mx > 0.0:
            try:
                res = ops.sinkhorn(a, b, M, float(eps), engine="resident", **kw)
                # a timeout (grid not co-resident) or a break of the scaling form (a U or V
                # out of float64's range, which OTT's lse mode does not hit): the passes
                if res.info_dev[3].item() not in (ops.L.SK_TIMEOUT, ops.L.SK_NUMERICAL_BREAK):
                    return res, scale
            except ops.L.OtfError:
                pass                          # shape not taken by the resident engine
    res = ops.sinkhorn(a, b, M, float(eps), **kw)
    return res, scale


def random_gamma_init_device(p, q, numItermax: int = 1000, stopThr: float = 1e-9) -> torch.Tensor:
    """perturbot ``random_gamma_init`` (utils.py:118-122) with the scaling on the device.

    The random matrix is the reference's draw, from NumPy's global generator: a dense
    ``scipy.sparse.random(len(p), len(q), density=1)`` with Beta(0.1, 0.1) entries (the
    reference reads it with ``.A``, which SciPy >= 1.14 removed; ``.toarray()`` is the
    same array).  ``sinkhorn_scaling(p, q, S)`` is POT's scaling iteration on the GIVEN
    kernel S with the squared marginal error: the POT-flavour device Sinkhorn on the
    cost -log S at reg 1 (K = exp(log S)), err_squared.  Returns the float64 plan on the
    device."""
    from scipy import stats
    from scipy.sparse import random as sprandom
    p = np.asarray(p, dtype=np.float64)
    q = np.asarray(q, dtype=np.float64)
    S = sprandom(len(p), len(q), density=1, data_rvs=stats.beta(1e-1, 1e-1).rvs).toarray()
    dev = _device()
    C = -torch.log(torch.as_tensor(S, dtype=torch.float64, device=dev))
    res = ops.sinkhorn(torch.as_tensor(p, device=dev), torch.as_tensor(q, device=dev), C, 1.0,
                       max_iter=int(numItermax), stop_thr=float(stopThr), flavor="pot",
                       err_squared=True, want_plan=True)
    return res.plan


def random_gamma_init(p, q, **kwargs) -> np.ndarray:
    """Drop-in for perturbot ``random_gamma_init`` (utils.py:118-122): a random coupling
    with marginals p, q (NumPy float64)."""
    kw = {k: kwargs[k] for k in ("numItermax", "stopThr") if k in kwargs}
    return ops.to_host(random_gamma_init_device(p, q, **kw))


def fot_numpy(X1, X2, Ts, v1=None, v2=None, niter=10, algo="emd", reg=0, algo2="emd", reg2=0,
              verbose=True, log=False, random_init=False, C_lin=None):
    """Feature OT given a fixed sample coupling Ts (perturbot fot.py:14-152).

    With Ts fixed the BCD cost M = constC - hC1 Ts hC2^T is constant, so the reference
    solves the same OTT problem twice and stops at i = 1 on |cost - cost_old| < 1e-7
    (fot.py:145).  The device solver runs it once; ``log['cost']`` repeats the value
    as the reference's two iterations would.  Note the reference's weights:
    ``Ts /= Ts.sum(); w1 = Ts.sum(axis=0); w2 = Ts.sum(axis=1)`` (fot.py:108-110).
    """
    dev = _device()
    Ts = np.asarray(Ts, dtype=np.float64)
    Ts = Ts / Ts.sum()
    Tv_init = None
    if random_init:
        # fot.py:115-116: the only effect is the first iteration's delta (the BCD still
        # stops at i = 1 on the cost test); the draw consumes NumPy's generator as there
        d1, d2_ = np.asarray(X1).shape[1], np.asarray(X2).shape[1]
        Tv_init = random_gamma_init_device(np.ones(d1) / d1 if v1 is None else v1,
                                           np.ones(d2_) / d2_ if v2 is None else v2)
    Xd = torch.as_tensor(np.asarray(X1), dtype=torch.float32, device=dev)
    Yd = torch.as_tensor(np.asarray(X2), dtype=torch.float32, device=dev)
    M = ops.feature_cost(Xd, Yd, Ts=torch.as_tensor(Ts, device=dev), weights="fot")
    res, _ = solve_ott(M, float(reg2))
    Tv = res.plan
    d, d2 = M.shape
    Tv0 = 1.0 / (d * d2) if Tv_init is None else Tv_init
    # cost, delta and the finiteness test on the device, one host read
    stats = torch.stack([(M * Tv).sum(), torch.linalg.norm(Tv - Tv0),
                         torch.isfinite(Tv).all().to(Tv.dtype)]).cpu().tolist()
    cost, delta, finite = float(stats[0]), float(stats[1]), stats[2] > 0.5
    costs = [cost]
    if verbose:
        print("Delta: {0}  Loss: {1}".format(delta, cost))
    if niter > 1:
        costs.append(cost)
        if verbose:
            print("Delta: {0}  Loss: {1}".format(0.0, cost))
            print("converged at iter ", 1)
    if not finite:
        raise FloatingPointError("non-finite feature coupling")
    Tv_np = ops.to_host(Tv)
    if log:
        return Tv_np, cost, {"cost": costs}
    return Tv_np, cost


def get_coupling_fot(
    data: Tuple[Dict[Number, np.ndarray], Dict[Number, np.ndarray]],
    Ts: Union[Dict[Number, np.ndarray], np.ndarray],
    eps=5e-3,
):
    """Feature-to-feature coupling given sample coupling(s) (perturbot fot.py:155-220).

    Label order is the insertion order of ``data[0]`` (fot.py:212-213).  Returns
    ``(Tv, log)``, or ``(-1, -1)`` on FloatingPointError like the reference.
    """
    X_dict, Y_dict = data
    if isinstance(Ts, dict):
        Ts = mdict_to_matrix(
            Ts,
            np.concatenate([np.ones(X_dict[l].shape[0]) * l for l in X_dict.keys()]),
            np.concatenate([np.ones(Y_dict[l].shape[0]) * l for l in X_dict.keys()]),
        )
    X = np.concatenate([X_dict[l] for l in X_dict.keys()])
    Y = np.concatenate([Y_dict[l] for l in X_dict.keys()])
    start = time.time()
    try:
        Tv, cost, log = fot_numpy(X, Y, Ts, log=True, reg=eps, reg2=eps, niter=2000)
    except FloatingPointError:
        return -1, -1
    log["time"] = time.time() - start
    return Tv, log


def _eot(Xs, Xt, eps):
    dev = _device()
    X = torch.as_tensor(np.asarray(Xs), dtype=torch.float32, device=dev)
    Y = torch.as_tensor(np.asarray(Xt), dtype=torch.float32, device=dev)
    t0 = time.time()
    C, cmax = ops.pairwise_cost(X, Y, metric="sqeuclidean", zero_diag=False, want_max=True)
    C = ops.scale_inplace(C.double(), cmax)      # PointCloud(..., scale_cost="max_cost")
    cost_time = time.time() - t0
    t0 = time.time()
    res, _ = solve_ott(C, float(eps), scale_cost=None)
    info = res.info()
    n, m = C.shape
    reg_ot_cost = float((res.u * (1.0 / n)).sum() + (res.v * (1.0 / m)).sum())
    log = {"n_iters_outer": info["niter"] + 1, "converged": info["status"] == 1,
           "OT cost": reg_ot_cost, "time": time.time() - t0, "cost_time": cost_time}
    return ops.to_host(res.plan), log


def get_coupling_eot_ott(data, eps: float = 5e-3):
    """EOT on the concatenated samples, labels ignored (perturbot ott_egwl.py:299-372)."""
    X_dict, Y_dict = data
    Xs = np.concatenate([X_dict[l] for l in X_dict.keys()], axis=0)
    Xt = np.concatenate([Y_dict[l] for l in X_dict.keys()], axis=0)
    return _eot(Xs, Xt, eps)


def get_coupling_leot_ott(data, eps: float = 5e-3):
    """Per-label EOT (perturbot ott_egwl.py:375-454): returns ({label: plan}, {label: log})."""
    X_dict, Y_dict = data
    Ts, logs = {}, {}
    for l in X_dict.keys():
        Ts[l], logs[l] = _eot(X_dict[l], Y_dict[l], eps)
    return Ts, logs


# ----------------------------------------------------------------------- entropic GW
def _egw_solve(pairs, eps, max_iterations, sinkhorn_max_iterations, labels=None):
    """Entropic GW (OTT GromovWasserstein) on PointCloud(x, x, scale_cost="max_cost")
    geometries, one device launch for every (X, Y) pair.  Returns plans + logs."""
    from . import gw

    dev = _device()
    t0 = time.time()
    C1s, C2s = [], []
    for X, Y in pairs:
        x = torch.nan_to_num(torch.as_tensor(np.asarray(X), device=dev).float())
        y = torch.nan_to_num(torch.as_tensor(np.asarray(Y), device=dev).float())
        C1, _ = gw.pairwise_cost_f64(x, None, metric="sqeuclidean", zero_diag=False, scale_max=True)
        C2, _ = gw.pairwise_cost_f64(y, None, metric="sqeuclidean", zero_diag=False, scale_max=True)
        C1s.append(C1)
        C2s.append(C2)
    torch.cuda.current_stream(dev).synchronize()
    cost_time = time.time() - t0
    t0 = time.time()
    res = gw.solve_batched(C1s, C2s, gw.GW_ENTROPIC, labels=labels, max_iter=max_iterations,
                           min_iter=5, threshold=1e-3, eps=float(eps),
                           sk_max_iter=sinkhorn_max_iterations, sk_inner=OTT_INNER,
                           sk_threshold=OTT_THRESHOLD, warm_start=True,
                           log_len=max(1, min(max_iterations, 4096)))
    plans = [T.cpu().numpy() for T in res.plans]
    infos = res.infos()
    elapsed = time.time() - t0
    logs = []
    for info in infos:
        if info["status"] == "timeout":
            raise RuntimeError("entropic GW: device time limit reached")
        logs.append({"n_iters_outer": info["n_iter"], "converged_inner": info["converged_inner"],
                     "converged_outer": info["converged"], "GW cost": info["cost"],
                     "time": elapsed, "cost_time": cost_time})
    return plans, logs


def get_coupling_egw_ott_fixed(
    data: Tuple[Dict[Number, np.ndarray], Dict[Number, np.ndarray]],
    eps: float = 5e-3,
    gw_max_iterations: int = 2000,
    sinkhorn_max_iterations: int = 2000,
) -> Tuple[Dict[Number, np.ndarray], Dict]:
    """Per-label entropic GW (MRI_PET_OT_OT_per_epoch_attn.py:129-186): NaN features
    are zeroed, ``PointCloud(x, x, scale_cost="max_cost")`` geometries, OTT
    ``GromovWasserstein(epsilon=eps, max_iterations=gw_max_iterations,
    linear_solver=Sinkhorn(max_iterations=sinkhorn_max_iterations))``.  All labels in
    one launch.  Returns ``({label: plan}, {label: log})``."""
    X_dict, Y_dict = data
    labels = list(X_dict.keys())
    plans, logs = _egw_solve([(X_dict[l], Y_dict[l]) for l in labels], eps, gw_max_iterations,
                             sinkhorn_max_iterations)
    return dict(zip(labels, plans)), dict(zip(labels, logs))


def epoch_label_groups(labels: torch.Tensor, max_per_label: int | None = 64):
    """``group_features_by_label`` (MRI_PET_OT_OT_per_epoch_attn.py:915-937) as row index
    sets: labels in ``np.unique`` order, the first ``max_per_label`` rows of each (one
    host read of the labels).  Returns ``[(label, int64 index array), ...]``."""
    lab = labels.reshape(-1).to("cpu").numpy()
    groups = []
    for l in np.unique(lab):
        idx = np.nonzero(lab == l)[0]
        if max_per_label is not None and max_per_label > 0:
            idx = idx[:max_per_label]
        groups.append((int(l), idx))
    return groups


def egw_label_plans(pets, mris, eps: float = 5e-3, gw_max_iterations: int = 2000,
                    sinkhorn_max_iterations: int = 2000):
    """``get_coupling_egw_ott_fixed`` (:954) on device tensors: every label's entropic GW
    (PET samples x MRI samples) in one launch.  Returns ``(plans, result)``."""
    from . import gw
    C1s, C2s = [], []
    for x, y in zip(pets, mris):
        C1s.append(gw.pairwise_cost_f64(x, None, metric="sqeuclidean", zero_diag=False, scale_max=True)[0])
        C2s.append(gw.pairwise_cost_f64(y, None, metric="sqeuclidean", zero_diag=False, scale_max=True)[0])
    egw = gw.solve_batched(C1s, C2s, gw.GW_ENTROPIC, max_iter=gw_max_iterations, min_iter=5,
                           threshold=1e-3, eps=float(eps), sk_max_iter=sinkhorn_max_iterations,
                           sk_inner=OTT_INNER, sk_threshold=OTT_THRESHOLD, warm_start=True,
                           log_len=max(1, min(gw_max_iterations, 4096)))
    return list(egw.plans), egw


def fot_from_label_plans(pets, mris, plans, eps: float = 5e-3):
    """``get_coupling_fot((pet, mri), Ts)`` (:959 -> perturbot fot.py:155-220) given the
    per-label sample plans: block-diagonal Ts (label order = data[0] keys), ``Ts /=
    Ts.sum()``, the fot-weighted float64 feature cost and the OTT solve with a host poll
    every 10 iterations.  Returns the ``SinkhornResult`` (plan = Tv, d_pet x d_mri)."""
    n = sum(int(T.shape[0]) for T in plans)
    dev = pets[0].device
    Ts = torch.zeros((n, n), dtype=torch.float64, device=dev)
    r = 0
    for T in plans:
        Ts[r:r + T.shape[0], r:r + T.shape[1]] = T
        r += T.shape[0]
    Ts = Ts / Ts.sum()
    M = ops.feature_cost(torch.cat(pets), torch.cat(mris), Ts=Ts, weights="fot")
    res, _ = solve_ott(M, float(eps), sync_every=OTT_INNER)
    return res


def per_epoch_coupling_device(mri: torch.Tensor, pet: torch.Tensor, labels: torch.Tensor,
                              eps: float = 5e-3, max_per_label: int | None = 64,
                              gw_max_iterations: int = 2000, sinkhorn_max_iterations: int = 2000,
                              comm=None):
    """``compute_pet_to_mri_coupling`` (MRI_PET_OT_OT_per_epoch_attn.py:940-960) on device
    tensors -- e.g. the all-gathered embedding shards of a data-parallel epoch -- without
    the NumPy round trips of the drop-ins.

    ``group_features_by_label`` (:915-937: labels in ``np.unique`` order, the first
    ``max_per_label`` rows of each) becomes index selects from one host read of the
    labels; ``get_coupling_egw_ott_fixed((pet, mri))`` runs every label's entropic GW in
    one launch (:954); ``get_coupling_fot((pet, mri), Ts)`` (:959 -> perturbot fot.py:155-220)
    builds the float64 feature cost from the block-diagonal Ts on the device (``Ts /=
    Ts.sum()``, fot weights) and runs the OTT solve with a host poll only every 10
    iterations (OTT's own check cadence).  Returns ``(Tv, info)``: Tv the PET->MRI feature
    plan (d_pet x d_mri float64, on the device) and ``info`` a callable returning the
    solver logs (it synchronises; the chain itself reads only the labels back).
    Equivalent to the NumPy chain ``get_coupling_egw_ott_fixed`` + ``get_coupling_fot``
    (tests/test_gpu_configs.py::test_config3_device_chain_matches_dropins).

    ``comm`` (an ``otfuse.comm.Communicator`` or anything with ``rank``, ``nranks`` and
    ``all_reduce``): the label split of ``otfuse.distributed.per_epoch_coupling_split`` --
    rank r solves the entropic GW of labels r, r + W, ... and one all-reduce assembles
    every label's plan on every rank; the same plans bit for bit."""
    groups = epoch_label_groups(labels, max_per_label)
    dev = mri.device
    idx = [torch.as_tensor(i, device=dev) for _, i in groups]
    pets = [torch.nan_to_num(pet.index_select(0, i).float()) for i in idx]
    mris = [torch.nan_to_num(mri.index_select(0, i).float()) for i in idx]
    if comm is not None and comm.nranks > 1:
        from .distributed import split_label_plans
        plans, egw = split_label_plans(
            pets, mris, comm,
            lambda p, m: egw_label_plans(p, m, eps, gw_max_iterations, sinkhorn_max_iterations))
    else:
        plans, egw = egw_label_plans(pets, mris, eps, gw_max_iterations, sinkhorn_max_iterations)
    res = fot_from_label_plans(pets, mris, plans, eps)

    def info():
        return {"egw": egw.infos() if egw is not None else [], "fot": res.info(),
                "labels": [l for l, _ in groups]}

    return res.plan, info


def get_coupling_egw_ott(data, eps: float = 5e-3):
    """Per-label entropic GW, OTT defaults for the inner Sinkhorn, max_iterations=1000
    (perturbot ott_egwl.py:129-206)."""
    return get_coupling_egw_ott_fixed(data, eps, gw_max_iterations=1000,
                                      sinkhorn_max_iterations=OTT_MAX_ITER)


def _concat(data):
    X_dict, Y_dict = data
    keys = list(X_dict.keys())
    Xs = np.concatenate([X_dict[l] for l in keys], axis=0)
    Xt = np.concatenate([Y_dict[l] for l in keys], axis=0)
    la = np.concatenate([np.repeat(l, X_dict[l].shape[0]) for l in keys])
    lb = np.concatenate([np.repeat(l, Y_dict[l].shape[0]) for l in keys])
    return Xs, Xt, la, lb


def get_coupling_egw_all_ott(data, eps: float = 5e-3):
    """Entropic GW on all samples, labels ignored (perturbot ott_egwl.py:209-296).
    Returns ``(T, log)``."""
    Xs, Xt, _, _ = _concat(data)
    plans, logs = _egw_solve([(Xs, Xt)], eps, 1000, OTT_MAX_ITER)
    return plans[0], logs[0]


def get_coupling_egw_labels_ott(data, eps: float = 5e-3):
    """Label-restricted entropic GW on all samples (perturbot ott_egwl.py:25-126): the
    coupling may only join samples with equal labels (the reference's patched OTT
    ``QuadraticProblem(labels_a, labels_b, block_diag_mat)``; here the linearised
    cost is +inf off the label blocks).  Returns ``({label: block}, log)``."""
    Xs, Xt, la, lb = _concat(data)
    uniq = np.unique(la)
    code = {v: i for i, v in enumerate(uniq)}
    ia = np.array([code[v] for v in la], np.int32)
    ib = np.array([code.get(v, -1 - i) for i, v in enumerate(lb)], np.int32)
    plans, logs = _egw_solve([(Xs, Xt)], eps, 2000, 2000, labels=[(ia, ib)])
    T = plans[0]
    T_dict = {l: T[la == l, :][:, lb == l] for l in uniq}
    return T_dict, logs[0]


# ---------------------------------------------------------------- POT GW (match/gw.py)
def _cdist_max(x, dev):
    """scipy ``cdist(x, x)`` (Euclidean) ``/ max`` in float64 on the device."""
    from . import gw
    t = torch.as_tensor(np.asarray(x), device=dev).float()
    C, _ = gw.pairwise_cost_f64(t, None, metric="euclidean", zero_diag=True, scale_max=True)
    return C


def _gw_labels(X_dict, Y_dict, solver, eps=None, max_iter=None):
    from . import gw
    dev = _device()
    labels = list(X_dict.keys())
    log = {"cost_time": {}, "time": {}}
    t0 = time.time()
    C1s = [_cdist_max(X_dict[l], dev) for l in labels]
    C2s = [_cdist_max(Y_dict[l], dev) for l in labels]
    torch.cuda.current_stream(dev).synchronize()
    ct = (time.time() - t0) / max(len(labels), 1)
    t0 = time.time()
    if solver == gw.GW_CG:
        res = gw.solve_batched(C1s, C2s, gw.GW_CG, max_iter=int(max_iter or 1e4), log_len=4096)
    else:
        res = gw.solve_batched(C1s, C2s, gw.GW_PGD, max_iter=int(max_iter or 1000), tol_abs=1e-9,
                               eps=float(eps), sk_max_iter=1000, sk_inner=10, sk_threshold=1e-9,
                               log_len=1024)
    Ts = [T.cpu().numpy() for T in res.plans]
    infos = res.infos()
    el = (time.time() - t0) / max(len(labels), 1)
    out = {}
    for l, T, info in zip(labels, Ts, infos):
        if info["status"] == "timeout":
            raise RuntimeError("GW: device time limit reached")
        out[l] = T
        log["cost_time"][l] = ct
        log["time"][l] = el
        if solver == gw.GW_CG:
            log[l] = {"loss": info["costs"], "gw_dist": info["cost"]}
        else:
            log[l] = {"err": info["costs"], "gw_dist": info["cost"]}
    return out, log


def gw_cg(X_dict, Y_dict):
    """Per-label POT CG-GW on cdist / max costs (perturbot match/gw.py:7-28).  The exact
    linear step is the device assignment solver on equal-size label groups and the
    device network simplex on unequal ones."""
    from . import gw
    return _gw_labels(X_dict, Y_dict, gw.GW_CG)


def egw_pgd(X_dict, Y_dict, epsilon=5e-3):
    """Per-label POT entropic GW, solver='PGD' (perturbot match/gw.py:31-59)."""
    from . import gw
    return _gw_labels(X_dict, Y_dict, gw.GW_PGD, eps=epsilon)


def _all(Xtot, Ytot, solver, eps=None, max_iter=None):
    Ts, log = _gw_labels({0: Xtot}, {0: Ytot}, solver, eps=eps, max_iter=max_iter)
    out = dict(log[0])
    out["time"] = log["time"][0]
    out["cost_time"] = log["cost_time"][0]
    return Ts[0], out


def gw_all(Xtot, Ytot):
    """POT CG-GW on all samples (perturbot match/gw.py:62-77, max_iter=1e8)."""
    from . import gw
    return _all(Xtot, Ytot, gw.GW_CG, max_iter=10 ** 8)


def egw_all(Xtot, Ytot, epsilon=5e-3):
    """POT entropic GW (PGD) on all samples (perturbot match/gw.py:80-102)."""
    from . import gw
    return _all(Xtot, Ytot, gw.GW_PGD, eps=epsilon)


def get_coupling_gw_cg(data):
    return gw_cg(data[0], data[1])


def get_coupling_egw(data, eps=5e-3):
    return egw_pgd(data[0], data[1], epsilon=eps)


def get_coupling_gw_all(data):
    """GW all-to-all, labels ignored (perturbot match/gw.py:119-126)."""
    X_dict, Y_dict = data
    Xtot = np.concatenate([X_dict[l] for l in X_dict.keys()], axis=0)
    Ytot = np.concatenate([Y_dict[l] for l in X_dict.keys()], axis=0)
    return gw_all(Xtot, Ytot)


def get_coupling_egw_all(data, eps=5e-3):
    """Entropic GW all-to-all, labels ignored (perturbot match/gw.py:129-137)."""
    X_dict, Y_dict = data
    Xtot = np.concatenate([X_dict[l] for l in X_dict.keys()], axis=0)
    Ytot = np.concatenate([Y_dict[l] for l in X_dict.keys()], axis=0)
    return egw_all(Xtot, Ytot, eps)


# ---------------------------------------------------------------- COOT-L (cot_labels.py)
def _feature_hist(D, labels):
    """cot_labels.py:110-122: column mass of the concatenated data when it is
    non-negative, else uniform (computed in the data's dtype, as the reference)."""
    Xc = np.concatenate([np.asarray(D[k]) for k in labels], axis=0)
    if (Xc >= 0).all():
        return np.asarray(Xc.sum(axis=0) / Xc.sum(), dtype=np.float64)
    return np.ones(Xc.shape[1]) / Xc.shape[1]


def cotl(X_dict, Y_dict, eps: float = 5e-3, niter: int = 100, v1=None, v2=None, w1=None,
         w2=None, log: bool = False, algo: str = "sinkhorn", algo2: str | None = None,
         C_lin=None, random_init: bool = False, numItermax: int = 10_000_000):
    """``cotl_numpy`` (perturbot/perturbot/match/cot_labels.py:14-225) on the device.

    Block-coordinate descent over per-label sample couplings Ts[k] and one feature
    coupling Tv: the sample costs ``constC_s - X_k Tv (2 Y_k)^T`` (+ ``C_lin``, the
    sample-cost prior of :175-176) and the feature cost ``sum_k constC_v,k - X_k^T Ts[k]
    (2 Y_k)`` come from ``otf_coupled_cost`` (float64, float32 squares).  Each stage
    takes its own solver, as the reference's independent ``algo`` (sample plans) /
    ``algo2`` (feature plan) branches: "sinkhorn" = OTT ``linear.solve(Geometry(M,
    epsilon=reg, scale_cost="max_cost"), max_iterations=2000)`` -- uniform marginals,
    as there -- on the device Sinkhorn (float64, lse mode); "emd" = ``pot.emd(w, w', M,
    numItermax=1e7)`` on the device network simplex (``otf_emd_solve``; the per-label
    sample plans of one step in one launch).  ``random_init``: Ts[k] =
    random_gamma_init(w1[k], w2[k]) for the labels in order, then Tv =
    random_gamma_init(v1, v2) (:133-135, same draws from NumPy's generator).
    Reference behaviour kept: the feature solve uses ``reg`` (:200), never reg2;
    ``delta`` counts only Tv (``Tsold = Ts`` aliases the dict updated in place,
    :167-172); Tv is renormalised when its mass is off by 1e-8; stop when delta < 1e-16
    or |cost change| < 1e-7.  Returns ``(Ts dict of numpy, Tv, cost[, {"cost": [...]}])``.
    """
    algo2 = algo if algo2 is None else algo2
    for a_ in (algo, algo2):
        if a_ not in ("sinkhorn", "emd"):
            raise NotImplementedError(f"algo={a_!r}")
    assert sorted(X_dict.keys()) == sorted(Y_dict.keys()), "Labels don't match in y1 & y2."
    dev = _device()
    labels = list(X_dict.keys())
    if v1 is None:
        v1 = _feature_hist(X_dict, labels)
    if v2 is None:
        v2 = _feature_hist(Y_dict, labels)
    Xs = {k: torch.as_tensor(np.asarray(X_dict[k]), device=dev).float() for k in labels}
    Ys = {k: torch.as_tensor(np.asarray(Y_dict[k]), device=dev).float() for k in labels}
    v1t = torch.as_tensor(np.asarray(v1, dtype=np.float64), device=dev)
    v2t = torch.as_tensor(np.asarray(v2, dtype=np.float64), device=dev)
    f64 = dict(dtype=torch.float64, device=dev)
    w1t = {k: (torch.full((Xs[k].shape[0],), 1.0 / Xs[k].shape[0], **f64) if w1 is None
               else torch.as_tensor(np.asarray(w1[k], dtype=np.float64), device=dev)) for k in labels}
    w2t = {k: (torch.full((Ys[k].shape[0],), 1.0 / Ys[k].shape[0], **f64) if w2 is None
               else torch.as_tensor(np.asarray(w2[k], dtype=np.float64), device=dev)) for k in labels}
    Clt = None if C_lin is None else torch.as_tensor(np.asarray(C_lin, dtype=np.float64), device=dev)
    d, d2 = Xs[labels[0]].shape[1], Ys[labels[0]].shape[1]
    if random_init:
        Ts = {k: random_gamma_init_device(w1t[k].cpu().numpy(), w2t[k].cpu().numpy()) for k in labels}
        Tv = random_gamma_init_device(v1t.cpu().numpy(), v2t.cpu().numpy())
    else:
        Ts = {k: torch.full((Xs[k].shape[0], Ys[k].shape[0]),
                            1.0 / (Xs[k].shape[0] * Ys[k].shape[0]), **f64) for k in labels}
        Tv = torch.full((d, d2), 1.0 / (d * d2), **f64)
    cost = np.inf
    costs = []
    for _ in range(niter):
        Tvold, costold = Tv, cost
        Ms = []
        for k in labels:  # sample costs of every label under the current Tv
            Mk = ops.coupled_cost(Xs[k], Ys[k], Tv, v1t, v2t)
            Ms.append(Mk if Clt is None else Mk + Clt)
        if algo == "emd":  # sample OT per label: every label's EMD in one launch
            for k, T in zip(labels, _emd_many([(w1t[k], w2t[k], Mk) for k, Mk in zip(labels, Ms)],
                                              numItermax)):
                Ts[k] = T
        else:
            for k, Mk in zip(labels, Ms):
                res, _ = solve_ott(Mk, eps, "max_cost", max_iterations=OTT_MAX_ITER)
                Ts[k] = res.plan
        M = None  # global feature OT
        for k in labels:
            Mv = ops.coupled_cost(Xs[k].T, Ys[k].T, Ts[k], w1t[k], w2t[k])
            M = Mv if M is None else M + Mv
        if algo2 == "emd":
            Tv = _emd_many([(v1t, v2t, M)], numItermax)[0]
        else:
            res, _ = solve_ott(M, eps, "max_cost", max_iterations=OTT_MAX_ITER)
            Tv = res.plan
        tot = float(Tv.sum())
        if not abs(tot - 1.0) < 1e-8:
            Tv = Tv / tot
        delta = float(torch.linalg.norm(Tv - Tvold))
        cost = float((M * Tv).sum())
        costs.append(cost)
        if delta < 1e-16 or abs(costold - cost) < 1e-7:
            break
    Ts_np = {k: Ts[k].cpu().numpy() for k in labels}
    if log:
        return Ts_np, ops.to_host(Tv), cost, {"cost": costs}
    return Ts_np, ops.to_host(Tv), cost


def cotl_numpy(X_dict, Y_dict, w1=None, w2=None, v1=None, v2=None, niter: int = 100,
               algo: str = "emd", reg: float = 0.2, algo2: str = "emd", reg2: float = 0.2,
               verbose: bool = True, log: bool = False, random_init: bool = False, C_lin=None):
    """Drop-in for perturbot ``cotl_numpy`` (cot_labels.py:14-225), same signature and
    returns; see ``cotl`` (reg2 is accepted and, as in the reference, unused)."""
    return cotl(X_dict, Y_dict, eps=reg, niter=niter, v1=v1, v2=v2, w1=w1, w2=w2, log=log,
                algo=algo, algo2=algo2, C_lin=C_lin, random_init=random_init)


def cotl_sinkhorn(X_dict, Y_dict, eps: float = 5e-3, eps2: float | None = None,
                  niter: int = 100, v1=None, v2=None, w1=None, w2=None, log: bool = False,
                  algo: str = "sinkhorn", numItermax: int = 10_000_000):
    """``cotl_numpy(..., algo=algo, algo2=algo, reg=eps, reg2=eps2)``: both stages on one
    solver (kept for the r02 callers; ``cotl`` takes every combination)."""
    return cotl(X_dict, Y_dict, eps=eps, niter=niter, v1=v1, v2=v2, w1=w1, w2=w2, log=log,
                algo=algo, algo2=algo, numItermax=numItermax)


def get_coupling_cotl_sinkhorn(data, eps: float = 5e-3, eps2: float | None = None):
    """perturbot cot_labels.py:279-340: COOT-L with Sinkhorn solves, niter=2000.
    Returns ``(Ts dict, log)`` (``(-1, -1)`` on a FloatingPointError, as the reference)."""
    X_dict, Y_dict = data
    start = time.time()
    try:
        Ts, Tv, cost, log = cotl_sinkhorn(X_dict, Y_dict, eps=eps, eps2=eps if eps2 is None else eps2,
                                          niter=2000, log=True)
    except FloatingPointError:
        return -1, -1
    log["time"] = time.time() - start
    return Ts, log


def _emd_many(problems, numItermax):
    """pot.emd on each (a, b, M) (device float64), b rescaled to a's mass as POT does;
    warns like POT when a solve stops at numItermax."""
    prep = []
    for a, b, M in problems:
        sa, sb = float(a.sum()), float(b.sum())
        np.testing.assert_almost_equal(sa, sb, err_msg="a and b vector must have the same sum",
                                       decimal=6)
        prep.append((a, b * (sa / sb), M))
    res = ops.emd_batched(prep, max_pivots=int(numItermax))
    for inf in res.infos():
        if inf["status"] == 1:
            warnings.warn("numItermax reached before optimality. Try to increase numItermax.",
                          UserWarning)
        elif inf["status"] != 0:
            warnings.warn(f"EMD: {inf['status_name']}", UserWarning)
    return res.plans


def get_coupling_cotl(data):
    """perturbot cot_labels.py:228-276: COOT-L with exact EMD on general marginals
    (``cotl_numpy(X_dict, Y_dict, log=True, niter=2000)``, algo = algo2 = "emd").
    Returns ``(Ts dict, log)`` (``(-1, -1)`` on a FloatingPointError, as the reference)."""
    X_dict, Y_dict = data
    start = time.time()
    try:
        Ts, Tv, cost, log = cotl_sinkhorn(X_dict, Y_dict, niter=2000, log=True, algo="emd")
    except FloatingPointError:
        return -1, -1
    log["time"] = time.time() - start
    return Ts, log
