"""CPU oracle for the Sinkhorn OT fusion path — TEST INFRASTRUCTURE ONLY.

This module is the parity checker (tests/), the smoke check
(``__graft_entry__.smoke``) and the timed CPU baseline (``bench.py``'s
``cpu_baseline`` leg).  Nothing in the product package imports it; the product
path is the HIP library and fails loudly when that library is missing.

Two restatements of the reference algorithm live here:

* ``libotoracle.so`` (``otoracle.c``, float64, OpenMP) — the fast one, used for
  the CPU baseline and the large parity cases;
* pure-NumPy functions (``*_np``) — small cases, and a cross-check of the C code.

Both follow the reference (file:line into /root/reference):

* feature cost     MRI_PET_OT_nojax.py:121-136
* pairwise cost    MRI_PET_OT_nojax.py:70-75 -> POT 0.9.6 ``ot.dist`` (not vendored)
* Sinkhorn-Knopp   MRI_PET_OT_nojax.py:143 -> POT ``sinkhorn_knopp``; vendored twin
                   perturbot/perturbot/match/utils.py:6-115
* log-domain       perturbot/perturbot/match/fot.py:128-134 -> OTT-jax 0.6.0
                   (absent here: parity unpinned)
* plan apply       MRI_PET_OT_nojax.py:701-721
* GW (CG, POT)     MRI_PET_OT_nojax.py:80-82 -> POT ``ot.gromov.gromov_wasserstein``
                   (absent: parity unpinned; the inner exact EMD / assignment is
                   cross-checked against scipy's ``linear_sum_assignment``)
* GW (entropic)    MRI_PET_OT_OT_per_epoch_attn.py:161-174, ott_egwl.py -> OTT
                   ``GromovWasserstein`` (absent: parity unpinned)

Pinning: the Sinkhorn, feature-cost and plan-apply restatements are checked
against golden vectors produced by the reference's own code in the survey
container (tests/golden/make_golden.py -> tests/golden/*.npz).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "libotoracle.so")
_lib = None

_dp = ctypes.POINTER(ctypes.c_double)
_fp = ctypes.POINTER(ctypes.c_float)
_ip = ctypes.POINTER(ctypes.c_int64)


def build() -> str:
    """Compile ``libotoracle.so`` with the committed Makefile."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        L.oro_set_threads.argtypes = [ctypes.c_int]
        L.oro_set_threads.restype = ctypes.c_int
        L.oro_pairwise_cost.argtypes = [_dp, _dp, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64,
                                        ctypes.c_int, ctypes.c_int, ctypes.c_int, _dp]
        L.oro_pairwise_cost.restype = ctypes.c_double
        L.oro_feature_cost.argtypes = [_dp, _dp, _dp, ctypes.c_int64, ctypes.c_int64,
                                       ctypes.c_int64, ctypes.c_int64, ctypes.c_int, ctypes.c_int,
                                       _dp]
        L.oro_feature_cost.restype = None
        L.oro_sinkhorn_knopp.argtypes = [_dp, _dp, _dp, ctypes.c_int64, ctypes.c_int64,
                                         ctypes.c_double, ctypes.c_double, ctypes.c_int,
                                         ctypes.c_double, ctypes.c_int, ctypes.c_int,
                                         _dp, _dp, _dp, _ip, _dp]
        L.oro_sinkhorn_knopp.restype = ctypes.c_int
        L.oro_sinkhorn_log.argtypes = [_dp, _dp, _dp, ctypes.c_int64, ctypes.c_int64,
                                       ctypes.c_double, ctypes.c_double, ctypes.c_int,
                                       ctypes.c_double, ctypes.c_int, _dp, _dp, _dp, _ip]
        L.oro_sinkhorn_log.restype = None
        L.oro_plan_apply.argtypes = [_dp, ctypes.c_int64, ctypes.c_int64, _fp, ctypes.c_int64,
                                     _fp, _fp]
        L.oro_plan_apply.restype = None
        _ii = ctypes.POINTER(ctypes.c_int)
        L.oro_lap.argtypes = [_dp, ctypes.c_int64, _ii]
        L.oro_lap.restype = ctypes.c_int
        L.oro_gw_cg.argtypes = [_dp, _dp, ctypes.c_int64, ctypes.c_int, ctypes.c_double,
                                ctypes.c_double, _dp, _dp, ctypes.c_int, _ip, _dp]
        L.oro_gw_cg.restype = ctypes.c_int
        L.oro_gw_entropic.argtypes = [_dp, _dp, ctypes.c_int64, ctypes.c_int64, _dp, _dp, _ii,
                                      _ii, ctypes.c_double, ctypes.c_int, ctypes.c_int,
                                      ctypes.c_double, ctypes.c_int, ctypes.c_int,
                                      ctypes.c_double, ctypes.c_int, _dp, _dp, ctypes.c_int,
                                      _ip, _dp]
        L.oro_gw_entropic.restype = ctypes.c_int
        L.oro_gw_pgd.argtypes = [_dp, _dp, ctypes.c_int64, ctypes.c_int64, _dp, _dp,
                                 ctypes.c_double, ctypes.c_int, ctypes.c_double, ctypes.c_int,
                                 ctypes.c_double, _dp, _dp, ctypes.c_int, _ip, _dp]
        L.oro_gw_pgd.restype = ctypes.c_int
        _lib = L
    return _lib


def set_threads(n: int) -> int:
    return lib().oro_set_threads(int(n))


def _d(x):
    return np.ascontiguousarray(x, dtype=np.float64)


def _ptr(a, t=_dp):
    return a.ctypes.data_as(t)


# --------------------------------------------------------------------------- C-backed
def pairwise_cost(X, Y, metric="sqeuclidean", zero_diag=False, scale_max=False):
    """Returns ``(C float64 (n, m), max of unscaled C)``."""
    X, Y = _d(X), _d(Y)
    n, d = X.shape
    m = Y.shape[0]
    C = np.empty((n, m), np.float64)
    mx = lib().oro_pairwise_cost(_ptr(X), _ptr(Y), n, m, d, int(metric == "euclidean"),
                                 int(zero_diag), int(scale_max), _ptr(C))
    return C, mx


def feature_cost(X, Y, Ts, weights="pot"):
    """Feature cost; float32 inputs are squared in float32 like the reference's X**2."""
    sq_f32 = int(np.asarray(X).dtype == np.float32 and np.asarray(Y).dtype == np.float32)
    X, Y, Ts = _d(X), _d(Y), _d(Ts)
    n, d = X.shape
    n2, d2 = Y.shape
    M = np.empty((d, d2), np.float64)
    lib().oro_feature_cost(_ptr(X), _ptr(Y), _ptr(Ts), n, n2, d, d2, sq_f32,
                           int(weights == "fot"), _ptr(M))
    return M


def sinkhorn_knopp(a, b, C, reg, numItermax=1000, stopThr=1e-9, cscale=1.0, check_every=10,
                   err_squared=False, want_plan=True):
    """POT ``sinkhorn_knopp`` semantics.  Returns ``(P|None, u, v, info dict)``."""
    a, b, C = _d(a), _d(b), _d(C)
    n, m = C.shape
    u = np.empty(n)
    v = np.empty(m)
    P = np.empty((n, m)) if want_plan else None
    info = np.zeros(4, np.int64)
    errlog = np.zeros(numItermax // max(check_every, 1) + 2)
    lib().oro_sinkhorn_knopp(_ptr(a), _ptr(b), _ptr(C), n, m, float(reg), float(cscale),
                             int(numItermax), float(stopThr), int(check_every), int(err_squared),
                             _ptr(u), _ptr(v), _ptr(P) if P is not None else None,
                             _ptr(info, _ip), _ptr(errlog))
    return P, u, v, {"niter": int(info[0]), "n_updates": int(info[1]),
                     "break_iter": int(info[2]), "err": errlog[: int(info[3])].tolist()}


def sinkhorn_log(a, b, C, reg, max_iter=2000, threshold=1e-3, inner=10, cscale=1.0):
    """OTT-flavour log-domain Sinkhorn (parity unpinned).  Returns ``(P, f, g, info)``."""
    a, b, C = _d(a), _d(b), _d(C)
    n, m = C.shape
    f = np.empty(n)
    g = np.empty(m)
    P = np.empty((n, m))
    info = np.zeros(2, np.int64)
    lib().oro_sinkhorn_log(_ptr(a), _ptr(b), _ptr(C), n, m, float(reg), float(cscale),
                           int(max_iter), float(threshold), int(inner), _ptr(f), _ptr(g),
                           _ptr(P), _ptr(info, _ip))
    return P, f, g, {"n_iters": int(info[0]), "converged": bool(info[1])}


def plan_apply(T, Z=None):
    """MRI_PET_OT_nojax.py:701-721 in float32.  Returns ``(T_normalised, Z @ T_n^T | None)``."""
    T = _d(T)
    d, d2 = T.shape
    Tn = np.empty((d, d2), np.float32)
    out = None
    if Z is not None:
        Z = np.ascontiguousarray(Z, dtype=np.float32)
        out = np.empty((Z.shape[0], d), np.float32)
    lib().oro_plan_apply(_ptr(T), d, d2, _ptr(Z, _fp) if Z is not None else None,
                         Z.shape[0] if Z is not None else 0, _ptr(Tn, _fp),
                         _ptr(out, _fp) if out is not None else None)
    return Tn, out


def lap(A):
    """Minimum-cost assignment (serial shortest augmenting paths).  Returns sigma."""
    A = _d(A)
    n = A.shape[0]
    sigma = np.empty(n, np.int32)
    rc = lib().oro_lap(_ptr(A), n, sigma.ctypes.data_as(ctypes.POINTER(ctypes.c_int)))
    if rc:
        raise FloatingPointError("oro_lap: non-finite cost")
    return sigma


def gw_cg(C1, C2, max_iter=10000, tol_rel=1e-9, tol_abs=1e-9, log_len=64):
    """POT CG-GW (uniform marginals, n x n).  Returns ``(G, info)``."""
    C1, C2 = _d(C1), _d(C2)
    n = C1.shape[0]
    G = np.empty((n, n))
    clog = np.zeros(log_len)
    info = np.zeros(3, np.int64)
    cost = ctypes.c_double()
    lib().oro_gw_cg(_ptr(C1), _ptr(C2), n, int(max_iter), float(tol_rel), float(tol_abs),
                    _ptr(G), _ptr(clog), log_len, _ptr(info, _ip), ctypes.byref(cost))
    it = int(info[0])
    return G, {"n_iter": it, "converged": bool(info[1]), "status": int(info[2]),
               "loss": clog[: min(it + 1, log_len)].tolist(), "gw_dist": cost.value}


def gw_entropic(C1, C2, eps, a=None, b=None, labels_a=None, labels_b=None, max_iter=2000,
                min_iter=5, threshold=1e-3, sk_max=2000, sk_inner=10, sk_thr=1e-3, warm=True,
                log_len=256):
    """OTT entropic GW.  Returns ``(P, info)``."""
    C1, C2 = _d(C1), _d(C2)
    n, m = C1.shape[0], C2.shape[0]
    P = np.empty((n, m))
    clog = np.zeros(log_len)
    info = np.zeros(5, np.int64)
    cost = ctypes.c_double()
    ip = ctypes.POINTER(ctypes.c_int)
    la = None if labels_a is None else np.ascontiguousarray(labels_a, np.int32)
    lb = None if labels_b is None else np.ascontiguousarray(labels_b, np.int32)
    a = None if a is None else _d(a)
    b = None if b is None else _d(b)
    lib().oro_gw_entropic(_ptr(C1), _ptr(C2), n, m, _ptr(a) if a is not None else None,
                          _ptr(b) if b is not None else None,
                          la.ctypes.data_as(ip) if la is not None else None,
                          lb.ctypes.data_as(ip) if lb is not None else None, float(eps),
                          int(max_iter), int(min_iter), float(threshold), int(sk_max),
                          int(sk_inner), float(sk_thr), int(bool(warm)), _ptr(P), _ptr(clog),
                          log_len, _ptr(info, _ip), ctypes.byref(cost))
    it = int(info[0])
    return P, {"n_iters": it, "converged": bool(info[1]), "converged_inner": bool(info[2]),
               "inner_iters": int(info[3]), "status": int(info[4]),
               "costs": clog[: min(it, log_len)].tolist(), "reg_gw_cost": cost.value}


def gw_pgd(C1, C2, eps, a=None, b=None, max_iter=1000, tol=1e-9, sk_max=1000, sk_thr=1e-9,
           log_len=128):
    """POT entropic GW, solver='PGD' (perturbot gw.py:31-59).  Returns ``(T, info)``."""
    C1, C2 = _d(C1), _d(C2)
    n, m = C1.shape[0], C2.shape[0]
    T = np.empty((n, m))
    elog = np.zeros(log_len)
    info = np.zeros(4, np.int64)
    cost = ctypes.c_double()
    a = None if a is None else _d(a)
    b = None if b is None else _d(b)
    lib().oro_gw_pgd(_ptr(C1), _ptr(C2), n, m, _ptr(a) if a is not None else None,
                     _ptr(b) if b is not None else None, float(eps), int(max_iter), float(tol),
                     int(sk_max), float(sk_thr), _ptr(T), _ptr(elog), log_len, _ptr(info, _ip),
                     ctypes.byref(cost))
    return T, {"n_iter": int(info[0]), "converged": bool(info[1]), "inner_iters": int(info[2]),
               "err": elog[: min(int(info[3]), log_len)].tolist(), "gw_dist": cost.value}


# --------------------------------------------------------------------------- NumPy
def gw_cg_np(C1, C2, max_iter=10000, tol_rel=1e-9, tol_abs=1e-9, p=None, q=None):
    """POT 0.9.6 ``gromov_wasserstein(C1, C2, p, q, 'square_loss')`` in NumPy.  The exact
    EMD of the linear step: scipy's ``linear_sum_assignment`` for uniform marginals on
    n x n (an independent LAP for cross-checking ``oro_lap`` / the device solver),
    otherwise the HiGHS transportation LP (``emd_lp``)."""
    from scipy.optimize import linear_sum_assignment

    C1, C2 = _d(C1), _d(C2)
    n, m = C1.shape[0], C2.shape[0]
    general = p is not None or q is not None or n != m
    p = np.full(n, 1.0 / n) if p is None else np.asarray(p, np.float64)
    q = np.full(m, 1.0 / m) if q is None else np.asarray(q, np.float64)
    constC = ((C1 ** 2) @ p)[:, None] + ((C2 ** 2) @ q)[None, :]
    hC1, hC2 = C1, 2.0 * C2

    def tens(G):
        return constC - hC1 @ G @ hC2.T

    G = np.outer(p, q)
    cost = float(np.sum(tens(G) * G))
    losses = [cost]
    it = 0
    while True:
        it += 1
        old = cost
        df = 2.0 * tens(G)
        Mi = df + df.min()
        if general:
            Gc = emd_lp(p, q, Mi)[0]
        else:
            rows, cols = linear_sum_assignment(Mi)
            Gc = np.zeros_like(G)
            Gc[rows, cols] = 1.0 / n
        dG = Gc - G
        dot = hC1 @ dG @ hC2.T
        a = -np.sum(dot * dG)
        b = -2.0 * np.sum(dot * G)
        if a > 0:
            alpha = min(1.0, max(0.0, -b / (2.0 * a)))
        else:
            alpha = 1.0 if a + b < 0 else 0.0
        cost = cost + a * alpha ** 2 + b * alpha
        G = G + alpha * dG
        losses.append(cost)
        absd = abs(cost - old)
        reld = absd / abs(cost) if cost != 0 else np.nan
        if reld < tol_rel or absd < tol_abs or it >= max_iter:
            break
    return G, {"n_iter": it, "loss": losses, "gw_dist": cost}


def gw_pgd_np(C1, C2, eps, p=None, q=None, max_iter=1000, tol=1e-9, sk_max=1000, sk_thr=1e-9):
    """POT 0.9.6 ``entropic_gromov_wasserstein(C1, C2, p, q, 'square_loss', epsilon,
    solver='PGD')`` in NumPy (symmetric C1, C2; the inner solve is ``sinkhorn_knopp_np``)."""
    C1, C2 = _d(C1), _d(C2)
    n, m = C1.shape[0], C2.shape[0]
    p = np.full(n, 1.0 / n) if p is None else _d(p)
    q = np.full(m, 1.0 / m) if q is None else _d(q)
    constC = ((C1 ** 2) @ p)[:, None] + ((C2 ** 2) @ q)[None, :]

    def tens(T):
        return constC - C1 @ T @ (2.0 * C2).T

    T = np.outer(p, q)
    cpt, err, errs = 0, 1.0, []
    while err > tol and cpt < max_iter:
        Tprev = T
        T, _, _, _ = sinkhorn_knopp_np(p, q, 2.0 * tens(T), eps, sk_max, sk_thr)
        if cpt % 10 == 0:
            err = np.linalg.norm(T - Tprev)
            errs.append(err)
        cpt += 1
    return T, {"n_iter": cpt, "err": errs, "gw_dist": float(np.sum(tens(T) * T))}


def coupled_cost_np(A, B, T, w1, w2):
    """perturbot utils.py:125-184 init_matrix_np + ``constC - hC1 T hC2^T``: squares of
    the float32 data in float32 (X**2), everything else in float64."""
    A = np.asarray(A, np.float32)
    B = np.asarray(B, np.float32)
    t1 = (A * A).astype(np.float64) @ _d(w1)
    t2 = (B * B).astype(np.float64) @ _d(w2)
    return t1[:, None] + t2[None, :] - (A.astype(np.float64) @ _d(T)) @ (2.0 * B.astype(np.float64)).T


def cotl_sinkhorn_np(X_dict, Y_dict, eps, niter=100):
    """cot_labels.py:14-225 with algo = algo2 = 'sinkhorn': OTT solves restated by the
    C log-domain Sinkhorn on max-scaled costs (uniform marginals), the BCD loop and its
    reference quirks (feature solve at eps, Tv-only delta, Tv renormalisation)."""
    labels = list(X_dict.keys())

    def hist(D):
        Xc = np.concatenate([np.asarray(D[k]) for k in labels], axis=0)
        if (Xc >= 0).all():
            return np.asarray(Xc.sum(axis=0) / Xc.sum(), dtype=np.float64)
        return np.ones(Xc.shape[1]) / Xc.shape[1]

    v1, v2 = hist(X_dict), hist(Y_dict)
    X = {k: np.asarray(X_dict[k], np.float32) for k in labels}
    Y = {k: np.asarray(Y_dict[k], np.float32) for k in labels}
    w1 = {k: np.ones(len(X[k])) / len(X[k]) for k in labels}
    w2 = {k: np.ones(len(Y[k])) / len(Y[k]) for k in labels}
    d, d2 = X[labels[0]].shape[1], Y[labels[0]].shape[1]
    Ts = {k: np.ones((len(X[k]), len(Y[k]))) / (len(X[k]) * len(Y[k])) for k in labels}
    Tv = np.ones((d, d2)) / (d * d2)

    def ott(M):
        n, m = M.shape
        P, *_ = sinkhorn_log(np.ones(n) / n, np.ones(m) / m, M, eps, max_iter=2000,
                             threshold=1e-3, cscale=1.0 / M.max())
        return P

    cost, costs = np.inf, []
    for _ in range(niter):
        Tvold, costold = Tv, cost
        for k in labels:
            Ts[k] = ott(coupled_cost_np(X[k], Y[k], Tv, v1, v2))
        M = 0
        for k in labels:
            M = M + coupled_cost_np(X[k].T, Y[k].T, Ts[k], w1[k], w2[k])
        Tv = ott(M)
        if not np.abs(Tv.sum() - 1.0) < 1e-8:
            Tv = Tv / Tv.sum()
        delta = np.linalg.norm(Tv - Tvold)
        cost = np.sum(M * Tv)
        costs.append(cost)
        if delta < 1e-16 or np.abs(costold - cost) < 1e-7:
            break
    return Ts, Tv, cost, {"cost": costs}


def emd_lp(a, b, M):
    """pot.emd (POT 0.9.x network simplex; POT is absent here) restated as the
    transportation LP min <M, T> s.t. T 1 = a, T^T 1 = b * sum(a) / sum(b), T >= 0,
    solved by scipy's HiGHS.  Generic costs have a unique optimum, so plans compare
    entry-wise.  Returns (T, cost)."""
    from scipy.optimize import linprog
    from scipy.sparse import coo_matrix
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    b = b * a.sum() / b.sum()
    M = np.asarray(M, np.float64)
    n, m = M.shape
    rows = np.concatenate([np.repeat(np.arange(n), m), n + np.tile(np.arange(m), n)])
    cols = np.concatenate([np.arange(n * m), np.arange(n * m)])
    A = coo_matrix((np.ones(2 * n * m), (rows, cols)), shape=(n + m, n * m)).tocsr()
    r = linprog(M.ravel(), A_eq=A, b_eq=np.concatenate([a, b]), bounds=(0, None), method="highs",
                options={"primal_feasibility_tolerance": 1e-10, "dual_feasibility_tolerance": 1e-10})
    if r.status != 0:
        raise RuntimeError(f"linprog: {r.message}")
    return r.x.reshape(n, m), float(r.fun)


def cotl_emd_np(X_dict, Y_dict, niter=100):
    """cot_labels.py:14-225 with algo = algo2 = 'emd' (pot.emd -> emd_lp): same BCD
    loop and quirks as cotl_sinkhorn_np."""
    labels = list(X_dict.keys())

    def hist(D):
        Xc = np.concatenate([np.asarray(D[k]) for k in labels], axis=0)
        if (Xc >= 0).all():
            return np.asarray(Xc.sum(axis=0) / Xc.sum(), dtype=np.float64)
        return np.ones(Xc.shape[1]) / Xc.shape[1]

    v1, v2 = hist(X_dict), hist(Y_dict)
    X = {k: np.asarray(X_dict[k], np.float32) for k in labels}
    Y = {k: np.asarray(Y_dict[k], np.float32) for k in labels}
    w1 = {k: np.ones(len(X[k])) / len(X[k]) for k in labels}
    w2 = {k: np.ones(len(Y[k])) / len(Y[k]) for k in labels}
    d, d2 = X[labels[0]].shape[1], Y[labels[0]].shape[1]
    Ts = {k: np.ones((len(X[k]), len(Y[k]))) / (len(X[k]) * len(Y[k])) for k in labels}
    Tv = np.ones((d, d2)) / (d * d2)
    cost, costs = np.inf, []
    for _ in range(niter):
        Tvold, costold = Tv, cost
        for k in labels:
            Ts[k] = emd_lp(w1[k], w2[k], coupled_cost_np(X[k], Y[k], Tv, v1, v2))[0]
        M = 0
        for k in labels:
            M = M + coupled_cost_np(X[k].T, Y[k].T, Ts[k], w1[k], w2[k])
        Tv = emd_lp(v1, v2, M)[0]
        if not np.abs(Tv.sum() - 1.0) < 1e-8:
            Tv = Tv / Tv.sum()
        delta = np.linalg.norm(Tv - Tvold)
        cost = np.sum(M * Tv)
        costs.append(cost)
        if delta < 1e-16 or np.abs(costold - cost) < 1e-7:
            break
    return Ts, Tv, cost, {"cost": costs}


def pairwise_cost_np(X, Y, metric="sqeuclidean", zero_diag=False):
    """POT ``euclidean_distances`` (via ``ot.dist``) in float64."""
    X, Y = _d(X), _d(Y)
    c = -2.0 * (X @ Y.T)
    c += np.einsum("ij,ij->i", X, X)[:, None]
    c += np.einsum("ij,ij->i", Y, Y)[None, :]
    c = np.maximum(c, 0.0)
    if metric == "euclidean":
        c = np.sqrt(c)
    if zero_diag:
        c = c * (1.0 - np.eye(c.shape[0], c.shape[1]))
    return c


def feature_cost_np(X, Y, Ts):
    """MRI_PET_OT_nojax.py:121-136 (keeps the inputs' dtype for X**2, as the reference)."""
    X, Y, Ts = np.asarray(X), np.asarray(Y), _d(Ts)
    w1 = Ts.sum(axis=1)
    t1 = (X ** 2).T @ w1
    w2 = Ts.sum(axis=0)
    t2 = (Y ** 2).T @ w2
    t3 = -2 * X.T @ Ts @ Y
    return t1[:, None] + t2[None, :] + t3


def block_diag_ts(ts_dict, x_dict, y_dict):
    """Block-diagonal Ts from a per-label dict, sorted label order (MRI_PET_OT_nojax.py:105-119)."""
    keys = sorted(x_dict.keys())
    nx = sum(len(x_dict[k]) for k in keys)
    ny = sum(len(y_dict[k]) for k in keys)
    T = np.zeros((nx, ny))
    ix = iy = 0
    for k in keys:
        a, b = len(x_dict[k]), len(y_dict[k])
        if k in ts_dict:
            T[ix:ix + a, iy:iy + b] = ts_dict[k]
        ix += a
        iy += b
    return T


def sinkhorn_knopp_np(a, b, M, reg, numItermax=1000, stopThr=1e-9, check_every=10):
    """POT 0.9.6 ``sinkhorn_knopp`` restated in NumPy (small problems only)."""
    a, b, M = _d(a), _d(b), _d(M)
    u = np.ones(len(a)) / len(a)
    v = np.ones(len(b)) / len(b)
    K = np.exp(M / (-reg))
    Kp = (1 / a).reshape(-1, 1) * K
    niter = 0
    errs = []
    for ii in range(numItermax):
        niter = ii
        uprev, vprev = u, v
        ktu = K.T @ u
        v = b / ktu
        u = 1.0 / (Kp @ v)
        if (np.any(ktu == 0) or np.any(np.isnan(u)) or np.any(np.isnan(v))
                or np.any(np.isinf(u)) or np.any(np.isinf(v))):
            u, v = uprev, vprev
            break
        if ii % check_every == 0:
            err = np.linalg.norm(np.einsum("i,ij,j->j", u, K, v) - b)
            errs.append(err)
            if err < stopThr:
                break
    return u.reshape(-1, 1) * K * v.reshape(1, -1), u, v, {"niter": niter, "err": errs}


def sinkhorn_scaling_np(a, b, K, numItermax=1000, stopThr=1e-9):
    """perturbot ``sinkhorn_scaling`` (utils.py:6-115) restated: POT's scaling
    iteration on a GIVEN kernel matrix K (no exp), revert-and-break on a zero K^T u or a
    non-finite scaling, marginal error as the SQUARED 2-norm every 10 iterations.
    Returns the plan u K v."""
    a, b, K = _d(a), _d(b), _d(K)
    u = np.ones(len(a)) / len(a)
    v = np.ones(len(b)) / len(b)
    Kp = (1 / a).reshape(-1, 1) * K
    for ii in range(int(numItermax)):
        uprev, vprev = u, v
        ktu = K.T @ u
        v = b / ktu
        u = 1.0 / (Kp @ v)
        if (np.any(ktu == 0) or np.any(np.isnan(u)) or np.any(np.isnan(v))
                or np.any(np.isinf(u)) or np.any(np.isinf(v))):
            u, v = uprev, vprev
            break
        if ii % 10 == 0:
            err = np.sum((np.einsum("i,ij,j->j", u, K, v) - b) ** 2)
            if not err > stopThr:   # the reference's `while err > stopThr`
                break
    return u.reshape(-1, 1) * K * v.reshape(1, -1)


def beta_kernel(n, m):
    """The random matrix of perturbot ``random_gamma_init`` (utils.py:118-122): a dense
    scipy.sparse.random(n, m, density=1) with Beta(0.1, 0.1) entries, drawn from
    NumPy's global generator exactly as the reference draws it."""
    from scipy import stats
    from scipy.sparse import random as sprandom
    return sprandom(n, m, density=1, data_rvs=stats.beta(1e-1, 1e-1).rvs).toarray()


def random_gamma_init_np(p, q, numItermax=1000, stopThr=1e-9):
    return sinkhorn_scaling_np(p, q, beta_kernel(len(p), len(q)), numItermax, stopThr)


def cotl_np(X_dict, Y_dict, eps=5e-3, niter=100, algo="sinkhorn", algo2="sinkhorn", C_lin=None,
            random_init=False):
    """cot_labels.py:14-225 (cotl_numpy) restated with every branch the reference has:
    per-stage solver algo (sample plans) / algo2 (feature plan) each 'sinkhorn' (OTT
    linear.solve on the max-scaled cost at reg, restated by the C log-domain Sinkhorn)
    or 'emd' (pot.emd -> emd_lp); the sample-cost prior C_lin added to every M_k (:175-176);
    random_init: Ts[k] = random_gamma_init(w1[k], w2[k]) for the labels in order, then
    Tv = random_gamma_init(v1, v2) (:133-135).  Quirks kept: feature solve at reg (:200),
    Tv-only delta (Tsold aliases Ts), Tv renormalisation, stop on delta < 1e-16 or
    |cost change| < 1e-7."""
    labels = list(X_dict.keys())

    def hist(D):
        Xc = np.concatenate([np.asarray(D[k]) for k in labels], axis=0)
        if (Xc >= 0).all():
            return np.asarray(Xc.sum(axis=0) / Xc.sum(), dtype=np.float64)
        return np.ones(Xc.shape[1]) / Xc.shape[1]

    v1, v2 = hist(X_dict), hist(Y_dict)
    X = {k: np.asarray(X_dict[k], np.float32) for k in labels}
    Y = {k: np.asarray(Y_dict[k], np.float32) for k in labels}
    w1 = {k: np.ones(len(X[k])) / len(X[k]) for k in labels}
    w2 = {k: np.ones(len(Y[k])) / len(Y[k]) for k in labels}
    d, d2 = X[labels[0]].shape[1], Y[labels[0]].shape[1]
    if random_init:
        Ts = {k: random_gamma_init_np(w1[k], w2[k]) for k in labels}
        Tv = random_gamma_init_np(v1, v2)
    else:
        Ts = {k: np.ones((len(X[k]), len(Y[k]))) / (len(X[k]) * len(Y[k])) for k in labels}
        Tv = np.ones((d, d2)) / (d * d2)

    def ott(M):
        n, m = M.shape
        P, *_ = sinkhorn_log(np.ones(n) / n, np.ones(m) / m, M, eps, max_iter=2000,
                             threshold=1e-3, cscale=1.0 / M.max())
        return P

    cost, costs = np.inf, []
    for _ in range(niter):
        Tvold, costold = Tv, cost
        for k in labels:
            Mk = coupled_cost_np(X[k], Y[k], Tv, v1, v2)
            if C_lin is not None:
                Mk = Mk + C_lin
            Ts[k] = emd_lp(w1[k], w2[k], Mk)[0] if algo == "emd" else ott(Mk)
        M = 0
        for k in labels:
            M = M + coupled_cost_np(X[k].T, Y[k].T, Ts[k], w1[k], w2[k])
        Tv = emd_lp(v1, v2, M)[0] if algo2 == "emd" else ott(M)
        if not np.abs(Tv.sum() - 1.0) < 1e-8:
            Tv = Tv / Tv.sum()
        delta = np.linalg.norm(Tv - Tvold)
        cost = np.sum(M * Tv)
        costs.append(cost)
        if delta < 1e-16 or np.abs(costold - cost) < 1e-7:
            break
    return Ts, Tv, cost, {"cost": costs}

