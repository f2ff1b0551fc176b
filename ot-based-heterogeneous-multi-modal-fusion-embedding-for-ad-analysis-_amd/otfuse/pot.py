"""Drop-ins for the POT calls and the POT-based coupling functions of the reference.

Same names, argument meaning and return conventions as the reference call sites:

* ``sinkhorn``  -> ``ot.sinkhorn(a, b, M, reg, numItermax, stopThr)`` used at
  MRI_PET_OT_nojax.py:143 (POT 0.9.6 ``sinkhorn_knopp``);
* ``dist`` / ``unif`` -> ``ot.dist`` / ``ot.unif`` (MRI_PET_OT_nojax.py:70-79);
* ``emd`` -> ``ot.emd`` (network simplex, general marginals; cot_labels.py:178,195);
* ``get_feature_coupling_pot`` -> MRI_PET_OT_nojax.py:91-145 (copy in MRI_T1_T2_OT.py:92-146).

NumPy inputs give NumPy outputs (float64 plans, like POT on the reference's
float64 ``M``) so the functions drop into the unchanged training scripts; torch
device tensors stay on the device end to end.  All arithmetic runs in the HIP
library — there is no CPU path.
"""
from __future__ import annotations

import time
import warnings
from typing import Dict, Tuple, Union
from numbers import Number

import numpy as np
import torch

from . import ops


def _device():
    if not torch.cuda.is_available():
        raise RuntimeError("otfuse needs a ROCm GPU (torch.cuda.is_available() is False)")
    return torch.device("cuda", torch.cuda.current_device())


def _as_dev(x, dtype, device):
    if isinstance(x, torch.Tensor):
        return x.to(device=device, dtype=dtype)
    return torch.as_tensor(np.asarray(x), dtype=dtype, device=device)


def unif(n: int, type_as=None):
    """``ot.unif``: uniform histogram of length n."""
    if isinstance(type_as, torch.Tensor):
        return torch.full((n,), 1.0 / n, dtype=type_as.dtype, device=type_as.device)
    return np.ones((n,)) / n


def dist(x1, x2=None, metric: str = "sqeuclidean"):
    """``ot.dist`` for the metrics the reference uses ('sqeuclidean', 'euclidean').

    POT zeroes the diagonal when ``x2`` is ``x1`` (or omitted).  The contraction runs
    on float32 MFMA; float64 inputs are rounded to float32 first.
    """
    same = x2 is None or x2 is x1
    is_torch = isinstance(x1, torch.Tensor) and x1.is_cuda
    dev = x1.device if is_torch else _device()
    X = _as_dev(x1, torch.float32, dev)
    Y = X if same else _as_dev(x2, torch.float32, dev)
    C, _ = ops.pairwise_cost(X, None if same else Y, metric=metric, zero_diag=same, want_max=False)
    if is_torch:
        return C.to(x1.dtype)
    dt = np.result_type(np.asarray(x1).dtype, np.float32) if x2 is None else \
        np.result_type(np.asarray(x1).dtype, np.asarray(x2).dtype)
    return C.cpu().numpy().astype(dt, copy=False)


def sinkhorn(a, b, M, reg: float, method: str = "sinkhorn", numItermax: int = 1000,
             stopThr: float = 1e-9, verbose: bool = False, log: bool = False, warn: bool = True,
             warmstart=None, **kwargs):
    """``ot.sinkhorn`` (method 'sinkhorn' = ``sinkhorn_knopp``) on the device.

    Semantics follow POT 0.9.6: u0 = 1/n, v0 = 1/m, v-update then u-update, revert to
    the previous iterate and stop on a zero in K^T u or nan/inf in u, v ("numerical
    errors" warning), L2 marginal error every 10 iterations against ``stopThr``.
    Computes in the dtype of ``M`` (float64 for the reference's feature costs).
    Extra keyword ``sync_every`` (default 50) sets how often the host polls the
    device-side convergence flag.
    """
    if method.lower() not in ("sinkhorn", "sinkhorn_knopp"):
        raise NotImplementedError(f"method {method!r}: only POT's sinkhorn_knopp is provided")
    if warmstart is not None:
        raise NotImplementedError("warmstart is not supported")
    is_torch = isinstance(M, torch.Tensor) and M.is_cuda
    dev = M.device if is_torch else _device()
    mdt = (M.dtype if is_torch else np.asarray(M).dtype)
    dt = torch.float32 if mdt in (torch.float32, np.float32) else torch.float64
    Md = _as_dev(M, dt, dev)
    n, m = Md.shape
    a = unif(n) if a is None or len(a) == 0 else a
    b = unif(m) if b is None or len(b) == 0 else b
    if np.ndim(b.cpu() if isinstance(b, torch.Tensor) else b) > 1:
        raise NotImplementedError("multiple target histograms (2-D b) are not supported")
    ad = _as_dev(a, dt, dev)
    bd = _as_dev(b, dt, dev)
    res = ops.sinkhorn(ad, bd, Md, float(reg), max_iter=int(numItermax), stop_thr=float(stopThr),
                       flavor="pot", sync_every=int(kwargs.get("sync_every", 50)), want_plan=True)
    info = res.info()
    if warn and info["status"] == 3:
        warnings.warn("Warning: numerical errors at iteration %d" % info["break_iter"])
    if warn and info["status"] == 2:
        warnings.warn("Sinkhorn did not converge. You might want to increase the number of "
                      "iterations `numItermax` or the regularization parameter `reg`.")
    if verbose:
        for k, e in enumerate(info["err"]):
            print("{:5d}|{:8e}|".format(10 * k, e))
    P = res.plan if is_torch else ops.to_host(res.plan)
    if not log:
        return P
    # a shifted float32 solve (ops.sinkhorn's default at 64 < max(M)/reg <= 700) holds
    # u~, v~; POT's log reports its own scalings u = 2^A u~, v = 2^B v~ (float64: at small
    # reg they can leave float32's range)
    u, v = res.pot_scalings() if res.shifted else (res.u, res.v)
    if not is_torch:
        u, v = u.cpu().numpy(), v.cpu().numpy()
    return P, {"err": info["err"], "niter": info["niter"], "u": u, "v": v,
               "status": info["status_name"]}


def emd(a, b, M, numItermax: int = 100000, log: bool = False, center_dual: bool = True,
        numThreads=1, check_marginals: bool = True):
    """``ot.emd`` (POT 0.9.x ``ot.lp.emd``, network simplex) on the device.

    As POT: empty ``a`` / ``b`` mean uniform; the masses must agree to 6 decimals
    (``check_marginals``) and ``b`` is rescaled to ``a``'s total; a solve that stops
    at ``numItermax`` pivots warns "numItermax reached before optimality".  The plan
    is float64 (NumPy in, NumPy out).  ``log`` returns ``cost``, ``warning`` and
    ``result_code`` (the duals are not returned).  Called by ``get_coupling_cotl``
    (cot_labels.py:178,195) via ``emd_batch``.
    """
    return emd_batch([(a, b, M)], numItermax=numItermax, log=log,
                     check_marginals=check_marginals)[0]


def emd_batch(problems, numItermax: int = 100000, log: bool = False, check_marginals: bool = True):
    """Several independent ``ot.emd`` problems in one device launch."""
    is_torch = isinstance(problems[0][2], torch.Tensor) and problems[0][2].is_cuda
    dev = problems[0][2].device if is_torch else _device()
    prep = []
    for a, b, M in problems:
        Md = _as_dev(M, torch.float64, dev)
        n, m = Md.shape
        a = unif(n) if a is None or len(a) == 0 else a
        b = unif(m) if b is None or len(b) == 0 else b
        ad = _as_dev(a, torch.float64, dev).reshape(-1)
        bd = _as_dev(b, torch.float64, dev).reshape(-1)
        sa, sb = float(ad.sum()), float(bd.sum())
        if check_marginals:
            np.testing.assert_almost_equal(sa, sb, err_msg="a and b vector must have the same sum",
                                           decimal=6)
        bd = bd * (sa / sb)
        prep.append((ad, bd, Md))
    res = ops.emd_batched(prep, max_pivots=int(numItermax))
    infos = res.infos()
    out = []
    for T, inf in zip(res.plans, infos):
        warn = None
        if inf["status"] == 1:
            warn = "numItermax reached before optimality. Try to increase numItermax."
        elif inf["status"] == 2:
            warn = "Problem infeasible. Check that a and b are in the simplex"
        elif inf["status"] == 3:
            warn = "Problem unbounded"
        if warn is not None:
            warnings.warn(warn, UserWarning)
        G = T if is_torch else T.cpu().numpy()
        if log:
            out.append((G, {"cost": inf["cost"], "warning": warn,
                            "result_code": {0: 1, 1: 3, 2: 0, 3: 2}[inf["status"]],
                            "n_pivots": inf["n_pivots"]}))
        else:
            out.append(G)
    return out


def _concat_sorted(X_dict, Y_dict):
    keys = sorted(X_dict.keys())
    X = np.concatenate([X_dict[k] for k in keys])
    Y = np.concatenate([Y_dict[k] for k in keys])
    return keys, X, Y


def block_diag_ts(Ts: Dict[Number, np.ndarray], X_dict, Y_dict) -> np.ndarray:
    """Per-label sample plans -> block-diagonal Ts in sorted label order
    (MRI_PET_OT_nojax.py:105-119; labels missing from ``Ts`` leave zero blocks)."""
    keys = sorted(X_dict.keys())
    n_x = sum(len(X_dict[k]) for k in keys)
    n_y = sum(len(Y_dict[k]) for k in keys)
    T = np.zeros((n_x, n_y))
    ix = iy = 0
    for k in keys:
        nx, ny = len(X_dict[k]), len(Y_dict[k])
        if k in Ts:
            T[ix:ix + nx, iy:iy + ny] = Ts[k]
        ix += nx
        iy += ny
    return T


def feature_coupling_pot_device(X: torch.Tensor, Y: torch.Tensor, Ts=None, ts_diag=None,
                                eps: float = 5e-3, numItermax: int = 2000, stopThr: float = 1e-9,
                                sync_every: int = 50):
    """Device form of get_feature_coupling_pot on already-concatenated X (n, d), Y (n2, d2):
    float64 feature cost + POT-flavour float64 Sinkhorn.  Returns ``ops.SinkhornResult``."""
    M = ops.feature_cost(X, Y, Ts=Ts, ts_diag=ts_diag, weights="pot")
    d, d2 = M.shape
    a = ops.uniform(d, torch.float64, M.device)
    b = ops.uniform(d2, torch.float64, M.device)
    return ops.sinkhorn(a, b, M, float(eps), max_iter=numItermax, stop_thr=stopThr, flavor="pot",
                        sync_every=sync_every, want_plan=True)


def _diag_or_none(T: np.ndarray):
    if T.ndim == 2 and T.shape[0] == T.shape[1]:
        d = np.diag(T)
        if np.count_nonzero(T - np.diag(d)) == 0:
            return d
    return None


def get_feature_coupling_pot(
    data: Tuple[Dict[Number, np.ndarray], Dict[Number, np.ndarray]],
    Ts: Union[Dict[Number, np.ndarray], np.ndarray],
    eps=5e-3,
):
    """Feature coupling using POT-semantics Sinkhorn (MRI_PET_OT_nojax.py:91-145).

    Concatenates the per-label arrays in sorted label order, assembles a block
    diagonal Ts from a dict, builds M = t1 + t2 - 2 X^T Ts Y in float64 and solves
    ``sinkhorn(1/d, 1/d', M, reg=eps, numItermax=2000)``.  Returns ``(Tv, {})`` with
    Tv a float64 (d, d') ndarray, like the reference.
    """
    X_dict, Y_dict = data
    _, X, Y = _concat_sorted(X_dict, Y_dict)
    if isinstance(Ts, dict):
        Ts = block_diag_ts(Ts, X_dict, Y_dict)
    Ts = np.asarray(Ts, dtype=np.float64)
    dev = _device()
    Xd = torch.as_tensor(X, dtype=torch.float32, device=dev)
    Yd = torch.as_tensor(Y, dtype=torch.float32, device=dev)
    diag = _diag_or_none(Ts)
    if diag is not None:
        res = feature_coupling_pot_device(Xd, Yd, ts_diag=torch.as_tensor(diag, device=dev),
                                          eps=eps)
    else:
        res = feature_coupling_pot_device(Xd, Yd, Ts=torch.as_tensor(Ts, device=dev), eps=eps)
    info = res.info()
    if info["status"] == 3:
        warnings.warn("Warning: numerical errors at iteration %d" % info["break_iter"])
    return ops.to_host(res.plan), {}


def get_coupling_gromov_pot(
    data: Tuple[Dict[Number, np.ndarray], Dict[Number, np.ndarray]], eps: float = 5e-3
) -> Tuple[Dict[Number, np.ndarray], Dict]:
    """Per-label Gromov-Wasserstein couplings (MRI_PET_OT_nojax.py:52-88).

    For every label (``data[0]`` insertion order, like the reference's loop):
    ``C1 = ot.dist(x, x, 'euclidean') / max``, ``C2`` likewise, then POT's exact CG
    ``gromov_wasserstein(C1, C2, unif, unif, 'square_loss', epsilon=eps)`` — the
    ``epsilon`` keyword is swallowed by POT's **kwargs, so ``eps`` has no effect
    there either.  Unequal group sizes take the network-simplex linear step.  All
    labels are solved concurrently in one device launch.  Plans
    come back as NumPy arrays in the features' dtype (POT returns ``type_as=C1``).
    Returns ``(Ts, log)`` with ``log[label]["time"]``.
    """
    from . import gw

    X_dict, Y_dict = data
    labels = list(X_dict.keys())
    dev = _device()
    start = {}
    C1s, C2s, dtypes = [], [], []
    for l in labels:
        start[l] = time.time()
        x = _as_dev(X_dict[l], torch.float32, dev)
        y = _as_dev(Y_dict[l], torch.float32, dev)
        C1, _ = gw.pairwise_cost_f64(x, None, metric="euclidean", zero_diag=True, scale_max=True)
        C2, _ = gw.pairwise_cost_f64(y, None, metric="euclidean", zero_diag=True, scale_max=True)
        C1s.append(C1)
        C2s.append(C2)
        dtypes.append(np.result_type(np.asarray(X_dict[l]).dtype, np.asarray(Y_dict[l]).dtype))
    res = gw.solve_batched(C1s, C2s, gw.GW_CG, max_iter=10000, log_len=1)
    plans = [T.cpu().numpy() for T in res.plans]
    end = time.time()
    Ts, log = {}, {}
    for l, T, dt in zip(labels, plans, dtypes):
        Ts[l] = T.astype(dt, copy=False)
        log[l] = {"time": end - start[l]}
    return Ts, log
