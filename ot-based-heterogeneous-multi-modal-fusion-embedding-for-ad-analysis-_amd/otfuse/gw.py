"""Gromov-Wasserstein couplings on the device.

Two solvers over the C ABI ``otf_gw_solve`` (csrc/otf_gw.hip), one workgroup per
problem, all problems of a call in one launch:

* ``gromov_wasserstein`` — POT 0.9.6 ``ot.gromov.gromov_wasserstein(C1, C2, p, q,
  'square_loss')``: conditional gradient with an exact EMD inner solve and the
  closed-form line search, as called by ``get_coupling_gromov_pot``
  (MRI_PET_OT_nojax.py:52-88).  The exact EMD for the callers' uniform, equal-size
  marginals is an optimal assignment / n, solved on the device.
* ``entropic_gromov_wasserstein`` — POT 0.9.6 ``ot.gromov.entropic_gromov_wasserstein(
  C1, C2, p, q, 'square_loss', epsilon, solver='PGD')``: sinkhorn_knopp inner solves on
  the gradient, as called by perturbot ``match/gw.py`` (egw_pgd, egw_all).
* ``entropic_gromov_wasserstein_ott`` — OTT-jax 0.6.0 ``GromovWasserstein(epsilon,
  linear_solver=Sinkhorn(max_iterations))``, as called by
  ``get_coupling_egw_ott_fixed`` (MRI_PET_OT_OT_per_epoch_attn.py:129-186) and
  perturbot ``ott_egwl.py``; optional labels restrict the coupling to equal labels.

POT and OTT are absent from the build container, so both are restatements of the
published algorithms (the oracle's ``gw_cg`` / ``gw_entropic`` are the CPU
twins): parity with the reference's own outputs is UNPINNED.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _lib as L

GW_CG, GW_ENTROPIC, GW_PGD = 0, 1, 2
GW_STATUS = {0: "running", 1: "converged", 2: "max_iter", 3: "numerical", 4: "timeout"}
GW_MAXN = 4096  # per side; past 1024 the kernel keeps its vectors in the workspace


GwOpts, GwProblem = L.GwOpts, L.GwProblem


def _bind(name):
    return getattr(L.lib(), name)


def _dev(t, name):
    if not isinstance(t, torch.Tensor) or not t.is_cuda:
        raise TypeError(f"{name} must be a ROCm device tensor")
    return t


# ------------------------------------------------------------------ sample costs
def pairwise_cost_f64(X: torch.Tensor, Y: torch.Tensor | None = None, metric: str = "sqeuclidean",
                      zero_diag: bool | None = None, scale_max: bool = False):
    """float64 ``ot.dist`` / ``PointCloud`` cost between float32 rows (POT order).

    Returns ``(C float64 (n, m), cmax (1,) float64)``; ``scale_max`` divides C by its
    max on the device (``C /= C.max()``, scale_cost="max_cost").
    """
    _dev(X, "X")
    same = Y is None or Y is X
    Y = X if same else _dev(Y, "Y")
    if zero_diag is None:
        zero_diag = same
    if metric not in ("sqeuclidean", "euclidean"):
        raise ValueError(f"metric {metric!r} not supported (sqeuclidean | euclidean)")
    if X.dim() != 2 or Y.dim() != 2 or X.shape[1] != Y.shape[1]:
        raise ValueError(f"X {tuple(X.shape)} and Y {tuple(Y.shape)} must be (n, d) and (m, d)")
    X = X.float().contiguous()
    Y = X if same else Y.float().contiguous()
    n, d = X.shape
    m = Y.shape[0]
    C = torch.empty((n, m), dtype=torch.float64, device=X.device)
    cmax = torch.empty(1, dtype=torch.float64, device=X.device)
    wsb = _bind("otf_cost_pairwise_f64_workspace_size")(n, m)
    ws = torch.empty(wsb, dtype=torch.uint8, device=X.device)
    met = L.OTF_EUCLIDEAN if metric == "euclidean" else L.OTF_SQEUCLIDEAN
    L.check(_bind("otf_cost_pairwise_f64")(
        X.data_ptr(), X.stride(0), Y.data_ptr(), Y.stride(0), n, m, d, met, int(zero_diag),
        int(bool(scale_max)), C.data_ptr(), C.stride(0), cmax.data_ptr(), ws.data_ptr(), wsb,
        L.stream_handle(X.device)), "otf_cost_pairwise_f64")
    return C, cmax


# ------------------------------------------------------------------ batched solve
class GwResult:
    """Couplings and per-problem logs of one ``solve_batched`` call."""

    def __init__(self, plans, info_raw, costlog, solver):
        self.plans = plans
        self._info = info_raw
        self._costlog = costlog
        self.solver = solver

    def infos(self):
        raw = self._info.cpu().numpy()
        ints = raw[:, :24].copy().view(np.int32).reshape(len(raw), 6)
        cost = raw[:, 24:32].copy().view(np.float64).reshape(len(raw))
        logs = self._costlog.cpu().numpy() if self._costlog is not None else None
        out = []
        for b in range(len(raw)):
            it = int(ints[b, 0])
            d = {"n_iter": it, "converged": bool(ints[b, 1]), "converged_inner": bool(ints[b, 2]),
                 "status": GW_STATUS.get(int(ints[b, 3]), str(int(ints[b, 3]))),
                 "inner_iters": int(ints[b, 4]), "cost": float(cost[b])}
            if logs is not None:
                k = it + 1 if self.solver == GW_CG else ((it + 9) // 10 if self.solver == GW_PGD else it)
                d["costs"] = logs[b, :min(k, logs.shape[1])].tolist()
            out.append(d)
        return out


def solve_batched(C1s, C2s, solver: int, ps=None, qs=None, labels=None, *, max_iter: int,
                  min_iter: int = 5, tol_rel: float = 1e-9, tol_abs: float = 1e-9,
                  threshold: float = 1e-3, eps: float = 0.0, sk_max_iter: int = 2000,
                  sk_inner: int = 10, sk_threshold: float = 1e-3, warm_start: bool = True,
                  log_len: int = 256) -> GwResult:
    """Solve len(C1s) independent GW problems in one launch (float64 device tensors)."""
    nprob = len(C1s)
    if nprob == 0 or len(C2s) != nprob:
        raise ValueError("C1s and C2s must be non-empty lists of equal length")
    dev = _dev(C1s[0], "C1").device
    keep = []
    probs = (GwProblem * nprob)()
    plans = []
    for b in range(nprob):
        C1 = _dev(C1s[b], "C1").to(torch.float64).contiguous()
        C2 = _dev(C2s[b], "C2").to(torch.float64).contiguous()
        n, m = C1.shape[0], C2.shape[0]
        if C1.shape != (n, n) or C2.shape != (m, m):
            raise ValueError("C1 must be (n, n) and C2 (m, m)")
        if n > GW_MAXN or m > GW_MAXN:
            raise NotImplementedError(f"GW problem {n}x{m}: at most {GW_MAXN} points per side")
        T = torch.empty((n, m), dtype=torch.float64, device=dev)
        plans.append(T)
        p = None if ps is None or ps[b] is None else ps[b].to(dev, torch.float64).contiguous()
        q = None if qs is None or qs[b] is None else qs[b].to(dev, torch.float64).contiguous()
        la = lb = None
        if labels is not None and labels[b] is not None:
            la = torch.as_tensor(labels[b][0], device=dev).to(torch.int32).contiguous()
            lb = torch.as_tensor(labels[b][1], device=dev).to(torch.int32).contiguous()
        keep += [C1, C2, p, q, la, lb]
        probs[b] = GwProblem(C1.data_ptr(), C1.stride(0), C2.data_ptr(), C2.stride(0),
                             L.ptr(p), L.ptr(q), L.ptr(la), L.ptr(lb), T.data_ptr(), T.stride(0),
                             n, m)
    opts = GwOpts(solver, int(max_iter), int(min_iter), int(sk_max_iter), int(sk_inner),
                  int(bool(warm_start)), float(tol_rel), float(tol_abs), float(threshold),
                  float(sk_threshold), float(eps))
    info = torch.zeros((nprob, 32), dtype=torch.uint8, device=dev)
    costlog = torch.zeros((nprob, log_len), dtype=torch.float64, device=dev)
    wsb = _bind("otf_gw_workspace_size")(nprob, probs)
    ws = torch.empty(max(wsb, 256), dtype=torch.uint8, device=dev)
    L.check(_bind("otf_gw_solve")(nprob, probs, ctypes.byref(opts), info.data_ptr(),
                                  costlog.data_ptr(), log_len, ws.data_ptr(), ws.numel(),
                                  L.stream_handle(dev)), "otf_gw_solve")
    res = GwResult(plans, info, costlog, solver)
    res._keep = keep + [ws]  # inputs stay alive until the caller synchronises
    return res


# ------------------------------------------------------------------ POT / OTT forms
def _symmetric(C):
    return bool(torch.allclose(C, C.T, atol=1e-10))


def gromov_wasserstein(C1, C2, p=None, q=None, loss_fun: str = "square_loss", symmetric=None,
                       log: bool = False, armijo: bool = False, G0=None, max_iter: float = 1e4,
                       tol_rel: float = 1e-9, tol_abs: float = 1e-9, **kwargs):
    """``ot.gromov.gromov_wasserstein`` (POT 0.9.6) on device tensors.

    Supported: square loss, symmetric C1 / C2, any marginals p / q (uniform on equal
    sizes: the linear step is the assignment solver; otherwise the device network
    simplex, ``emd_block``), the default line search and G0 = p q^T.  Extra keywords
    (``epsilon=`` at MRI_PET_OT_nojax.py:81) are ignored, as POT's **kwargs do.
    Returns G (and log with 'loss', 'gw_dist').
    """
    if loss_fun != "square_loss":
        raise NotImplementedError(f"loss_fun={loss_fun!r}: only 'square_loss'")
    if armijo or G0 is not None:
        raise NotImplementedError("armijo / G0 are not supported")
    n, m = C1.shape[0], C2.shape[0]
    pq = []
    for w, k in ((p, n), (q, m)):
        if w is None or torch.allclose(torch.as_tensor(w, dtype=torch.float64).cpu(),
                                       torch.full((k,), 1.0 / k, dtype=torch.float64), rtol=0, atol=0):
            pq.append(None)
        else:
            pq.append(torch.as_tensor(w, dtype=torch.float64, device=C1.device))
    if symmetric is None:
        symmetric = _symmetric(C1) and _symmetric(C2)
    if not symmetric:
        raise NotImplementedError("asymmetric C1 / C2 are not supported")
    res = solve_batched([C1], [C2], GW_CG, ps=[pq[0]], qs=[pq[1]], max_iter=int(max_iter),
                        tol_rel=tol_rel, tol_abs=tol_abs, log_len=min(int(max_iter) + 1, 4096))
    G = res.plans[0]
    if log:
        info = res.infos()[0]
        return G, {"loss": info["costs"], "gw_dist": info["cost"], "n_iter": info["n_iter"]}
    return G


def entropic_gromov_wasserstein(C1, C2, p=None, q=None, loss_fun: str = "square_loss",
                                epsilon: float = 0.1, symmetric=None, G0=None,
                                max_iter: int = 1000, tol: float = 1e-9, solver: str = "PGD",
                                warmstart: bool = False, verbose: bool = False, log: bool = False,
                                **kwargs):
    """``ot.gromov.entropic_gromov_wasserstein`` (POT 0.9.6) on device tensors, as called
    by perturbot/perturbot/match/gw.py:47-57 and :90-99.

    Supported: square loss, symmetric C1 / C2, solver='PGD', G0 = p q^T, no warm start;
    p / q may be any histograms (None: uniform).  Keywords for the inner
    ``ot.sinkhorn`` (numItermax, stopThr) are honoured, as POT forwards **kwargs.
    Returns T (and log with 'err' every 10th iteration and 'gw_dist').
    """
    if loss_fun != "square_loss":
        raise NotImplementedError(f"loss_fun={loss_fun!r}: only 'square_loss'")
    if solver != "PGD":
        raise NotImplementedError(f"solver={solver!r}: only 'PGD'")
    if G0 is not None or warmstart:
        raise NotImplementedError("G0 / warmstart are not supported")
    sk_max = int(kwargs.pop("numItermax", 1000))
    sk_thr = float(kwargs.pop("stopThr", 1e-9))
    kwargs.pop("method", None)
    if kwargs:
        raise TypeError(f"unsupported keywords: {sorted(kwargs)}")
    if symmetric is None:
        symmetric = _symmetric(C1) and _symmetric(C2)
    if not symmetric:
        raise NotImplementedError("asymmetric C1 / C2 are not supported")
    dev = C1.device
    pq = [None if w is None else torch.as_tensor(w, dtype=torch.float64, device=dev) for w in (p, q)]
    res = solve_batched([C1], [C2], GW_PGD, ps=[pq[0]], qs=[pq[1]], max_iter=int(max_iter),
                        tol_abs=float(tol), eps=float(epsilon), sk_max_iter=sk_max, sk_inner=10,
                        sk_threshold=sk_thr, log_len=max(1, (int(max_iter) + 9) // 10))
    T = res.plans[0]
    if log:
        info = res.infos()[0]
        if info["status"] == "timeout":
            raise RuntimeError("entropic GW (PGD): device time limit reached")
        return T, {"err": info["costs"], "gw_dist": info["cost"], "n_iter": info["n_iter"],
                   "inner_iters": info["inner_iters"]}
    return T


def entropic_gromov_wasserstein_ott(C1, C2, epsilon: float, a=None, b=None, labels_a=None,
                                    labels_b=None, max_iterations: int = 50,
                                    min_iterations: int = 5, threshold: float = 1e-3,
                                    sinkhorn_max_iterations: int = 2000,
                                    sinkhorn_threshold: float = 1e-3,
                                    inner_iterations: int = 10, warm_start: bool = True):
    """OTT ``GromovWasserstein(epsilon, ...)(QuadraticProblem(geom_xx, geom_yy))`` on
    precomputed (already max-scaled) costs.  Returns ``(P, info)`` with OTT's
    n_iters / converged / linear convergence / reg_gw_cost / costs."""
    lab = None if labels_a is None else [(labels_a, labels_b)]
    res = solve_batched([C1], [C2], GW_ENTROPIC, ps=[a], qs=[b], labels=lab,
                        max_iter=max_iterations, min_iter=min_iterations, threshold=threshold,
                        eps=epsilon, sk_max_iter=sinkhorn_max_iterations,
                        sk_inner=inner_iterations, sk_threshold=sinkhorn_threshold,
                        warm_start=warm_start, log_len=max(1, min(max_iterations, 4096)))
    return res.plans[0], res.infos()[0]
