"""Device-tensor ops over the C ABI (include/otfuse.h).

Every function takes / returns torch tensors that live on a ROCm device, enqueues
HIP kernels on the current torch stream and never copies through the host (the
Sinkhorn solver syncs only when ``sync_every > 0``).  Shapes and dtypes are
checked here so the C side only sees layouts it supports; anything else raises.
"""
from __future__ import annotations

import ctypes
import warnings
from dataclasses import dataclass, field

import numpy as np
import torch

from . import _lib as L

_VEC = {torch.float32: 4, torch.float64: 2, torch.float16: 8}   # elements per 16 B
_DT = {torch.float32: L.OTF_F32, torch.float64: L.OTF_F64, torch.float16: L.OTF_F16}
_EMB_DT = {torch.float32: L.OTF_F32, torch.bfloat16: L.OTF_BF16, torch.float16: L.OTF_F16}


def _dev(t: torch.Tensor, name: str):
    if not isinstance(t, torch.Tensor) or not t.is_cuda:
        raise TypeError(f"{name} must be a ROCm device tensor")
    return t


def _rowmajor(t: torch.Tensor, vec: int = 1) -> torch.Tensor:
    """A row-major view whose leading dimension is a multiple of ``vec`` and whose
    rows start 16-byte aligned; copies into a padded buffer only when needed."""
    if (t.dim() == 2 and t.stride(1) == 1 and t.stride(0) >= t.shape[1]
            and t.stride(0) % vec == 0 and t.data_ptr() % 16 == 0):
        return t
    n, m = t.shape
    ld = -(-m // vec) * vec
    buf = torch.zeros((n, ld), dtype=t.dtype, device=t.device)
    buf[:, :m].copy_(t)
    return buf[:, :m]


def _alloc_rowmajor(n: int, m: int, dtype, device, vec: int) -> torch.Tensor:
    ld = -(-m // vec) * vec
    return torch.empty((n, ld), dtype=dtype, device=device)[:, :m]


# --------------------------------------------------------------------------- cost
def pairwise_cost(X: torch.Tensor, Y: torch.Tensor | None = None, metric: str = "sqeuclidean",
                  zero_diag: bool | None = None, want_max: bool = True, algo: str = "split16",
                  workspace: torch.Tensor | None = None):
    """``ot.dist``-style pairwise cost on MFMA.  Returns ``(C float32 (n, m), cmax (1,))``.

    ``zero_diag`` defaults to POT's ``X is Y`` rule (MRI_PET_OT_nojax.py:70-71 passes the
    same array twice).  ``cmax`` is a device scalar with max(C) (None if not wanted).
    ``algo``: "split16" (hi/lo fp16 MFMA, fp32-accurate, default) or "f32"
    (v_mfma_f32_32x32x2_f32).
    """
    _dev(X, "X")
    same = Y is None or Y is X
    Y = X if Y is None else _dev(Y, "Y")
    if zero_diag is None:
        zero_diag = same
    if metric not in ("sqeuclidean", "euclidean"):
        raise ValueError(f"metric {metric!r} not supported (sqeuclidean | euclidean)")
    if X.dim() != 2 or Y.dim() != 2 or X.shape[1] != Y.shape[1]:
        raise ValueError(f"X {tuple(X.shape)} and Y {tuple(Y.shape)} must be (n, d) and (m, d)")
    if algo == "split16":
        C, cmax, _ = pairwise_cost_ex(X, None if same else Y, metric, zero_diag, torch.float32,
                                      workspace, in_dtype=torch.float32)
        return C, (cmax if want_max else None)
    X = _rowmajor(X.float(), 4)
    Y = X if same else _rowmajor(Y.float(), 4)
    n, d = X.shape
    m = Y.shape[0]
    C = _alloc_rowmajor(n, m, torch.float32, X.device, 4)
    cmax = torch.empty(1, dtype=torch.float32, device=X.device) if want_max else None
    met = L.OTF_EUCLIDEAN if metric == "euclidean" else L.OTF_SQEUCLIDEAN
    lib = L.lib()
    if algo == "f32":
        L.check(lib.otf_cost_pairwise(
            X.data_ptr(), X.stride(0), Y.data_ptr(), Y.stride(0), n, m, d, met, int(zero_diag),
            C.data_ptr(), C.stride(0), L.ptr(cmax), L.stream_handle(X.device)), "otf_cost_pairwise")
    else:
        raise ValueError(f"algo {algo!r}")
    return C, (mark_cost_max(cmax) if cmax is not None else None)


def mark_cost_max(t: torch.Tensor) -> torch.Tensor:
    """Tags a device scalar as max(C) of the cost it scales (scale_cost = "max_cost"), so
    ``sinkhorn`` may take max(C / cost_scale) = 1 without reading C.  The library's cost
    builders tag the maxima they return; an untagged ``cost_scale`` is measured."""
    t._otf_cost_max = True
    return t


def is_cost_max(t) -> bool:
    return bool(getattr(t, "_otf_cost_max", False))


def cost_last_phases() -> tuple[float, float]:
    """(prep_ms, kernel_ms) of the last pairwise_cost / pairwise_cost_ex call made with
    OTF_COST_PHASES=1 in the environment (profiling; synchronises on that call)."""
    p, k = ctypes.c_float(), ctypes.c_float()
    L.check(L.lib().otf_cost_last_phases(ctypes.byref(p), ctypes.byref(k)), "otf_cost_last_phases")
    return float(p.value), float(k.value)


def pairwise_cost_ex(X: torch.Tensor, Y: torch.Tensor | None = None, metric: str = "sqeuclidean",
                     zero_diag: bool | None = None, out_dtype=torch.float32,
                     workspace: torch.Tensor | None = None, in_dtype=None):
    """Pairwise cost with fp16 inputs and / or fp16 storage (BASELINE config 5).

    ``in_dtype`` (default: float16 if X is float16 else float32): float32 runs the
    split-fp16 contraction, float16 the native fp16 MFMA.  ``out_dtype`` float16
    stores ``C * 2^-k`` (<= 1, k from the row norms).  Returns ``(C, cmax, unit)``:
    ``cmax`` = max of the stored values (the ``cost_scale`` for "max_cost"),
    ``unit`` = 2^k (true cost = stored * unit), both device float scalars.
    """
    _dev(X, "X")
    same = Y is None or Y is X
    Y = X if Y is None else _dev(Y, "Y")
    if zero_diag is None:
        zero_diag = same
    if metric not in ("sqeuclidean", "euclidean"):
        raise ValueError(f"metric {metric!r} not supported (sqeuclidean | euclidean)")
    if X.dim() != 2 or Y.dim() != 2 or X.shape[1] != Y.shape[1]:
        raise ValueError(f"X {tuple(X.shape)} and Y {tuple(Y.shape)} must be (n, d) and (m, d)")
    if in_dtype is None:
        in_dtype = torch.float16 if X.dtype == torch.float16 else torch.float32
    if in_dtype not in (torch.float32, torch.float16) or out_dtype not in (torch.float32, torch.float16):
        raise TypeError("pairwise_cost_ex: float32 / float16 inputs and outputs only")
    X = _rowmajor(X.to(in_dtype), 1)
    Y = X if same else _rowmajor(Y.to(in_dtype), 1)
    n, d = X.shape
    m = Y.shape[0]
    C = _alloc_rowmajor(n, m, out_dtype, X.device, _VEC[out_dtype])
    cmax = torch.empty(1, dtype=torch.float32, device=X.device)
    unit = torch.empty(1, dtype=torch.float32, device=X.device)
    met = L.OTF_EUCLIDEAN if metric == "euclidean" else L.OTF_SQEUCLIDEAN
    lib = L.lib()
    wsb = lib.otf_cost_ex_workspace_size(n, m, d, _DT[in_dtype])
    if workspace is None or workspace.numel() < wsb:
        workspace = torch.empty(wsb, dtype=torch.uint8, device=X.device)
    L.check(lib.otf_cost_pairwise_ex(
        X.data_ptr(), X.stride(0), Y.data_ptr(), Y.stride(0), _DT[in_dtype], n, m, d, met,
        int(zero_diag), C.data_ptr(), C.stride(0), _DT[out_dtype], cmax.data_ptr(), unit.data_ptr(),
        workspace.data_ptr(), workspace.numel(), L.stream_handle(X.device)), "otf_cost_pairwise_ex")
    return C, mark_cost_max(cmax), unit


def scale_inplace(C: torch.Tensor, s: torch.Tensor) -> torch.Tensor:
    """``C /= s`` with a device scalar ``s`` (MRI_PET_OT_nojax.py:74-75)."""
    if s.dtype != C.dtype:
        s = s.to(C.dtype)
    if C.dtype not in (torch.float32, torch.float64):
        raise TypeError("scale_inplace: C must be float32 or float64")
    L.check(L.lib().otf_scale_inplace(C.data_ptr(), C.shape[0], C.shape[1], C.stride(0),
                                      _DT[C.dtype], s.data_ptr(), L.stream_handle(C.device)),
            "otf_scale_inplace")
    return C


def feature_cost(X: torch.Tensor, Y: torch.Tensor, Ts: torch.Tensor | None = None,
                 ts_diag: torch.Tensor | None = None, weights: str = "pot") -> torch.Tensor:
    """Feature cost ``M = t1 + t2 - 2 X^T Ts Y`` in float64 (MRI_PET_OT_nojax.py:121-136).

    ``weights="pot"``: w1 = Ts.sum(1), w2 = Ts.sum(0) (get_feature_coupling_pot);
    ``weights="fot"``: w1 = Ts.sum(0), w2 = Ts.sum(1) (perturbot fot.py:109-118).
    Give ``Ts`` (n, n2) or its diagonal ``ts_diag`` (n,).  X, Y may be float32,
    bfloat16 or float16 (BASELINE config 4: bf16 encoder outputs): the kernels read them
    as stored and widen each element exactly to float32, the reference's arithmetic on
    the rounded values; other dtypes are cast to float32.
    """
    _dev(X, "X")
    _dev(Y, "Y")
    if (Ts is None) == (ts_diag is None):
        raise ValueError("pass exactly one of Ts / ts_diag")
    edt = X.dtype if (X.dtype == Y.dtype and X.dtype in _EMB_DT) else torch.float32
    X = _rowmajor(X.to(edt))
    Y = _rowmajor(Y.to(edt))
    n, d = X.shape
    n2, d2 = Y.shape
    if Ts is not None:
        Ts = _rowmajor(Ts.to(torch.float64))
        if tuple(Ts.shape) != (n, n2):
            raise ValueError(f"Ts {tuple(Ts.shape)} must be ({n}, {n2})")
    else:
        ts_diag = ts_diag.to(torch.float64).contiguous()
        if n != n2 or ts_diag.numel() != n:
            raise ValueError("diagonal Ts needs n == n2 == len(ts_diag)")
    mode = {"pot": 0, "fot": 1}[weights]
    M = torch.empty((d, d2), dtype=torch.float64, device=X.device)
    lib = L.lib()
    wsb = lib.otf_feature_cost_workspace_size(n, n2, d, d2)
    ws = torch.empty(wsb, dtype=torch.uint8, device=X.device)
    L.check(lib.otf_feature_cost_ex(
        X.data_ptr(), X.stride(0), Y.data_ptr(), Y.stride(0), _EMB_DT[edt], n, n2, d, d2, L.ptr(Ts),
        Ts.stride(0) if Ts is not None else 0, L.ptr(ts_diag), mode, M.data_ptr(), M.stride(0),
        ws.data_ptr(), wsb, L.stream_handle(X.device)), "otf_feature_cost_ex")
    return M


def coupled_cost(A: torch.Tensor, B: torch.Tensor, T: torch.Tensor, w1: torch.Tensor,
                 w2: torch.Tensor) -> torch.Tensor:
    """COOT cost ``M = (A*A) w1 [:, None] + (B*B) w2 [None, :] - 2 A T B^T`` in float64
    (perturbot utils.py:125-184 ``init_matrix_np`` + ``constC - hC1 T hC2^T``).

    A (p, r), B (q, s) are float32 and may be strided views (``X.T`` costs nothing);
    T (r, s), w1 (r,), w2 (s,) float64.
    """
    for t, nm in ((A, "A"), (B, "B"), (T, "T"), (w1, "w1"), (w2, "w2")):
        _dev(t, nm)
    if A.dtype != torch.float32:
        A = A.float()
    if B.dtype != torch.float32:
        B = B.float()
    p, r = A.shape
    q, s = B.shape
    T = _rowmajor(T.to(torch.float64))
    if tuple(T.shape) != (r, s):
        raise ValueError(f"T {tuple(T.shape)} must be ({r}, {s})")
    w1 = w1.to(torch.float64).contiguous()
    w2 = w2.to(torch.float64).contiguous()
    if w1.numel() != r or w2.numel() != s:
        raise ValueError("w1 / w2 must have len r / s")
    M = torch.empty((p, q), dtype=torch.float64, device=A.device)
    lib = L.lib()
    wsb = lib.otf_coupled_cost_workspace_size(p, q, r)
    ws = torch.empty(wsb, dtype=torch.uint8, device=A.device)
    L.check(lib.otf_coupled_cost(A.data_ptr(), A.stride(0), A.stride(1), B.data_ptr(), B.stride(0),
                                 B.stride(1), p, q, r, s, T.data_ptr(), T.stride(0), w1.data_ptr(),
                                 w2.data_ptr(), M.data_ptr(), M.stride(0), ws.data_ptr(), wsb,
                                 L.stream_handle(A.device)), "otf_coupled_cost")
    return M


def to_host(t: torch.Tensor) -> np.ndarray:
    """Device tensor -> NumPy through pinned memory: one DMA at the full PCIe rate instead
    of a pageable staging copy (the drop-ins return NumPy plans of up to 2048^2 float64
    = 34 MB per call).  Small tensors take the plain path."""
    if not t.is_cuda or t.numel() * t.element_size() < (1 << 20):
        return t.detach().cpu().numpy()
    h = torch.empty(t.shape, dtype=t.dtype, pin_memory=True)
    h.copy_(t.detach())
    return h.numpy()


# --------------------------------------------------------------------------- Sinkhorn
@dataclass
class SinkhornResult:
    u: torch.Tensor                 # POT: scaling u (u~ of the shifted kernel); OTT: potential f
    v: torch.Tensor                 # POT: scaling v (v~ of the shifted kernel); OTT: potential g
    plan: torch.Tensor | None
    info_dev: torch.Tensor          # int32[8] otf_sinkhorn_info on the device
    errlog_dev: torch.Tensor        # float64 marginal errors on the device
    flavor: str = "pot"
    # shifted kernel (opts.shift): base-2 exponent offsets A (n), B (m) in the workspace,
    # POT's scalings are u = 2^A u~, v = 2^B v~ (see pot_scalings)
    shift_a: torch.Tensor | None = None
    shift_b: torch.Tensor | None = None
    cost_max: torch.Tensor | None = None  # sinkhorn_pairwise: max of the unscaled cost (device)
    _info: dict | None = field(default=None, repr=False)

    @property
    def shifted(self) -> bool:
        return self.shift_a is not None

    def pot_scalings(self):
        """POT's scaling vectors ``(u, v)`` in float64 -- identical to ``(u, v)`` for a
        plain solve, ``(2^A u~, 2^B v~)`` for a shifted one (whose scalings can leave
        float32's range at small reg: v ~ exp(0.5 / reg) on a max-normalised cost)."""
        if self.flavor != "pot":
            raise ValueError("pot_scalings: POT-flavour results only")
        u, v = self.u.double(), self.v.double()
        if self.shifted:
            u = u * torch.exp2(self.shift_a.double())
            v = v * torch.exp2(self.shift_b.double())
        return u, v

    def info(self) -> dict:
        """Reads the device-side outcome (synchronises on first call)."""
        if self._info is None:
            vals = self.info_dev.cpu().tolist()
            d = dict(zip(L.INFO_FIELDS, vals))
            d["status_name"] = L.STATUS_NAMES.get(d["status"], "?")
            d["engine_name"] = L.ENGINE_NAMES.get(d["engine"], "?")
            if d["status"] == L.SK_TIMEOUT or d["stalled"]:
                raise L.OtfError("persistent Sinkhorn: a device-wide exchange made no progress "
                                 "for the stall limit (stalled=%d); results are invalid" % d["stalled"])
            if d["fallback"]:
                warnings.warn(
                    "persistent Sinkhorn engine could not become co-resident within OTF_REG_MS "
                    "(another persistent kernel held the CUs); the relay fallback solved the "
                    "problem instead (same POT result, slower: ~4 ms at 4096^2 float64)",
                    RuntimeWarning, stacklevel=2)
            if d["status"] == L.SK_RUNNING or not d["stop"]:
                # every engine writes a final status and stop = 1; a solve that left
                # them untouched never ran to its end (u, v, plan are uninitialised)
                raise L.OtfError("Sinkhorn: the solve reported no final status; results are "
                                 "invalid")
            d["err"] = self.errlog_dev[: max(d["n_err"], 0)].cpu().tolist()
            if (self.flavor == "pot" and self.u.dtype == torch.float32 and not self.shifted
                    and d["status"] == L.SK_NUMERICAL_BREAK and d["break_iter"] <= 1):
                warnings.warn(
                    "float32 POT Sinkhorn broke at iteration %d: a row or column of "
                    "K = exp(-C/reg) underflows (or its scaling overflows) in float32 -- POT's "
                    "float64 solve may not break there.  Use shift=True (the shifted kernel, "
                    "float32) or precision='fp64' for parity with the reference's float64 "
                    "path." % d["break_iter"],
                    RuntimeWarning, stacklevel=2)
            self._info = d
        return self._info


def sinkhorn_workspace_bytes(n: int, m: int, dtype, max_iter: int) -> int:
    return int(L.lib().otf_sinkhorn_workspace_size(n, m, _DT[dtype], max_iter))


_UNIFORM: dict = {}


def uniform(n: int, dtype, device) -> torch.Tensor:
    """The uniform marginal 1/n as a cached device tensor (read-only: the solves copy it
    into their workspace), so a training step does not pay a fill launch per marginal."""
    key = (int(n), dtype, torch.device(device))
    t = _UNIFORM.get(key)
    if t is None:
        t = _UNIFORM[key] = torch.full((int(n),), 1.0 / int(n), dtype=dtype, device=device)
    return t


def sinkhorn_workspace(n: int, m: int, dtype, max_iter: int, device) -> torch.Tensor:
    wsb = L.lib().otf_sinkhorn_workspace_size(n, m, _DT[dtype], max_iter)
    return torch.empty(wsb, dtype=torch.uint8, device=device)


# float32 POT switches to the shifted kernel when max(C / cost_scale) / reg exceeds
# SHIFT_RANGE: K = exp(-C/reg) stays in float32's normal range up to 87, the scalings
# (~exp(0.5 / reg) on a max-normalised cost) up to ~170; 64 keeps a margin to both.  Past
# SHIFT_RANGE_F64 POT's own float64 K has exact zeros (exp underflows below -745) and
# POT breaks on them; the plain float32 kernel reproduces that break, so it stays plain.
SHIFT_RANGE = 64.0
SHIFT_RANGE_F64 = 700.0
_SHIFT_ENGINES = ("auto", "mesh", "sweep", "stream")


def _cost_ratio(C: torch.Tensor, reg: float, cost_scale) -> float:
    """max(C / cost_scale) / reg.  A ``cost_scale`` tagged as max(C) (mark_cost_max: the
    library's cost builders) gives 1 / reg without touching C; otherwise one device
    reduction and a host read."""
    if cost_scale is not None and is_cost_max(cost_scale):
        return 1.0 / float(reg)
    cmax = float(C.amax()) if C.numel() else 0.0
    if cost_scale is not None:
        cs = float(cost_scale.reshape(-1)[0])
        cmax = cmax / cs if cs != 0.0 else (0.0 if cmax == 0.0 else float("inf"))
    return cmax / float(reg)


def _want_shift(C: torch.Tensor, reg: float, cost_scale, flavor: str, dt, engine: str,
                ratio: float | None = None) -> bool:
    if flavor != "pot" or dt != torch.float32 or engine not in _SHIFT_ENGINES:
        return False
    r = _cost_ratio(C, reg, cost_scale) if ratio is None else ratio
    return SHIFT_RANGE < r <= SHIFT_RANGE_F64


def sinkhorn(a: torch.Tensor, b: torch.Tensor, C: torch.Tensor, reg: float, max_iter: int = 1000,
             stop_thr: float = 1e-9, flavor: str = "pot", cost_scale: torch.Tensor | None = None,
             check_every: int = 10, err_squared: bool = False, sync_every: int = 0,
             want_plan: bool = True, plan_dtype=None, workspace: torch.Tensor | None = None,
             plan_out: torch.Tensor | None = None, engine: str = "auto",
             deterministic: bool = False, precision: str = "as_given",
             shift: bool | None = None) -> SinkhornResult:
    """Entropic OT on the device.  ``flavor="pot"`` is POT's sinkhorn_knopp (u, v scalings,
    revert-and-break), ``flavor="ott"`` OTT's lse-mode solver (potentials f, g).

    ``cost_scale`` (device scalar) divides the cost first (scale_cost="max_cost").
    Compute dtype = ``C.dtype`` (float32 or float64); a float16 ``C`` (fp16 cost
    storage, BASELINE config 5) is computed in float32.  ``deterministic=True``
    reduces the column sums in a fixed order without float atomics (gather / mesh engines
    by construction, else the sweep engine's fixed-order mode; POT flavour):
    bitwise-identical results run to run.

    ``precision``: "as_given" computes in C's dtype; "fp64" in float64 (the reference's
    POT path is float64 NumPy); "auto" computes a float32 / float16 POT solve in float32
    where that holds POT's result -- max(C / cost_scale) / reg <= SHIFT_RANGE, or the
    shifted kernel applies (below) -- and promotes it to float64 otherwise (past
    SHIFT_RANGE_F64, on an engine without the shifted kernel, or with ``shift=False``),
    where float32 kernel-domain POT would break at iteration 0 or lose the plan.

    ``shift`` (float32 POT only): run POT's iteration on the shifted kernel
    K~ = 2^(C ks + A_i + B_j) (include/otfuse.h opts.shift) -- the same iterates, with
    offsets from a log-domain first half-iteration, so that no plan entry that matters is
    formed from a flushed float32 exp and the scalings stay in range.  None (default)
    turns it on when SHIFT_RANGE (64) < max(C / cost_scale) / reg <= SHIFT_RANGE_F64 (700)
    on an engine that runs it (mesh, sweep, stream, AUTO): with ``cost_scale`` the ratio is
    taken as 1 / reg (C / cost_scale <= 1, scale_cost = "max_cost"), without it from
    C.amax() (one reduction and a host read).  Plain float32 kernel-domain POT
    moves the plan by 2.2e-3 at reg = 0.01 on the metric shape and breaks at iteration 0
    at reg = 5e-3; the shifted form holds 1e-4 of the float64 reference at both
    (tests/test_gpu_precision.py).  ``u``/``v`` of a shifted result are u~, v~;
    ``pot_scalings()`` gives POT's.
    """
    _dev(C, "C")
    if precision not in ("as_given", "fp64", "auto"):
        raise ValueError(f"precision must be 'as_given', 'fp64' or 'auto', not {precision!r}")
    if precision == "auto" and flavor == "pot" and C.dtype != torch.float64:
        ratio = _cost_ratio(C, reg, cost_scale)
        if ratio > SHIFT_RANGE:
            shifts = shift is not False and _want_shift(C, reg, cost_scale, flavor, torch.float32,
                                                        engine, ratio)
            if shifts:
                shift = True
            else:
                # promoted: the float64 solve needs no shift (and takes none: the shifted
                # kernel is a float32 form), whatever the caller asked for
                precision = "fp64"
                shift = False
    if precision == "fp64" and C.dtype != torch.float64:
        C = C.double()
        if cost_scale is not None:
            cost_scale = cost_scale.double()
        if workspace is not None and workspace.numel() < sinkhorn_workspace_bytes(C.shape[0], C.shape[1], torch.float64, max_iter):
            workspace = None
    if C.dtype not in _VEC:
        raise TypeError("C must be float16, float32 or float64")
    cost_f16 = C.dtype == torch.float16
    dt = torch.float32 if cost_f16 else C.dtype
    if shift is None:
        shift = _want_shift(C, reg, cost_scale, flavor, dt, engine)
    elif shift and (flavor != "pot" or dt != torch.float32):
        raise ValueError("shift: float32 POT-flavour solves only")
    n, m = C.shape
    C = _rowmajor(C, _VEC[C.dtype])
    a = _dev(a, "a").to(dt).contiguous()
    b = _dev(b, "b").to(dt).contiguous()
    if a.numel() != n or b.numel() != m:
        raise ValueError(f"a ({a.numel()}) / b ({b.numel()}) do not match C {tuple(C.shape)}")
    if cost_scale is not None:
        cost_scale = cost_scale.to(dt).contiguous()
    dev = C.device
    u = torch.empty(n, dtype=dt, device=dev)
    v = torch.empty(m, dtype=dt, device=dev)
    info = torch.empty(L.INFO_INT32S, dtype=torch.int32, device=dev)
    # written by the solve for every check it reports (info n_err): no zero fill needed
    errlog = torch.empty(max_iter // max(check_every, 1) + 2, dtype=torch.float64, device=dev)
    if workspace is None:
        workspace = sinkhorn_workspace(n, m, dt, max_iter, dev)
    P = None
    if want_plan:
        pdt = dt if plan_dtype is None else plan_dtype
        P = plan_out if plan_out is not None else _alloc_rowmajor(n, m, pdt, dev, 4)
        if P.dtype not in _DT or tuple(P.shape) != (n, m):
            raise ValueError("plan_out must be (n, m) float32/float64")
    opts = L.SinkhornOpts(reg=float(reg), stop_thr=float(stop_thr), max_iter=int(max_iter),
                          check_every=int(check_every),
                          flavor=L.OTF_FLAVOR_OTT if flavor == "ott" else L.OTF_FLAVOR_POT,
                          err_squared=int(err_squared), sync_every=int(sync_every),
                          engine=L.ENGINES[engine], cost_f16=int(cost_f16),
                          deterministic=int(bool(deterministic)), shift=int(bool(shift)))
    L.check(L.lib().otf_sinkhorn(
        a.data_ptr(), b.data_ptr(), C.data_ptr(), n, m, C.stride(0), _DT[dt], L.ptr(cost_scale),
        ctypes.byref(opts), u.data_ptr(), v.data_ptr(), L.ptr(P), P.stride(0) if P is not None else 0,
        _DT[P.dtype] if P is not None else 0, info.data_ptr(), errlog.data_ptr(),
        workspace.data_ptr(), workspace.numel(), L.stream_handle(dev)), "otf_sinkhorn")
    sa = sb = None
    if shift:
        oa, ob = ctypes.c_size_t(), ctypes.c_size_t()
        L.check(L.lib().otf_sinkhorn_shift_offsets(n, m, _DT[dt], int(max_iter), ctypes.byref(oa),
                                                   ctypes.byref(ob)), "otf_sinkhorn_shift_offsets")
        # views into the workspace: valid until the workspace is reused by another solve
        sa = workspace[oa.value: oa.value + 4 * n].view(torch.float32)
        sb = workspace[ob.value: ob.value + 4 * m].view(torch.float32)
    return SinkhornResult(u=u, v=v, plan=P, info_dev=info, errlog_dev=errlog, flavor=flavor,
                          shift_a=sa, shift_b=sb)


def sinkhorn_pairwise_workspace(n: int, m: int, max_iter: int, device, d: int | None = None,
                                precision: str = "fp64") -> torch.Tensor:
    if precision == "fp32":
        if d is None:
            raise ValueError("the float32 pairwise workspace depends on d")
        wsb = L.lib().otf_sinkhorn_pairwise_f32_workspace_size(n, m, d, max_iter)
    else:
        wsb = L.lib().otf_sinkhorn_pairwise_f64_workspace_size(n, m, max_iter)
    return torch.empty(wsb, dtype=torch.uint8, device=device)


def sinkhorn_pairwise(X: torch.Tensor, Y: torch.Tensor, reg: float, a: torch.Tensor | None = None,
                      b: torch.Tensor | None = None, metric: str = "sqeuclidean", scale_max: bool = True,
                      max_iter: int = 1000, stop_thr: float = 1e-9, check_every: int = 10,
                      err_squared: bool = False, want_plan: bool = True, plan_dtype=None,
                      workspace: torch.Tensor | None = None, plan_out: torch.Tensor | None = None,
                      engine: str = "auto", precision: str = "fp64") -> SinkhornResult:
    """The reference's cost + solve in float64, fused where the shape allows: POT's
    ``M = euclidean_distances(X, Y, squared=True); M /= M.max(); ot.sinkhorn(a, b, M, reg)``
    (MRI_PET_OT_nojax.py:70-75, :143) from float32 embeddings ``X`` (n, d), ``Y`` (m, d).

    For the float64 mesh's shapes (n = 512..4096 a power-of-two multiple of 128, m a
    multiple of 512 up to 4096, d a multiple of 16) every workgroup of the solve's launch
    builds its tile of the cost on the float64 matrix cores in its prologue (no n x m cost
    in HBM, otf_sinkhorn_pairwise_f64); other shapes run the cost and the solve as two
    calls.  ``a``/``b`` default to the uniform marginals.  The result's ``cost_max`` holds
    max(M) before the scaling (a device scalar).

    ``precision="fp32"``: the same segment in float32 compute (otf_sinkhorn_pairwise_f32): the
    split-fp16 cost (``pairwise_cost``'s) and the float32 POT engines, within 1e-4 of the
    float64 plan; with ``engine="mesh"`` and the float32 mesh's whole-tile shapes (n a multiple
    of 128, m a multiple of 512 up to 4096) the cost tiles are built in the solve's prologue,
    bitwise the two calls' results (AUTO runs the two calls: measured faster).  Where ``sinkhorn`` would take the shifted kernel (reg < 1/64 with
    ``scale_max``; and without ``scale_max``) the two calls run.  ``plan_dtype`` defaults to
    the compute precision (float64 / float32)."""
    _dev(X, "X")
    _dev(Y, "Y")
    if metric not in ("sqeuclidean", "euclidean"):
        raise ValueError(f"metric {metric!r} not supported (sqeuclidean | euclidean)")
    if X.dim() != 2 or Y.dim() != 2 or X.shape[1] != Y.shape[1]:
        raise ValueError(f"X {tuple(X.shape)} and Y {tuple(Y.shape)} must be (n, d) and (m, d)")
    if precision not in ("fp64", "fp32"):
        raise ValueError(f"precision {precision!r} (fp64 | fp32)")
    if precision == "fp32":
        return _sinkhorn_pairwise_f32(X, Y, reg, a, b, metric, scale_max, max_iter, stop_thr, check_every,
                                      err_squared, want_plan, plan_dtype, workspace, plan_out, engine)
    if plan_dtype is None:
        plan_dtype = torch.float64
    X = X.float().contiguous()
    Y = Y.float().contiguous()
    n, d = X.shape
    m = Y.shape[0]
    dev = X.device
    a = uniform(n, torch.float64, dev) if a is None else _dev(a, "a").double().contiguous()
    b = uniform(m, torch.float64, dev) if b is None else _dev(b, "b").double().contiguous()
    if a.numel() != n or b.numel() != m:
        raise ValueError(f"a ({a.numel()}) / b ({b.numel()}) do not match ({n}, {m})")
    u = torch.empty(n, dtype=torch.float64, device=dev)
    v = torch.empty(m, dtype=torch.float64, device=dev)
    cmax = torch.empty(1, dtype=torch.float64, device=dev)
    info = torch.empty(L.INFO_INT32S, dtype=torch.int32, device=dev)
    errlog = torch.empty(max_iter // max(check_every, 1) + 2, dtype=torch.float64, device=dev)
    if workspace is None:
        workspace = sinkhorn_pairwise_workspace(n, m, max_iter, dev)
    P = None
    if want_plan:
        P = plan_out if plan_out is not None else _alloc_rowmajor(n, m, plan_dtype, dev, 4)
        if P.dtype not in _DT or tuple(P.shape) != (n, m):
            raise ValueError("plan_out must be (n, m) float32/float64")
    opts = L.SinkhornOpts(reg=float(reg), stop_thr=float(stop_thr), max_iter=int(max_iter),
                          check_every=int(check_every), flavor=L.OTF_FLAVOR_POT,
                          err_squared=int(err_squared), sync_every=0, engine=L.ENGINES[engine],
                          cost_f16=0, deterministic=0, shift=0)
    met = L.OTF_EUCLIDEAN if metric == "euclidean" else L.OTF_SQEUCLIDEAN
    L.check(L.lib().otf_sinkhorn_pairwise_f64(
        X.data_ptr(), X.stride(0), Y.data_ptr(), Y.stride(0), n, m, d, met, int(bool(scale_max)),
        a.data_ptr(), b.data_ptr(), ctypes.byref(opts), u.data_ptr(), v.data_ptr(), L.ptr(P),
        P.stride(0) if P is not None else 0, _DT[P.dtype] if P is not None else 0, cmax.data_ptr(),
        info.data_ptr(), errlog.data_ptr(), workspace.data_ptr(), workspace.numel(),
        L.stream_handle(dev)), "otf_sinkhorn_pairwise_f64")
    return SinkhornResult(u=u, v=v, plan=P, info_dev=info, errlog_dev=errlog, flavor="pot", cost_max=cmax)


def _sinkhorn_pairwise_f32(X, Y, reg, a, b, metric, scale_max, max_iter, stop_thr, check_every, err_squared,
                           want_plan, plan_dtype, workspace, plan_out, engine) -> SinkhornResult:
    """sinkhorn_pairwise(precision="fp32"): otf_sinkhorn_pairwise_f32, or -- where the float32
    solve takes the shifted kernel -- pairwise_cost + sinkhorn (the same two calls)."""
    X = _rowmajor(X.float(), 4)
    Y = _rowmajor(Y.float(), 4)
    n, d = X.shape
    m = Y.shape[0]
    dev = X.device
    a = uniform(n, torch.float32, dev) if a is None else _dev(a, "a").float().contiguous()
    b = uniform(m, torch.float32, dev) if b is None else _dev(b, "b").float().contiguous()
    if a.numel() != n or b.numel() != m:
        raise ValueError(f"a ({a.numel()}) / b ({b.numel()}) do not match ({n}, {m})")
    pdt = torch.float32 if plan_dtype is None else plan_dtype
    if not scale_max or 1.0 / float(reg) > SHIFT_RANGE:
        # the shifted kernel (or, unscaled, the test for it) needs a pass over C: the two calls,
        # sinkhorn deciding the shift as it does for any float32 cost
        C, cmax = pairwise_cost(X, Y, metric, zero_diag=False)
        return sinkhorn(a, b, C, reg, max_iter=max_iter, stop_thr=stop_thr, check_every=check_every,
                        err_squared=err_squared, cost_scale=cmax if scale_max else None, want_plan=want_plan,
                        plan_dtype=pdt, plan_out=plan_out, engine=engine)
    u = torch.empty(n, dtype=torch.float32, device=dev)
    v = torch.empty(m, dtype=torch.float32, device=dev)
    cmax = torch.empty(1, dtype=torch.float32, device=dev)
    info = torch.empty(L.INFO_INT32S, dtype=torch.int32, device=dev)
    errlog = torch.empty(max_iter // max(check_every, 1) + 2, dtype=torch.float64, device=dev)
    if workspace is None:
        workspace = sinkhorn_pairwise_workspace(n, m, max_iter, dev, d=d, precision="fp32")
    P = None
    if want_plan:
        P = plan_out if plan_out is not None else _alloc_rowmajor(n, m, pdt, dev, 4)
        if P.dtype not in _DT or tuple(P.shape) != (n, m):
            raise ValueError("plan_out must be (n, m) float32/float64")
    opts = L.SinkhornOpts(reg=float(reg), stop_thr=float(stop_thr), max_iter=int(max_iter),
                          check_every=int(check_every), flavor=L.OTF_FLAVOR_POT,
                          err_squared=int(err_squared), sync_every=0, engine=L.ENGINES[engine],
                          cost_f16=0, deterministic=0, shift=0)
    met = L.OTF_EUCLIDEAN if metric == "euclidean" else L.OTF_SQEUCLIDEAN
    L.check(L.lib().otf_sinkhorn_pairwise_f32(
        X.data_ptr(), X.stride(0), Y.data_ptr(), Y.stride(0), n, m, d, met, int(bool(scale_max)),
        a.data_ptr(), b.data_ptr(), ctypes.byref(opts), u.data_ptr(), v.data_ptr(), L.ptr(P),
        P.stride(0) if P is not None else 0, _DT[P.dtype] if P is not None else 0, cmax.data_ptr(),
        info.data_ptr(), errlog.data_ptr(), workspace.data_ptr(), workspace.numel(),
        L.stream_handle(dev)), "otf_sinkhorn_pairwise_f32")
    return SinkhornResult(u=u, v=v, plan=P, info_dev=info, errlog_dev=errlog, flavor="pot",
                          cost_max=mark_cost_max(cmax))


def sinkhorn_profile(a, b, C, reg, iters, cost_scale=None, flavor="pot", workspace=None) -> float:
    """Runs exactly ``iters`` iterations with a HIP event pair around every pass;
    returns the mean pass duration in ms (bench.py's roofline probe)."""
    cost_f16 = C.dtype == torch.float16
    dt = torch.float32 if cost_f16 else C.dtype
    n, m = C.shape
    C = _rowmajor(C, _VEC[C.dtype])
    a = a.to(dt).contiguous()
    b = b.to(dt).contiguous()
    if cost_scale is not None:
        cost_scale = cost_scale.to(dt).contiguous()
    u = torch.empty(n, dtype=dt, device=C.device)
    v = torch.empty(m, dtype=dt, device=C.device)
    info = torch.empty(L.INFO_INT32S, dtype=torch.int32, device=C.device)
    if workspace is None:
        workspace = sinkhorn_workspace(n, m, dt, iters, C.device)
    opts = L.SinkhornOpts(reg=float(reg), stop_thr=-1.0, max_iter=int(iters), check_every=10,
                          flavor=L.OTF_FLAVOR_OTT if flavor == "ott" else L.OTF_FLAVOR_POT,
                          err_squared=0, sync_every=0, engine=L.ENGINE_STREAM,
                          cost_f16=int(cost_f16))
    avg = ctypes.c_float(0.0)
    L.check(L.lib().otf_sinkhorn_profile(
        a.data_ptr(), b.data_ptr(), C.data_ptr(), n, m, C.stride(0), _DT[dt], L.ptr(cost_scale),
        ctypes.byref(opts), u.data_ptr(), v.data_ptr(), info.data_ptr(), workspace.data_ptr(),
        workspace.numel(), ctypes.byref(avg), L.stream_handle(C.device)), "otf_sinkhorn_profile")
    return float(avg.value)


# --------------------------------------------------------------------------- plan use
def plan_postprocess(T: torch.Tensor, nan_fill: float = 1e-8, rownorm: bool = True) -> torch.Tensor:
    """MRI_PET_OT_nojax.py:702-715: float32 cast, NaN -> 1e-8, row normalisation."""
    _dev(T, "T")
    T = _rowmajor(T if T.dtype in _DT else T.double())
    d, d2 = T.shape
    Tn = torch.empty((d, d2), dtype=torch.float32, device=T.device)
    L.check(L.lib().otf_plan_postprocess(T.data_ptr(), d, d2, T.stride(0), _DT[T.dtype],
                                         float(nan_fill), int(rownorm), Tn.data_ptr(), Tn.stride(0),
                                         L.stream_handle(T.device)), "otf_plan_postprocess")
    return Tn


def gemm_f32(A: torch.Tensor, B: torch.Tensor, transpose_b: bool = False) -> torch.Tensor:
    """``A @ B`` (or ``A @ B^T``) in float32 on the HIP GEMM kernel."""
    A = _dev(A, "A").float()
    B = _dev(B, "B").float()
    M, K = A.shape
    if transpose_b:
        N, K2 = B.shape
        sb0, sb1 = B.stride(1), B.stride(0)
    else:
        K2, N = B.shape
        sb0, sb1 = B.stride(0), B.stride(1)
    if K != K2:
        raise ValueError(f"inner dimensions differ: {K} vs {K2}")
    out = torch.empty((M, N), dtype=torch.float32, device=A.device)
    L.check(L.lib().otf_gemm_f32(A.data_ptr(), A.stride(0), A.stride(1), B.data_ptr(), sb0, sb1,
                                 out.data_ptr(), out.stride(0), M, N, K, 1.0, 0.0,
                                 L.stream_handle(A.device)), "otf_gemm_f32")
    return out


def cosine_align(X: torch.Tensor, Y: torch.Tensor, ok: torch.Tensor | None = None,
                 sk_info: torch.Tensor | None = None):
    """``1 - mean_b cos(X_b, Y_b)`` with torch's normalize / cosine_similarity clamps
    (cosine_loss, MRI_PET_OT_nojax.py:552-560) and its gradients, in ONE launch
    (otf_cosine_align).  X: (B, d) float32 / bfloat16 / float16 (read as stored), Y:
    (B, d) float32.  ``ok`` (device bool scalar, optional) and a non-finite loss give
    an exact-zero loss and gradients (the NaN -> 0 swap of :724-725); so does a solve
    that did not finish when ``sk_info`` (the SinkhornResult's device info words) is
    given -- checked inside the same launch.
    Returns ``(loss (0-dim float32), gx (B, d), gy (B, d), keep (uint8 scalar))``."""
    _dev(X, "X")
    _dev(Y, "Y")
    if X.dim() == 1:
        X = X.unsqueeze(0)
    if Y.dim() == 1:
        Y = Y.unsqueeze(0)
    if X.dtype not in _EMB_DT:
        X = X.float()
    X = X.contiguous()
    Y = Y.float().contiguous()
    B, d = X.shape
    if tuple(Y.shape) != (B, d):
        raise ValueError(f"X {tuple(X.shape)} and Y {tuple(Y.shape)} differ")
    dev = X.device
    loss = torch.empty((), dtype=torch.float32, device=dev)
    gx = torch.empty((B, d), dtype=torch.float32, device=dev)
    gy = torch.empty((B, d), dtype=torch.float32, device=dev)
    keep = torch.empty((), dtype=torch.uint8, device=dev)
    okp = None
    if ok is not None:
        ok = _dev(ok, "ok").to(torch.uint8).reshape(())
        okp = ok.data_ptr()
    infop = None
    if sk_info is not None:
        if sk_info.dtype != torch.int32 or sk_info.numel() < L.INFO_INT32S or not sk_info.is_contiguous():
            raise ValueError("sk_info must be a SinkhornResult's contiguous int32 info words")
        infop = _dev(sk_info, "sk_info").data_ptr()
    L.check(L.lib().otf_cosine_align(X.data_ptr(), X.stride(0), _EMB_DT[X.dtype], Y.data_ptr(),
                                     Y.stride(0), B, d, okp, infop, loss.data_ptr(), gx.data_ptr(), d,
                                     gy.data_ptr(), d, keep.data_ptr(), L.stream_handle(dev)),
            "otf_cosine_align")
    return loss, gx, gy, keep


def ot_align_backward(gx: torch.Tensor, gy: torch.Tensor, Tn: torch.Tensor,
                      g_loss: torch.Tensor | None = None, g_ot: torch.Tensor | None = None,
                      keep: torch.Tensor | None = None):
    """Backward of ``ot = pet @ Tn^T`` under the alignment loss in ONE launch
    (otf_ot_align_backward): ``g_pet = (g_loss * gy + g_ot) @ Tn``, ``g_mri = g_loss * gx``.
    Without ``g_ot`` and with ``keep == 0`` g_pet is exact zeros (Tn may hold NaN)."""
    for t, nm in ((gx, "gx"), (gy, "gy"), (Tn, "Tn")):
        _dev(t, nm)
    gx = gx.float().contiguous()
    gy = gy.float().contiguous()
    Tn = Tn.float().contiguous()
    B, d = gy.shape
    d_, d2 = Tn.shape
    if d_ != d or tuple(gx.shape) != (B, d):
        raise ValueError("gx / gy (B, d) and Tn (d, d2) do not match")
    dev = gy.device
    if g_loss is not None:
        g_loss = g_loss.float().reshape(()).contiguous()
    if g_ot is not None:
        g_ot = g_ot.float().contiguous()
        if tuple(g_ot.shape) != (B, d):
            raise ValueError("g_ot must be (B, d)")
    g_mri = torch.empty((B, d), dtype=torch.float32, device=dev)
    g_pet = torch.empty((B, d2), dtype=torch.float32, device=dev)
    L.check(L.lib().otf_ot_align_backward(
        gx.data_ptr(), d, gy.data_ptr(), d, L.ptr(g_ot), d, L.ptr(g_loss), L.ptr(keep),
        Tn.data_ptr(), Tn.stride(0), B, d, d2, g_mri.data_ptr(), d, g_pet.data_ptr(), d2,
        L.stream_handle(dev)), "otf_ot_align_backward")
    return g_mri, g_pet


def plan_postprocess_apply(T: torch.Tensor, Z: torch.Tensor, nan_fill: float = 1e-8,
                           rownorm: bool = True):
    """Fused MRI_PET_OT_nojax.py:702-718 in one pass over the plan: returns
    ``(Z @ Tn^T, Tn)`` with Tn the post-processed float32 plan (NaN -> nan_fill, rows
    normalised, zero rows -> 1e-8) -- otf_plan_postprocess_apply."""
    _dev(T, "T")
    _dev(Z, "Z")
    T = _rowmajor(T if T.dtype in (torch.float32, torch.float64) else T.double())
    Z = Z.float().contiguous()
    d, d2 = T.shape
    B = Z.shape[0]
    if Z.dim() != 2 or Z.shape[1] != d2:
        raise ValueError(f"Z {tuple(Z.shape)} must be (B, {d2})")
    out = torch.empty((B, d), dtype=torch.float32, device=T.device)
    Tn = torch.empty((d, d2), dtype=torch.float32, device=T.device)
    L.check(L.lib().otf_plan_postprocess_apply(
        T.data_ptr(), d, d2, T.stride(0), _DT[T.dtype], float(nan_fill), int(rownorm), Z.data_ptr(),
        Z.stride(0), B, out.data_ptr(), out.stride(0), Tn.data_ptr(), Tn.stride(0),
        L.stream_handle(T.device)), "otf_plan_postprocess_apply")
    return out, Tn


class PostprocessApply(torch.autograd.Function):
    """``Z @ Tn^T`` with Tn = post-processed raw plan T (constant): one fused kernel
    forward, ``G @ Tn`` backward (MRI_PET_OT_nojax.py:702-718)."""

    @staticmethod
    def forward(ctx, Z, T):
        out, Tn = plan_postprocess_apply(T, Z)
        ctx.save_for_backward(Tn)
        ctx.zdtype = Z.dtype
        ctx.mark_non_differentiable(Tn)
        return out, Tn

    @staticmethod
    def backward(ctx, grad, _gtn):
        (Tn,) = ctx.saved_tensors
        return gemm_f32(grad.contiguous(), Tn).to(ctx.zdtype), None


class PlanApply(torch.autograd.Function):
    """``Z @ T^T`` with a constant plan T (MRI_PET_OT_nojax.py:718); backward ``G @ T``."""

    @staticmethod
    def forward(ctx, Z, T):
        ctx.save_for_backward(T)
        return gemm_f32(Z, T, transpose_b=True)

    @staticmethod
    def backward(ctx, grad):
        (T,) = ctx.saved_tensors
        return gemm_f32(grad.contiguous(), T), None


def apply_plan(Z: torch.Tensor, T: torch.Tensor) -> torch.Tensor:
    return PlanApply.apply(Z, T.detach())


# ---------------------------------------------------------------- exact EMD
@dataclass
class EmdResult:
    """Plans (device float64) of a batched ``otf_emd_solve``; ``infos()`` syncs."""
    plans: list
    info_raw: torch.Tensor
    _keep: list = field(default_factory=list, repr=False)

    def infos(self):
        raw = self.info_raw.cpu().numpy().tobytes()
        out = []
        for b in range(len(self.plans)):
            rec = raw[24 * b:24 * (b + 1)]
            cost = float(np.frombuffer(rec[0:8], np.float64)[0])
            status, piv = (int(x) for x in np.frombuffer(rec[8:16], np.int32))
            art = float(np.frombuffer(rec[16:24], np.float64)[0])
            out.append({"cost": cost, "status": status, "status_name": L.EMD_STATUS.get(status, str(status)),
                        "n_pivots": piv, "max_artificial_flow": art})
        return out


def emd_max_nodes() -> int:
    """Largest n + m + 1 of an exact EMD (n * m + n + m < 2^31 must hold as well)."""
    return int(L.lib().otf_emd_max_nodes())


def emd_lds_nodes() -> int:
    """n + m + 1 up to which the network simplex keeps its tree in LDS."""
    return int(L.lib().otf_emd_lds_nodes())


def emd_batched(problems, max_pivots: int = 100000) -> EmdResult:
    """Exact EMD for each ``(a, b, M)`` (device float64; b already scaled to a's mass):
    one workgroup per problem, one launch per 64 problems (``otf_emd_solve``)."""
    if len(problems) == 0:
        raise ValueError("no problems")
    keep, plans = [], []
    probs = (L.EmdProblem * len(problems))()
    dev = None
    for k, (a, b, M) in enumerate(problems):
        M = _dev(M, "M").to(torch.float64).contiguous()
        dev = M.device
        n, m = M.shape
        a = a.to(dev, torch.float64).contiguous()
        b = b.to(dev, torch.float64).contiguous()
        if a.numel() != n or b.numel() != m:
            raise ValueError(f"a ({a.numel()}) / b ({b.numel()}) do not match M {tuple(M.shape)}")
        if n + m + 1 > emd_max_nodes() or n * m + n + m >= 2 ** 31 - 1:
            raise NotImplementedError(f"EMD {n}x{m}: n * m + n + m must be < 2^31")
        T = torch.empty((n, m), dtype=torch.float64, device=dev)
        plans.append(T)
        keep += [a, b, M]
        probs[k] = L.EmdProblem(a.data_ptr(), b.data_ptr(), M.data_ptr(), M.stride(0), T.data_ptr(),
                                T.stride(0), n, m)
    info = torch.zeros(24 * len(problems), dtype=torch.uint8, device=dev)
    L.check(L.lib().otf_emd_solve(len(problems), probs, int(max_pivots), info.data_ptr(),
                                  L.stream_handle(dev)), "otf_emd_solve")
    return EmdResult(plans, info, keep)
