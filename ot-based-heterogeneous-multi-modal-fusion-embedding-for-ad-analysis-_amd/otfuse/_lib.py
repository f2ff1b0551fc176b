"""ctypes binding of ``libotfuse.so`` — the C ABI declared in ``include/otfuse.h``.

The library is the product: every op in this package calls into it and there is
no CPU fallback.  ``lib()`` raises if the shared object is missing, so a GPU box
without the built extension fails loudly instead of silently computing elsewhere.

``torch`` is imported first on purpose: PyTorch-ROCm ships its own
``libamdhip64.so`` (soname ``libamdhip64.so.7``); loading it before
``libotfuse.so`` makes the dynamic linker bind our NEEDED entry to the same HIP
runtime, so torch's device pointers and streams are valid on our side.
"""
from __future__ import annotations

import ctypes
import os
import re

import torch  # noqa: F401  (must precede the CDLL load, see module docstring)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "lib", "libotfuse.so")
HEADER_PATH = os.path.abspath(os.path.join(_HERE, "..", "..", "include", "otfuse.h"))

OTF_OK, OTF_EINVAL, OTF_EUNSUPPORTED, OTF_EHIP = 0, 1, 2, -1
OTF_F32, OTF_F64, OTF_F16, OTF_BF16 = 0, 1, 2, 3
OTF_SQEUCLIDEAN, OTF_EUCLIDEAN = 0, 1
OTF_FLAVOR_POT, OTF_FLAVOR_OTT = 0, 1
OTF_RED_SUM, OTF_RED_MAX = 0, 1
COMM_ID_BYTES = 128
SK_RUNNING, SK_CONVERGED, SK_MAX_ITER, SK_NUMERICAL_BREAK, SK_TIMEOUT = 0, 1, 2, 3, 4
STATUS_NAMES = {0: "running", 1: "converged", 2: "max_iter", 3: "numerical_break",
                4: "timeout"}
ENGINE_AUTO, ENGINE_STREAM, ENGINE_RESIDENT, ENGINE_TILED, ENGINE_SWEEP, ENGINE_GATHER, ENGINE_MESH = (
    0, 1, 2, 3, 4, 5, 6)
ENGINES = {"auto": ENGINE_AUTO, "stream": ENGINE_STREAM, "resident": ENGINE_RESIDENT,
           "tiled": ENGINE_TILED, "sweep": ENGINE_SWEEP, "gather": ENGINE_GATHER,
           "mesh": ENGINE_MESH}
ENGINE_NAMES = {v: k for k, v in ENGINES.items()}


class SinkhornOpts(ctypes.Structure):
    _fields_ = [("reg", ctypes.c_double), ("stop_thr", ctypes.c_double),
                ("max_iter", ctypes.c_int32), ("check_every", ctypes.c_int32),
                ("flavor", ctypes.c_int32), ("err_squared", ctypes.c_int32),
                ("sync_every", ctypes.c_int32), ("engine", ctypes.c_int32),
                ("cost_f16", ctypes.c_int32), ("n_total", ctypes.c_int32),
                ("deterministic", ctypes.c_int32), ("shift", ctypes.c_int32)]


class GwOpts(ctypes.Structure):
    _fields_ = [("solver", ctypes.c_int32), ("max_iter", ctypes.c_int32),
                ("min_iter", ctypes.c_int32), ("sk_max_iter", ctypes.c_int32),
                ("sk_inner", ctypes.c_int32), ("warm_start", ctypes.c_int32),
                ("tol_rel", ctypes.c_double), ("tol_abs", ctypes.c_double),
                ("threshold", ctypes.c_double), ("sk_threshold", ctypes.c_double),
                ("eps", ctypes.c_double)]


class GwProblem(ctypes.Structure):
    _fields_ = [("C1", ctypes.c_void_p), ("ldc1", ctypes.c_int64),
                ("C2", ctypes.c_void_p), ("ldc2", ctypes.c_int64),
                ("p", ctypes.c_void_p), ("q", ctypes.c_void_p),
                ("labels_a", ctypes.c_void_p), ("labels_b", ctypes.c_void_p),
                ("T", ctypes.c_void_p), ("ldt", ctypes.c_int64),
                ("n", ctypes.c_int64), ("m", ctypes.c_int64)]


class EmdProblem(ctypes.Structure):
    _fields_ = [("a", ctypes.c_void_p), ("b", ctypes.c_void_p),
                ("M", ctypes.c_void_p), ("ldm", ctypes.c_int64),
                ("T", ctypes.c_void_p), ("ldt", ctypes.c_int64),
                ("n", ctypes.c_int32), ("m", ctypes.c_int32)]


EMD_STATUS = {0: "optimal", 1: "max_iter", 2: "infeasible", 3: "unbounded"}

INFO_FIELDS = ("stop", "last_good", "niter", "status", "n_err", "break_iter", "engine", "stalled",
               "fallback")
INFO_INT32S = len(INFO_FIELDS)  # otf_sinkhorn_info is 9 x int32

_vp = ctypes.c_void_p
_i64 = ctypes.c_int64
_i32 = ctypes.c_int32
_SIGS = {
    "otf_version": (ctypes.c_char_p, []),
    "otf_cost_pairwise": (ctypes.c_int, [_vp, _i64, _vp, _i64, _i64, _i64, _i64, _i32, _i32, _vp,
                                         _i64, _vp, _vp]),
    "otf_cost_split16_workspace_size": (ctypes.c_size_t, [_i64, _i64, _i64]),
    "otf_cost_pairwise_split16": (ctypes.c_int, [_vp, _i64, _vp, _i64, _i64, _i64, _i64, _i32,
                                                 _i32, _vp, _i64, _vp, _vp, ctypes.c_size_t, _vp]),
"otf_cost_ex_workspace_size": (ctypes.c_size_t, [_i64, _i64, _i64, _i32]),
    "otf_cost_pairwise_ex": (ctypes.c_int, [_vp, _i64, _vp, _i64, _i32, _i64, _i64, _i64, _i32, _i32,
                                            _vp, _i64, _i32, _vp, _vp, _vp, ctypes.c_size_t, _vp]),
    "otf_scale_inplace": (ctypes.c_int, [_vp, _i64, _i64, _i64, _i32, _vp, _vp]),
    "otf_feature_cost_workspace_size": (ctypes.c_size_t, [_i64, _i64, _i64, _i64]),
    "otf_feature_cost": (ctypes.c_int, [_vp, _i64, _vp, _i64, _i64, _i64, _i64, _i64, _vp, _i64,
                                        _vp, _i32, _vp, _i64, _vp, ctypes.c_size_t, _vp]),
    "otf_feature_cost_ex": (ctypes.c_int, [_vp, _i64, _vp, _i64, _i32, _i64, _i64, _i64, _i64, _vp,
                                           _i64, _vp, _i32, _vp, _i64, _vp, ctypes.c_size_t, _vp]),
    "otf_coupled_cost_workspace_size": (ctypes.c_size_t, [_i64, _i64, _i64]),
    "otf_coupled_cost": (ctypes.c_int, [_vp, _i64, _i64, _vp, _i64, _i64, _i64, _i64, _i64, _i64,
                                        _vp, _i64, _vp, _vp, _vp, _i64, _vp, ctypes.c_size_t,
                                        _vp]),
    "otf_sinkhorn_workspace_size": (ctypes.c_size_t, [_i64, _i64, _i32, _i32]),
    "otf_sinkhorn_shift_offsets": (ctypes.c_int, [_i64, _i64, _i32, _i32, ctypes.POINTER(ctypes.c_size_t),
                                                  ctypes.POINTER(ctypes.c_size_t)]),
    "otf_sinkhorn_fallback_count": (ctypes.c_int, [ctypes.POINTER(ctypes.c_uint64)]),
    "otf_sinkhorn": (ctypes.c_int, [_vp, _vp, _vp, _i64, _i64, _i64, _i32, _vp,
                                    ctypes.POINTER(SinkhornOpts), _vp, _vp, _vp, _i64, _i32, _vp,
                                    _vp, _vp, ctypes.c_size_t, _vp]),
    "otf_sinkhorn_profile": (ctypes.c_int, [_vp, _vp, _vp, _i64, _i64, _i64, _i32, _vp,
                                            ctypes.POINTER(SinkhornOpts), _vp, _vp, _vp, _vp,
                                            ctypes.c_size_t, ctypes.POINTER(ctypes.c_float), _vp]),
    "otf_sinkhorn_pass": (ctypes.c_int, [_vp, _vp, _vp, _i64, _i64, _i64, _i32, _vp,
                                         ctypes.POINTER(SinkhornOpts), _i32, _vp, _vp, _vp,
                                         ctypes.c_size_t, ctypes.POINTER(ctypes.c_void_p),
                                         ctypes.POINTER(ctypes.c_int64), _vp]),
    "otf_sinkhorn_finish": (ctypes.c_int, [_vp, _vp, _vp, _i64, _i64, _i64, _i32, _vp,
                                           ctypes.POINTER(SinkhornOpts), _vp, _vp, _vp, _i64, _i32,
                                           _vp, _vp, _vp, ctypes.c_size_t, _vp]),
    "otf_comm_unique_id": (ctypes.c_int, [_vp]),
    "otf_comm_init": (ctypes.c_int, [ctypes.POINTER(ctypes.c_void_p), _vp, _i32, _i32]),
    "otf_comm_destroy": (ctypes.c_int, [_vp]),
    "otf_comm_all_reduce": (ctypes.c_int, [_vp, _i64, _i32, _i32, _vp, _vp]),
    "otf_comm_all_gather": (ctypes.c_int, [_vp, _vp, _i64, _i32, _vp, _vp]),
    "otf_sinkhorn_row_sharded": (ctypes.c_int, [_vp, _vp, _vp, _i64, _i64, _i64, _i32, _vp,
                                                ctypes.POINTER(SinkhornOpts), _vp, _vp, _vp, _vp,
                                                _i64, _i32, _vp, _vp, _vp, ctypes.c_size_t, _vp]),
    "otf_cost_last_phases": (ctypes.c_int, [ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_float)]),
    "otf_xpeer_handle_size": (ctypes.c_size_t, []),
    "otf_xpeer_create": (ctypes.c_int, [_i32, _i32, _i64, ctypes.POINTER(ctypes.c_void_p), _vp]),
    "otf_xpeer_connect": (ctypes.c_int, [_vp, _vp]),
    "otf_xpeer_destroy": (ctypes.c_int, [_vp]),
    "otf_sinkhorn_xsweep": (ctypes.c_int, [_vp, _vp, _vp, _i64, _i64, _i64, _i32, _vp,
                                           ctypes.POINTER(SinkhornOpts), _vp, _vp, _vp, _vp, _i64,
                                           _i32, _vp, _vp, _vp, ctypes.c_size_t, _vp]),
    "otf_plan_postprocess": (ctypes.c_int, [_vp, _i64, _i64, _i64, _i32, ctypes.c_float, _i32,
                                            _vp, _i64, _vp]),
    "otf_plan_postprocess_apply": (ctypes.c_int, [_vp, _i64, _i64, _i64, _i32, ctypes.c_float, _i32,
                                                  _vp, _i64, _i64, _vp, _i64, _vp, _i64, _vp]),
    "otf_gemm_f32": (ctypes.c_int, [_vp, _i64, _i64, _vp, _i64, _i64, _vp, _i64, _i64, _i64, _i64,
                                    ctypes.c_float, ctypes.c_float, _vp]),
    "otf_cosine_align": (ctypes.c_int, [_vp, _i64, _i32, _vp, _i64, _i64, _i64, _vp, _vp, _vp, _vp,
                                        _i64, _vp, _i64, _vp, _vp]),
    "otf_ot_align_backward": (ctypes.c_int, [_vp, _i64, _vp, _i64, _vp, _i64, _vp, _vp, _vp, _i64,
                                             _i64, _i64, _i64, _vp, _i64, _vp, _i64, _vp]),
    "otf_cost_pairwise_f64_workspace_size": (ctypes.c_size_t, [ctypes.c_int64, ctypes.c_int64]),
    "otf_cost_pairwise_f64": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p,
                                             ctypes.c_int64, ctypes.c_int64, ctypes.c_int64,
                                             ctypes.c_int64, ctypes.c_int32, ctypes.c_int32,
                                             ctypes.c_int32, ctypes.c_void_p, ctypes.c_int64,
                                             ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                             ctypes.c_void_p]),
    "otf_sinkhorn_pairwise_f64_workspace_size": (ctypes.c_size_t, [_i64, _i64, _i32]),
    "otf_sinkhorn_pairwise_f64": (ctypes.c_int, [_vp, _i64, _vp, _i64, _i64, _i64, _i64, _i32, _i32, _vp, _vp,
                                                 ctypes.POINTER(SinkhornOpts), _vp, _vp, _vp, _i64, _i32, _vp,
                                                 _vp, _vp, _vp, ctypes.c_size_t, _vp]),
    "otf_sinkhorn_pairwise_f32_workspace_size": (ctypes.c_size_t, [_i64, _i64, _i64, _i32]),
    "otf_sinkhorn_pairwise_f32": (ctypes.c_int, [_vp, _i64, _vp, _i64, _i64, _i64, _i64, _i32, _i32, _vp, _vp,
                                                 ctypes.POINTER(SinkhornOpts), _vp, _vp, _vp, _i64, _i32, _vp,
                                                 _vp, _vp, _vp, ctypes.c_size_t, _vp]),
    "otf_emd_max_nodes": (ctypes.c_int, []),
    "otf_emd_lds_nodes": (ctypes.c_int, []),
    "otf_emd_solve": (ctypes.c_int, [_i32, ctypes.POINTER(EmdProblem), _i64, _vp, _vp]),
    "otf_gw_workspace_size": (ctypes.c_size_t, [ctypes.c_int32, ctypes.POINTER(GwProblem)]),
    "otf_gw_solve": (ctypes.c_int, [ctypes.c_int32, ctypes.POINTER(GwProblem),
                                    ctypes.POINTER(GwOpts), ctypes.c_void_p, ctypes.c_void_p,
                                    ctypes.c_int32, ctypes.c_void_p, ctypes.c_size_t,
                                    ctypes.c_void_p]),
}

_lib = None


class OtfError(RuntimeError):
    pass


def lib():
    """Load ``libotfuse.so`` (raises if it has not been built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise OtfError(
                f"otfuse HIP library not found at {LIB_PATH}; build it with "
                "`python -c 'import __graft_entry__ as g; g.build()'` (hipcc, gfx950)")
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def declared_symbols():
    """Entry points declared in include/otfuse.h (used by the ABI tests)."""
    src = open(HEADER_PATH).read()
    return sorted(set(re.findall(r"\b(otf_[a-z0-9_]+)\s*\(", src)))


def check(rc: int, what: str):
    if rc != OTF_OK:
        kind = {OTF_EINVAL: "invalid argument", OTF_EUNSUPPORTED: "unsupported shape/config",
                OTF_EHIP: "HIP runtime error"}.get(rc, f"error {rc}")
        raise OtfError(f"{what}: {kind} (rc={rc})")


def ptr(t) -> int | None:
    return None if t is None else t.data_ptr()


def stream_handle(device=None) -> int:
    return torch.cuda.current_stream(device).cuda_stream
