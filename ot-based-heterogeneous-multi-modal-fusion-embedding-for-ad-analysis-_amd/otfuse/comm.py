"""RCCL communicator over the C ABI (``otf_comm_*`` in include/otfuse.h).

One process per GPU.  Rank 0 draws the 128-byte RCCL unique id, torch.distributed
broadcasts it (any backend), every rank joins.  The collectives are enqueued on the
current torch stream of the tensor's device, like every other op of this package, so
a whole row-sharded Sinkhorn solve (``otf_sinkhorn_row_sharded``) runs its per-
iteration all-reduces without returning to Python.  The reference has no collective
(SURVEY.md §5); these carry the exchanges of SURVEY.md §8e.
"""
from __future__ import annotations

import ctypes

import torch
import torch.distributed as dist

from . import _lib as L
from . import ops

# element types the RCCL collectives take (bf16: the config-4 encoder outputs)
_COMM_DT = {torch.float32: L.OTF_F32, torch.float64: L.OTF_F64, torch.float16: L.OTF_F16,
            torch.bfloat16: L.OTF_BF16}


class Communicator:
    """An RCCL communicator of ``nranks`` processes (``group``'s ranks, or one rank)."""

    def __init__(self, group=None, device=None):
        if dist.is_available() and dist.is_initialized():
            self.rank = dist.get_rank(group)
            self.nranks = dist.get_world_size(group)
        else:
            self.rank, self.nranks = 0, 1
        self.device = torch.device("cuda", torch.cuda.current_device()) if device is None else device
        lib = L.lib()
        uid = (ctypes.c_uint8 * L.COMM_ID_BYTES)()
        if self.rank == 0:
            L.check(lib.otf_comm_unique_id(ctypes.cast(uid, ctypes.c_void_p)), "otf_comm_unique_id")
        if self.nranks > 1:
            on_dev = dist.get_backend(group) == "nccl"
            t = torch.tensor(list(bytes(uid)), dtype=torch.uint8,
                             device=self.device if on_dev else "cpu")
            src = dist.get_global_rank(group, 0) if group is not None else 0
            dist.broadcast(t, src=src, group=group)
            uid = (ctypes.c_uint8 * L.COMM_ID_BYTES)(*t.cpu().tolist())
        h = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            L.check(lib.otf_comm_init(ctypes.byref(h), ctypes.cast(uid, ctypes.c_void_p),
                                      self.nranks, self.rank), "otf_comm_init")
        self.handle = h

    def close(self):
        if self.handle is not None and self.handle.value:
            L.check(L.lib().otf_comm_destroy(self.handle), "otf_comm_destroy")
        self.handle = None

    def all_reduce(self, t: torch.Tensor, op: str = "sum") -> torch.Tensor:
        """In place; float32 / float64 / float16 / bfloat16, contiguous."""
        ops._dev(t, "t")
        if not t.is_contiguous() or t.dtype not in _COMM_DT:
            raise TypeError("all_reduce: contiguous float16/bfloat16/32/64 tensors only")
        red = {"sum": L.OTF_RED_SUM, "max": L.OTF_RED_MAX}[op]
        L.check(L.lib().otf_comm_all_reduce(t.data_ptr(), t.numel(), _COMM_DT[t.dtype], red, self.handle,
                                            L.stream_handle(t.device)), "otf_comm_all_reduce")
        return t

    def all_gather(self, t: torch.Tensor) -> torch.Tensor:
        """Concatenation of every rank's equally-shaped ``t`` along dim 0, rank order."""
        ops._dev(t, "t")
        t = t.contiguous()
        if t.dtype not in _COMM_DT:
            raise TypeError("all_gather: float16/bfloat16/32/64 tensors only")
        out = torch.empty((self.nranks * t.shape[0],) + tuple(t.shape[1:]), dtype=t.dtype,
                          device=t.device)
        L.check(L.lib().otf_comm_all_gather(t.data_ptr(), out.data_ptr(), t.numel(), _COMM_DT[t.dtype],
                                            self.handle, L.stream_handle(t.device)),
                "otf_comm_all_gather")
        return out

    def all_gather_rows(self, t: torch.Tensor) -> tuple[torch.Tensor, list[int]]:
        """Concatenation of every rank's (n_r, ...) ``t`` along dim 0 in rank order when
        the n_r differ: the row counts are exchanged first (one tiny all-gather and one
        host read), the shards padded to the largest for the collective and trimmed
        after.  Returns (rows, [n_0, ..., n_{R-1}])."""
        ops._dev(t, "t")
        n = torch.tensor([float(t.shape[0])], dtype=torch.float64, device=t.device)
        sizes = [int(x) for x in self.all_gather(n).cpu().tolist()]
        nmax = max(sizes)
        if all(s == nmax for s in sizes):
            return self.all_gather(t), sizes
        pad = t.new_zeros((nmax,) + tuple(t.shape[1:]))
        pad[: t.shape[0]] = t
        out = self.all_gather(pad)
        return torch.cat([out[r * nmax: r * nmax + sizes[r]] for r in range(self.nranks)]), sizes
