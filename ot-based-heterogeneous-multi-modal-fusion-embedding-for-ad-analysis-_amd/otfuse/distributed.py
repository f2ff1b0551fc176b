"""Multi-GPU pieces of the path: one process per GPU, torch.distributed over RCCL.

The reference has no distributed code; these are the two exchanges
the path actually needs:

* ``all_gather_rows`` — the per-epoch global OT (MRI_PET_OT_OT_per_epoch_attn.py:940-960)
  extracts features per data-parallel shard; one all-gather gives every rank the
  full (N x d) embedding set and labels before the solve.
* ``sharded_feature_cost`` — for a sample coupling Ts that is block-diagonal along
  the shards (Ts = I/B per batch, MRI_PET_OT_nojax.py:688), the feature cost
  decomposes as M = sum_r (t1_r + t2_r - 2 X_r^T Ts_r Y_r): ONE all-reduce(SUM)
  of the d x d2 float64 partials (1 MiB at d = 512... 32 MiB at d = 2048) replaces
  gathering the embeddings.  The Sinkhorn solve is then replicated (it is tiny).

Independent problems (per-rank minibatches / labels) need no collective at all;
bench.py scales that way ("weak", replicas).
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from . import ops


def all_gather_rows(local: torch.Tensor, group=None) -> torch.Tensor:
    """Concatenate every rank's (n_r, ...) tensor along dim 0 in rank order.
    Unequal n_r are padded to the max for the collective and trimmed after."""
    world = dist.get_world_size(group)
    if world == 1:
        return local
    n = torch.tensor([local.shape[0]], dtype=torch.int64, device=local.device)
    sizes = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(sizes, n, group=group)
    sizes = [int(s.item()) for s in sizes]
    nmax = max(sizes)
    pad = local.new_zeros((nmax,) + tuple(local.shape[1:]))
    pad[: local.shape[0]] = local
    out = local.new_empty((world * nmax,) + tuple(local.shape[1:]))
    dist.all_gather_into_tensor(out, pad.contiguous(), group=group)
    return torch.cat([out[r * nmax: r * nmax + sizes[r]] for r in range(world)])


def _local_feature_cost(X, Y, Ts=None, ts_diag=None, weights="pot"):
    return ops.feature_cost(X, Y, Ts=Ts, ts_diag=ts_diag, weights=weights)


def sharded_feature_cost(X_local: torch.Tensor, Y_local: torch.Tensor, Ts_local=None,
                         ts_diag_local=None, weights: str = "pot", group=None) -> torch.Tensor:
    """Global feature cost from per-rank shards with block-diagonal Ts (one all-reduce)."""
    M = _local_feature_cost(X_local, Y_local, Ts=Ts_local, ts_diag=ts_diag_local, weights=weights)
    if dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(M, op=dist.ReduceOp.SUM, group=group)
    return M


def sharded_batch_feature_plan(mri_local: torch.Tensor, pet_local: torch.Tensor, global_batch: int,
                               eps: float = 1e-2, numItermax: int = 2000, stopThr: float = 1e-9,
                               group=None):
    """Per-batch PET->MRI feature plan of a data-parallel batch sharded over ranks:
    Ts = I / B_global restricted to the local rows, one all-reduce, replicated solve."""
    B = mri_local.shape[0]
    ts = torch.full((B,), 1.0 / global_batch, dtype=torch.float64, device=mri_local.device)
    M = sharded_feature_cost(mri_local.detach(), pet_local.detach(), ts_diag_local=ts, group=group)
    d, d2 = M.shape
    a = torch.full((d,), 1.0 / d, dtype=torch.float64, device=M.device)
    b = torch.full((d2,), 1.0 / d2, dtype=torch.float64, device=M.device)
    res = ops.sinkhorn(a, b, M, float(eps), max_iter=numItermax, stop_thr=stopThr, flavor="pot",
                       sync_every=50, want_plan=True)
    return res.plan, res


def gather_epoch_features(mri_local: torch.Tensor, pet_local: torch.Tensor,
                          labels_local: torch.Tensor, group=None):
    """All-gather the per-shard backbone features and labels of one epoch
    (feature_extract, MRI_PET_OT_OT_per_epoch_attn.py:889-912, run data-parallel)."""
    return (all_gather_rows(mri_local, group), all_gather_rows(pet_local, group),
            all_gather_rows(labels_local, group))
