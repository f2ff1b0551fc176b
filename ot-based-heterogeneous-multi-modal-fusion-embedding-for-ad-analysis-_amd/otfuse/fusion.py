"""Model-level seam: the OT block of ``MultimodalMRI_PET_OT.forward`` on the device.

The reference (MRI_PET_OT_nojax.py:679-725) copies ``mri_fused`` / ``pet_fused`` to
the host, runs POT in float64, copies the plan back and post-processes it in
torch.  Here the whole block stays on the device and in HIP kernels:

    feature cost (float64, Ts = I/B)  ->  POT-flavour Sinkhorn (float64, eps 1e-2,
    2000 iterations, stopThr 1e-9)  ->  NaN -> 1e-8 + row normalisation (float32)
    ->  ot_mri_from_pet = pet_fused @ T^T (HIP GEMM, autograd)  ->  cosine loss.

``group_features_by_label`` mirrors MRI_PET_OT_nojax.py:884-903 for the per-epoch path.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F

from . import ops
from .pot import feature_coupling_pot_device


def cosine_loss(x, y):
    """1 - mean cosine similarity (MRI_PET_OT_nojax.py:552-560)."""
    if x.dim() == 1:
        x = x.unsqueeze(0)
    if y.dim() == 1:
        y = y.unsqueeze(0)
    x = F.normalize(x, p=2, dim=1)
    y = F.normalize(y, p=2, dim=1)
    return 1 - F.cosine_similarity(x, y).mean()


def batch_feature_plan(mri_fused: torch.Tensor, pet_fused: torch.Tensor, eps: float = 1e-2,
                       numItermax: int = 2000, stopThr: float = 1e-9, sync_every: int = 50):
    """PET->MRI feature coupling of one batch, Ts = eye(B)/B (MRI_PET_OT_nojax.py:683-699).
    Returns the raw float64 plan (d, d) and the SinkhornResult."""
    B = mri_fused.shape[0]
    ts_diag = torch.full((B,), 1.0 / B, dtype=torch.float64, device=mri_fused.device)
    res = feature_coupling_pot_device(mri_fused.detach(), pet_fused.detach(), ts_diag=ts_diag,
                                      eps=eps, numItermax=numItermax, stopThr=stopThr,
                                      sync_every=sync_every)
    return res.plan, res


def ot_alignment_loss(mri_fused: torch.Tensor, pet_fused: torch.Tensor,
                      T_feature_pet2mri: torch.Tensor | None = None, eps: float = 1e-2,
                      numItermax: int = 2000, stopThr: float = 1e-9):
    """The training-time OT block of forward (MRI_PET_OT_nojax.py:679-725).

    Returns ``(ot_loss, ot_mri_from_pet, T)``; T is the post-processed float32 plan.
    A provided ``T_feature_pet2mri`` is applied as is (the reference skips the
    post-processing for a given plan).  A NaN loss becomes 0 without a host sync.
    """
    if T_feature_pet2mri is None:
        plan, _ = batch_feature_plan(mri_fused, pet_fused, eps, numItermax, stopThr)
        T = ops.plan_postprocess(plan, nan_fill=1e-8, rownorm=True)
    else:
        T = T_feature_pet2mri.float()
    ot_mri_from_pet = ops.apply_plan(pet_fused, T)
    ot_loss = cosine_loss(mri_fused, ot_mri_from_pet)
    ot_loss = torch.nan_to_num(ot_loss, nan=0.0)
    return ot_loss, ot_mri_from_pet, T


def group_features_by_label(y, p, max_samples_per_label=None):
    """Group features by label, first ``max_samples_per_label`` rows per label
    (MRI_PET_OT_nojax.py:884-903; MRI_PET_OT_OT_per_epoch_attn.py:915-937)."""
    unique_labels = np.unique(y)
    grouped = {int(label): [] for label in unique_labels}
    for label, features in zip(y, p):
        grouped[int(label)].append(features)
    for label in grouped:
        if grouped[label]:
            arr = np.stack(grouped[label])
            if (max_samples_per_label is not None and max_samples_per_label > 0
                    and arr.shape[0] > max_samples_per_label):
                arr = arr[:max_samples_per_label]
            grouped[label] = arr
    return grouped
