"""Model-level seam: the OT block of ``MultimodalMRI_PET_OT.forward`` on the device.

The reference (MRI_PET_OT_nojax.py:679-725) copies ``mri_fused`` / ``pet_fused`` to
the host, runs POT in float64, copies the plan back and post-processes it in
torch.  Here the whole block stays on the device and in HIP kernels:

    feature cost (float64, Ts = I/B; float32 / bf16 / fp16 embeddings read as
    stored)  ->  POT-flavour Sinkhorn (float64, eps 1e-2, 2000 iterations, stopThr
    1e-9, one persistent launch, no host sync)  ->  ONE fused kernel: NaN -> 1e-8 + row
    normalisation (float32) and ot_mri_from_pet = pet_fused @ T^T (autograd: G @ T)
    ->  cosine loss, zeroed with its gradients when non-finite (the reference's
    NaN -> 0 at :724-725 replaces the loss by a constant) or when the solve reported a
    stalled device barrier (decided on the device: no host sync).

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
                       numItermax: int = 2000, stopThr: float = 1e-9, sync_every: int = 0):
    """PET->MRI feature coupling of one batch, Ts = eye(B)/B (MRI_PET_OT_nojax.py:683-699).
    Returns the raw float64 plan (d, d) and the SinkhornResult."""
    B = mri_fused.shape[0]
    ts_diag = ops.uniform(B, torch.float64, mri_fused.device)   # Ts = eye(B) / B
    res = feature_coupling_pot_device(mri_fused.detach(), pet_fused.detach(), ts_diag=ts_diag,
                                      eps=eps, numItermax=numItermax, stopThr=stopThr,
                                      sync_every=sync_every)
    return res.plan, res


class _OTAlignLoss(torch.autograd.Function):
    """ot_mri_from_pet = pet_fused @ Tn^T and cosine_loss(mri_fused, ot_mri_from_pet) as
    one autograd node (MRI_PET_OT_nojax.py:702-725), three HIP launches per training
    step: ``raw=True`` fuses the plan post-processing into the apply
    (otf_plan_postprocess_apply, one pass; else T is applied as given), the loss and
    both its gradients come from ONE workgroup (otf_cosine_align), and the backward is
    ONE launch (otf_ot_align_backward: G @ Tn and the loss scaling).  A non-finite loss
    -- or a solve that did not finish (its info words, read by the loss kernel) -- becomes a constant 0
    that sends no gradient to mri_fused / pet_fused, like the reference's swap for
    torch.tensor(0.0) at :724-725; the zeroing is a select in the kernels, never
    0 * NaN, and needs no host sync."""

    @staticmethod
    def forward(ctx, mri, pet, T, info, raw):
        ctx.set_materialize_grads(False)   # an unused ot_mri_from_pet sends None, not zeros
        if raw:
            ot, Tn = ops.plan_postprocess_apply(T, pet)
        else:
            Tn = T.float().contiguous()
            ot = ops.gemm_f32(pet.float(), Tn, transpose_b=True)
        loss, gx, gy, keep = ops.cosine_align(mri.detach(), ot, sk_info=info)
        ctx.save_for_backward(gx, gy, Tn, keep)
        ctx.dtypes = (mri.dtype, pet.dtype)
        ctx.mark_non_differentiable(Tn)
        return loss, ot, Tn

    @staticmethod
    def backward(ctx, g_loss, g_ot, _g_tn):
        gx, gy, Tn, keep = ctx.saved_tensors
        g_mri, gpet = ops.ot_align_backward(gx, gy, Tn, g_loss=g_loss, g_ot=g_ot, keep=keep)
        return g_mri.to(ctx.dtypes[0]), gpet.to(ctx.dtypes[1]), None, None, None


def ot_alignment_loss(mri_fused: torch.Tensor, pet_fused: torch.Tensor,
                      T_feature_pet2mri: torch.Tensor | None = None, eps: float = 1e-2,
                      numItermax: int = 2000, stopThr: float = 1e-9):
    """The training-time OT block of forward (MRI_PET_OT_nojax.py:679-725).

    Returns ``(ot_loss, ot_mri_from_pet, T)``; T is the post-processed float32 plan.
    A provided ``T_feature_pet2mri`` is applied as is (the reference skips the
    post-processing for a given plan).  A NaN loss becomes 0 (and contributes no
    gradient) without a host sync; so does the loss of a solve whose device barrier
    stalled (status timeout), instead of training on an invalid plan.
    """
    if T_feature_pet2mri is None:
        plan, res = batch_feature_plan(mri_fused, pet_fused, eps, numItermax, stopThr)
        # the loss kernel checks that the solve finished (final status written, not
        # running / timeout, stop set, no stalled workgroup) from the info words itself
        ot_loss, ot_mri_from_pet, T = _OTAlignLoss.apply(mri_fused, pet_fused, plan, res.info_dev, True)
    else:
        ot_loss, ot_mri_from_pet, T = _OTAlignLoss.apply(mri_fused, pet_fused, T_feature_pet2mri,
                                                         None, False)
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
