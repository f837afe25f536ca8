"""Cross-entropy.

Supports class-index targets (BASELINE configs) and probability targets — the path the reference
actually exercises: `F.cross_entropy(output, ys)` with float ys (`ddp_gpus.py:40,60`) and
`nn.CrossEntropyLoss()(outputs, one_hot)` (`03_model_parallel.ipynb` raw lines 382, 389).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from .._native import C


class _CrossEntropyFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, target, ignore_index, smoothing, reduction, num_valid):
        logits = logits.contiguous()
        target = target.contiguous()
        if target.is_floating_point():
            target = target.float()
        loss_rows, lse = C().ce_fwd(logits, target, ignore_index, smoothing, num_valid)
        if target.is_floating_point():
            count = torch.full((), float(logits.shape[0]), device=logits.device)
        else:
            count = (target != ignore_index).sum().float()
        ctx.save_for_backward(logits, target, lse, count)
        ctx.cfg = (ignore_index, smoothing, reduction, num_valid)
        if reduction == "mean":
            return loss_rows.sum() / count
        if reduction == "sum":
            return loss_rows.sum()
        return loss_rows

    @staticmethod
    def backward(ctx, g):
        logits, target, lse, count = ctx.saved_tensors
        ignore_index, smoothing, reduction, num_valid = ctx.cfg
        if reduction == "none":
            raise NotImplementedError("per-row cross-entropy backward: use reduction='mean' or 'sum'")
        scale = g.float() / count if reduction == "mean" else g.float()
        d = C().ce_bwd(logits, target, lse, scale.reshape(1).contiguous(), 1.0, ignore_index, smoothing, num_valid)
        return d, None, None, None, None, None


def cross_entropy(logits, target, ignore_index: int = -100, label_smoothing: float = 0.0, reduction: str = "mean",
                  num_valid_classes: int = 0):
    """``num_valid_classes``: logits beyond this column are padding (vocab padded to a multiple of 64 for
    the GEMMs) — excluded from the softmax and given zero gradient, so the loss equals the unpadded one."""
    if logits.dim() > 2:
        logits = logits.reshape(-1, logits.shape[-1])
        target = target.reshape(-1) if not target.is_floating_point() else target.reshape(-1, logits.shape[-1])
    if logits.is_cuda and logits.dim() == 2:
        return _CrossEntropyFn.apply(logits, target, ignore_index, label_smoothing, reduction, num_valid_classes)
    if num_valid_classes and num_valid_classes < logits.shape[-1]:
        logits = logits[:, :num_valid_classes]
    return F.cross_entropy(logits.float(), target.float() if target.is_floating_point() else target,
                           ignore_index=ignore_index, label_smoothing=label_smoothing, reduction=reduction)
