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
    def forward(ctx, logits, target, ignore_index, smoothing, reduction):
        logits = logits.contiguous()
        target = target.contiguous()
        if target.is_floating_point():
            target = target.float()
        loss_rows, lse = C().ce_fwd(logits, target, ignore_index, smoothing)
        if target.is_floating_point():
            count = torch.full((), float(logits.shape[0]), device=logits.device)
        else:
            count = (target != ignore_index).sum().float()
        ctx.save_for_backward(logits, target, lse, count)
        ctx.cfg = (ignore_index, smoothing, reduction)
        if reduction == "mean":
            return loss_rows.sum() / count
        if reduction == "sum":
            return loss_rows.sum()
        return loss_rows

    @staticmethod
    def backward(ctx, g):
        logits, target, lse, count = ctx.saved_tensors
        ignore_index, smoothing, reduction = ctx.cfg
        if reduction == "none":
            raise NotImplementedError("per-row cross-entropy backward: use reduction='mean' or 'sum'")
        scale = g.float() / count if reduction == "mean" else g.float()
        d = C().ce_bwd(logits, target, lse, scale.reshape(1).contiguous(), 1.0, ignore_index, smoothing)
        return d, None, None, None, None


def cross_entropy(logits, target, ignore_index: int = -100, label_smoothing: float = 0.0, reduction: str = "mean"):
    if logits.is_cuda and logits.dim() == 2:
        return _CrossEntropyFn.apply(logits, target, ignore_index, label_smoothing, reduction)
    return F.cross_entropy(logits.float(), target.float() if target.is_floating_point() else target,
                           ignore_index=ignore_index, label_smoothing=label_smoothing, reduction=reduction)
