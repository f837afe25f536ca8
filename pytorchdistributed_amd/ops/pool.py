"""Pooling over channels-last activations (SURVEY §2.5 K06 MaxPool2d(3,2,1), K07 AdaptiveAvgPool2d(1);
reference `03_model_parallel.ipynb` raw lines 333 and 341)."""
from __future__ import annotations

import torch
import torch.nn.functional as F

from .._native import C


class _MaxPoolFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, k, s, p):
        y, idx = C().maxpool_fwd(x.contiguous(), k, s, p)
        ctx.save_for_backward(idx)
        ctx.cfg = (x.shape[1], x.shape[2], k, s, p)
        return y

    @staticmethod
    def backward(ctx, dy):
        (idx,) = ctx.saved_tensors
        H, W, k, s, p = ctx.cfg
        return C().maxpool_bwd(dy.contiguous(), idx, H, W, k, s, p), None, None, None


class _AvgPoolFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, out_fp32):
        ctx.hw = (x.shape[1], x.shape[2])
        return C().avgpool_fwd(x.contiguous(), not out_fp32)

    @staticmethod
    def backward(ctx, dy):
        return C().avgpool_bwd(dy.contiguous(), *ctx.hw), None


def max_pool2d(x, kernel_size=3, stride=2, padding=1):
    if x.is_cuda and x.dtype == torch.bfloat16:
        return _MaxPoolFn.apply(x, kernel_size, stride, padding)
    y = F.max_pool2d(x.permute(0, 3, 1, 2), kernel_size, stride, padding)
    return y.permute(0, 2, 3, 1).contiguous()


def global_avg_pool2d(x, out_fp32=False):
    """``[N,H,W,C] -> [N,C]`` spatial mean."""
    if x.is_cuda and x.dtype == torch.bfloat16:
        return _AvgPoolFn.apply(x, out_fp32)
    y = x.float().mean(dim=(1, 2))
    return y if out_fp32 else y.to(x.dtype)
