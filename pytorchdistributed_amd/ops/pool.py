"""Pooling over channels-last activations (SURVEY §2.5 K06 MaxPool2d(3,2,1), K07 AdaptiveAvgPool2d(1);
reference `03_model_parallel.ipynb` raw lines 333 and 341)."""
from __future__ import annotations

import os

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


_FUSED_BWD = os.environ.get("PDA_STEM_POOL_BN_BWD", "1") == "1"


class _BnReluMaxPoolFn(torch.autograd.Function):
    """``max_pool2d(relu(batch_norm(z)))`` for the ResNet stem, the BN finalized from the stem conv's
    epilogue statistics table: the pool applies BN + ReLU to each window element as it loads it, so the
    BN output (the largest activation of the network) is never stored.  Backward: the pool's gather
    backward, then the BN+ReLU backward with the mask recomputed from z and the saved scale / shift."""

    @staticmethod
    def forward(ctx, z, gamma, beta, running_mean, running_var, table, shift, nbt, momentum, eps, k, s, p):
        z = z.contiguous()
        y, idx, mean, invstd, ss = C().bn_relu_maxpool_fwd(z, table, shift, gamma, beta, running_mean, running_var,
                                                             nbt, momentum, eps, k, s, p)
        ctx.save_for_backward(z, idx, mean, invstd, ss, gamma)
        ctx.beta = beta
        ctx.cfg = (z.shape[1], z.shape[2], k, s, p)
        return y

    @staticmethod
    def backward(ctx, dy):
        from ..parallel.flat import grad_target

        z, idx, mean, invstd, ss, gamma = ctx.saved_tensors
        H, W, k, s, p = ctx.cfg
        beta = ctx.beta
        ng = ctx.needs_input_grad
        tg = grad_target(gamma) if gamma is not None and ng[1] else None
        tb = grad_target(beta) if beta is not None and ng[2] else None
        if (tg is None) != (tb is None):
            tg = tb = None
        if _FUSED_BWD and C().stem_pool_bn_bwd_ok(H, W, z.shape[-1], k, s, p):
            # pool gradient gathered in registers by both BN-backward passes (never stored)
            dz, dg, db = C().stem_pool_bn_bwd(dy.contiguous(), idx, z, ss, mean, invstd, gamma, tg, tb)
        else:
            da = C().maxpool_bwd(dy.contiguous(), idx, H, W, k, s, p)
            dz, _, dg, db = C().bn_bwd(da, z, None, ss, mean, invstd, gamma, True, False, tg, tb)
        return (dz, dg if gamma is not None and ng[1] else None, db if beta is not None and ng[2] else None) \
            + (None,) * 10


def bn_relu_max_pool2d(z, bn, stats, kernel_size=3, stride=2, padding=1):
    """GPU training path of ``max_pool2d(relu(bn(z)))``; ``stats = (table, shift)`` from
    ``Conv2d(..., bn=bn)``."""
    table, shift = stats
    return _BnReluMaxPoolFn.apply(z, bn.weight, bn.bias, bn.running_mean, bn.running_var, table, shift,
                                  bn.num_batches_tracked, bn.momentum, bn.eps, kernel_size, stride, padding)


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
    if x.is_cuda and x.dtype == torch.float32 and x.shape[-1] % 4 == 0:
        from .fp32 import MaxPoolF32Fn

        return MaxPoolF32Fn.apply(x, kernel_size, stride, padding)
    y = F.max_pool2d(x.permute(0, 3, 1, 2), kernel_size, stride, padding)
    return y.permute(0, 2, 3, 1).contiguous()


def global_avg_pool2d(x, out_fp32=False):
    """``[N,H,W,C] -> [N,C]`` spatial mean."""
    if x.is_cuda and x.dtype == torch.bfloat16:
        return _AvgPoolFn.apply(x, out_fp32)
    if x.is_cuda and x.dtype == torch.float32:
        from .fp32 import AvgPoolF32Fn

        return AvgPoolF32Fn.apply(x)
    y = x.float().mean(dim=(1, 2))
    return y if out_fp32 else y.to(x.dtype)
