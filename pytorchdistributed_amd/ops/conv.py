"""2-D convolution, channels-last (reference: torchvision ResNet-50 convs
`03 模型并行/03_model_parallel.ipynb` raw lines 314, 325-349, reached through cuDNN).

GPU: implicit-GEMM MFMA kernels (`csrc/kernels/gemm_conv.hip`) for forward, data-gradient (the
stride is folded into the gather, weights transposed to [C_in, R, S, C_out] on the fly) and
weight-gradient (split-K over N*P*Q with a deterministic slab reduction).
"""
from __future__ import annotations

import os

import torch
import torch.nn.functional as F

from .._native import C
from ..parallel.flat import grad_target
from . import streams as _streams
from .grad_join import MaskedGrad


# PDA_WGRAD_SIDE_1X1=0: 1x1 weight gradients (HBM-bound like the BN kernels they would overlap) stay on
# the compute stream; only the MFMA-bound 3x3 / 7x7 ones go to the side stream (A/B knob)
_SIDE_1X1 = os.environ.get("PDA_WGRAD_SIDE_1X1", "1") == "1"


def _ref_conv(x, w, stride, padding, dilation, bias=None):
    y = F.conv2d(x.permute(0, 3, 1, 2), w.permute(0, 3, 1, 2), bias, stride, padding, dilation)
    return y.permute(0, 2, 3, 1).contiguous()


class _Conv2dFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, bias, stride, padding, dilation, relu, join, bnb=None):
        x = x.contiguous()
        w = w.contiguous()
        y = C().conv_fwd(x, w, stride, padding, dilation, bias, relu)
        ctx.save_for_backward(x, w, y if relu else None)
        ctx.cfg = (stride, padding, dilation, relu, bias is not None)
        ctx.wparam = w
        ctx.join = join
        ctx.bnb = bnb
        return y

    @staticmethod
    def backward(ctx, dy):
        return _Conv2dFn._backward(ctx, dy)

    @staticmethod
    def _backward(ctx, dy):
        x, w, y = ctx.saved_tensors
        stride, padding, dilation, relu, has_bias = ctx.cfg
        dy = dy.contiguous()
        if relu:
            dy = C().relu_bwd(dy, y)
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            join = ctx.join
            if join is not None and not join.is_last():
                join.stash(C().conv_dgrad(dy, w, x.shape[1], x.shape[2], stride, padding, dilation, None))
            else:
                # the BN that produced x: its backward sums come out of this dgrad's epilogue (its dy = dx);
                # with a join, only as its last contributor (checked before take() resets the join)
                bnb = getattr(ctx, "bnb", None)
                join_last = join is not None and join.is_last()
                addend = join.take() if join is not None else None
                bits = None
                if isinstance(addend, MaskedGrad):  # residual gradient = dz * ReLU mask, applied in the epilogue
                    addend, bits = addend.grad, addend.bits
                kw = {}
                if bnb is not None and bnb.usable(join_last, join is not None, stride, addend) and \
                        bnb.z.shape == x.shape:
                    kw = bnb.dgrad_kwargs()
                dx = C().conv_dgrad(dy, w, x.shape[1], x.shape[2], stride, padding, dilation, addend, bits, **kw)
                if kw:
                    bnb.mark_filled(dx)
        ctx.bnb = None
        if ctx.needs_input_grad[1]:
            target = grad_target(ctx.wparam)
            args = (dy, x, w.shape[1], w.shape[2], stride, padding, dilation, w.dtype == torch.float32, target)
            # Off the critical path: the wgrad overlaps the BN backward / dgrad of the layers below it.
            # Only when the kernel writes the parameter's final gradient storage (a flat-buffer slot that
            # AccumulateGrad adopts without a kernel); a freshly allocated dw would be read on the main
            # stream by AccumulateGrad's accumulate / clone, which knows nothing of the side stream.
            if target is not None and _streams.side_ok(ctx.wparam) and (_SIDE_1X1 or w.shape[1] * w.shape[2] > 1):
                with _streams.wgrad_stream(dy.device, dy, x):
                    dw = C().conv_wgrad(*args)
            else:
                dw = C().conv_wgrad(*args)
        if has_bias and ctx.needs_input_grad[2]:
            db = dy.reshape(-1, dy.shape[-1]).sum(0, dtype=torch.float32).to(dy.dtype)
        return dx, dw, db, None, None, None, None, None, None


class _Conv2dStatsFn(torch.autograd.Function):
    """Conv forward whose GEMM epilogue also accumulates the BatchNorm sums of its output
    (sum(y - K), sum((y - K)^2) per channel, K = ``shift``) into a zeroed [R, 2, C_out] table (tile t
    adds into row t % R), so the following BatchNorm skips its statistics pass over y.  Backward is
    the plain conv backward."""

    @staticmethod
    def forward(ctx, x, w, stride, padding, dilation, shift, table, join, bnb=None):
        x = x.contiguous()
        w = w.contiguous()
        y = C().conv_fwd_stats(x, w, stride, padding, dilation, shift, table)
        ctx.save_for_backward(x, w, None)
        ctx.cfg = (stride, padding, dilation, False, False)
        ctx.wparam = w
        ctx.join = join
        ctx.bnb = bnb
        return y

    @staticmethod
    def backward(ctx, dy):
        dx, dw, _db, *_ = _Conv2dFn._backward(ctx, dy)
        return dx, dw, None, None, None, None, None, None, None


def conv2d_bn_stats(x: torch.Tensor, weight: torch.Tensor, stride: int = 1, padding: int = 0, dilation: int = 1,
                    shift: torch.Tensor = None, table: torch.Tensor = None, grad_join=None):
    """GPU only: returns y and adds ``(sum(y - shift), sum((y - shift)^2))`` per channel into the rows of
    ``table`` ([R, 2, C_out] fp32, zero on entry; the consuming BN finalize re-zeroes it)."""
    if weight.shape[-1] != x.shape[-1]:
        weight = F.pad(weight, (0, x.shape[-1] - weight.shape[-1]))
    return _Conv2dStatsFn.apply(x, weight, stride, padding, dilation, shift, table, grad_join,
                                getattr(x, "_pda_bnb", None))


def conv2d(x: torch.Tensor, weight: torch.Tensor, bias=None, stride: int = 1, padding: int = 0, dilation: int = 1,
           relu: bool = False, grad_join=None) -> torch.Tensor:
    """``y[N,P,Q,Co] = conv(x[N,H,W,Ci], weight[Co,R,S,Ci])`` (+bias, optional fused ReLU).
    ``grad_join`` (:class:`~.grad_join.GradJoin`): x's gradient from other consumers is added inside
    the dgrad kernel's store when this conv is the last of them to run backward."""
    if x.is_cuda:
        if weight.shape[-1] != x.shape[-1]:  # stem: input channels padded to a multiple of 8
            weight = F.pad(weight, (0, x.shape[-1] - weight.shape[-1]))
        if x.dtype == torch.float32:  # split-bf16 operands on the same MFMA kernels (ops/fp32.py)
            from . import fp32

            return fp32.conv2d(x, weight, bias, stride, padding, dilation, relu)
        return _Conv2dFn.apply(x, weight, bias, stride, padding, dilation, relu, grad_join,
                               getattr(x, "_pda_bnb", None))
    if weight.shape[-1] != x.shape[-1]:
        x = x[..., : weight.shape[-1]]
    y = _ref_conv(x, weight, stride, padding, dilation, bias)
    return torch.relu(y) if relu else y
