"""fp32 training path: the reference's own ResNet-50 workloads at their precision.

The reference trains in fp32 (`03 模型并行/03_model_parallel.ipynb` raw lines 369-391; models at 314 and
417), its convs running TF32 on cuDNN.  gfx950 has no xf32 MFMA and its f32-input MFMA is 1/16 of the
bf16 rate, so conv GEMMs here run on the bf16 MFMA kernels with split operands (`csrc/kernels/fp32x3.hip`):
``x = hi + lo`` (two bf16), ``x.w ~ hi.hi + hi.lo + lo.hi`` accumulated in fp32 — the three products
laid side by side along the GEMM's K, so one launch of the ordinary conv kernel computes them
(``PDA_FP32_SPLIT=4`` adds ``lo.lo``).  ``hi + lo`` carries 16 significant bits of x, so every
product is good to ~2^-17 relative (~1e-5 per GEMM; TF32, the reference's A100 conv precision, keeps
11 bits: ~5e-4) — whole-model gradients land >5x closer to an fp64 oracle than TF32 convs
(tests/test_fp32_gpu.py).  BatchNorm, pooling and
the ReLU / residual epilogues are native fp32 kernels; the Linear layer keeps the exact fp32 SIMT
GEMM (`ops/linear.py`) and cross-entropy reads fp32 logits natively.
"""
from __future__ import annotations

import os

import torch

from .._native import C
from ..parallel.flat import grad_target

# segment s of an operand is its lo part when bit s is set: A = (hi, hi, lo[, lo]), B = (hi, lo, hi[, lo])
_MASKS = {3: (0b100, 0b010), 4: (0b1100, 0b1010)}
NSEG = 3
MASK_A, MASK_B = _MASKS[3]


def set_split(n: int) -> None:
    """Number of split products per fp32 GEMM: 3 (hi.hi + hi.lo + lo.hi) or 4 (+ lo.lo); both are bound
    by the 16-bit hi + lo representation of the operands (~1e-5 relative)."""
    global NSEG, MASK_A, MASK_B
    if n not in _MASKS:
        raise ValueError("the fp32 split must be 3 or 4")
    NSEG = n
    MASK_A, MASK_B = _MASKS[n]


set_split(int(os.environ.get("PDA_FP32_SPLIT", "3")))


def _split(t: torch.Tensor, mask: int, stack: bool) -> torch.Tensor:
    return C().split_bf16(t.contiguous(), NSEG, mask, stack)


class Conv2dF32Fn(torch.autograd.Function):
    """fp32 conv (NHWC x, OHWI w) through split-bf16 operands on the MFMA implicit-GEMM kernels:
    fwd splits along the input channels, dgrad along the output channels (w stacked on C_out), wgrad
    along the batch (dy and x stacked on N)."""

    @staticmethod
    def forward(ctx, x, w, bias, stride, padding, dilation, relu):
        x = x.contiguous()
        w = w.contiguous()
        y = C().conv_fwd(_split(x, MASK_A, False), _split(w, MASK_B, False), stride, padding, dilation, bias, relu,
                         out_f32=True)
        ctx.save_for_backward(x, w, y if relu else None)
        ctx.cfg = (stride, padding, dilation, relu, bias is not None)
        ctx.wparam = w
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w, y = ctx.saved_tensors
        stride, padding, dilation, relu, has_bias = ctx.cfg
        dy = dy.contiguous()
        if relu:
            dy = C().relu_bwd(dy, y)
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = C().conv_dgrad(_split(dy, MASK_A, False), _split(w, MASK_B, True), x.shape[1], x.shape[2], stride,
                                padding, dilation, out_f32=True)
        if ctx.needs_input_grad[1]:
            target = grad_target(ctx.wparam)
            dw = C().conv_wgrad(_split(dy, MASK_B, True), _split(x, MASK_A, True), w.shape[1], w.shape[2], stride,
                                padding, dilation, True, target)
        if has_bias and ctx.needs_input_grad[2]:
            db = dy.reshape(-1, dy.shape[-1]).sum(0)
        return dx, dw, db, None, None, None, None


def conv2d(x, w, bias=None, stride=1, padding=0, dilation=1, relu=False):
    return Conv2dF32Fn.apply(x, w, bias, stride, padding, dilation, relu)


class BatchNormF32Fn(torch.autograd.Function):
    """BatchNorm over the last dim (+ residual, ReLU) of fp32 activations; training statistics from a
    shifted two-pass reduction with a double-precision finalize (`fp32x3.hip`)."""

    @staticmethod
    def forward(ctx, x, gamma, beta, residual, running_mean, running_var, training, momentum, eps, relu, nbt):
        x = x.contiguous()
        res = residual.contiguous() if residual is not None else None
        if training:
            y, mean, invstd = C().bn_f32_fwd_train(x, res, gamma, beta, running_mean, running_var, momentum, eps,
                                                   relu, nbt)
        else:
            mean = running_mean
            invstd = torch.rsqrt(running_var + eps)
            g = gamma if gamma is not None else torch.ones_like(invstd)
            b = beta if beta is not None else torch.zeros_like(invstd)
            ss = torch.cat([g * invstd, b - mean * g * invstd])
            y = C().bn_f32_apply(x, res, ss, relu)
        ctx.save_for_backward(x, y if relu else None, mean, invstd, gamma)
        ctx.cfg = (training, residual is not None, beta is not None)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, y, mean, invstd, gamma = ctx.saved_tensors
        training, has_res, has_beta = ctx.cfg
        dy = dy.contiguous()
        if training:
            dx, g, dgamma, dbeta = C().bn_f32_bwd(dy, x, y, mean, invstd, gamma, has_res)
        else:  # eval-mode backward (frozen statistics): elementwise, torch ops are fine
            g = dy * (y > 0) if y is not None else dy
            gf = g.reshape(-1, g.shape[-1])
            xh = (x.reshape(-1, x.shape[-1]) - mean) * invstd
            dgamma, dbeta = (gf * xh).sum(0), gf.sum(0)
            dx = g * (invstd * (gamma if gamma is not None else 1.0))
        return (dx, dgamma if gamma is not None else None, dbeta if has_beta else None, g if has_res else None,
                None, None, None, None, None, None, None)


def batch_norm(x, gamma, beta, running_mean, running_var, training, momentum, eps, residual=None, relu=False,
               num_batches_tracked=None):
    if momentum is None:
        raise NotImplementedError("fp32 BatchNorm: cumulative moving average (momentum=None) is not supported")
    return BatchNormF32Fn.apply(x, gamma, beta, residual, running_mean, running_var, training, momentum, eps, relu,
                                num_batches_tracked if training else None)


class MaxPoolF32Fn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, k, s, p):
        y, idx = C().maxpool_f32_fwd(x.contiguous(), k, s, p)
        ctx.save_for_backward(idx)
        ctx.cfg = (x.shape[1], x.shape[2], k, s, p)
        return y

    @staticmethod
    def backward(ctx, dy):
        (idx,) = ctx.saved_tensors
        H, W, k, s, p = ctx.cfg
        return C().maxpool_f32_bwd(dy.contiguous(), idx, H, W, k, s, p), None, None, None


class AvgPoolF32Fn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        ctx.hw = (x.shape[1], x.shape[2])
        return C().avgpool_f32_fwd(x.contiguous())

    @staticmethod
    def backward(ctx, dy):
        return C().avgpool_f32_bwd(dy.contiguous(), *ctx.hw)
