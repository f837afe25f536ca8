"""Activations (SURVEY §2.5 K03 ReLU, K21 GELU-tanh / SwiGLU) over the native elementwise kernels."""
from __future__ import annotations

import torch
import torch.nn.functional as F

from .._native import C


class _ActFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, op):
        x = x.contiguous()
        y = C().act_fwd(x, op)
        ctx.save_for_backward(y if op == 0 else x)
        ctx.op = op
        return y

    @staticmethod
    def backward(ctx, dy):
        (ref,) = ctx.saved_tensors
        return C().act_bwd(dy.contiguous(), ref, ctx.op), None


class _SwiGLUFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, gu):
        gu = gu.contiguous()
        ctx.save_for_backward(gu)
        return C().swiglu_fwd(gu)

    @staticmethod
    def backward(ctx, dy):
        (gu,) = ctx.saved_tensors
        return C().swiglu_bwd(dy.contiguous(), gu)


def _native_ok(x):
    return x.is_cuda and x.dtype in (torch.float32, torch.bfloat16)


def relu(x):
    return _ActFn.apply(x, 0) if _native_ok(x) else torch.relu(x)


def gelu_tanh(x):
    return _ActFn.apply(x, 1) if _native_ok(x) else F.gelu(x.float(), approximate="tanh").to(x.dtype)


def swiglu(gate_up):
    """``silu(g) * u`` for a fused ``[..., 2F]`` gate|up projection output."""
    if _native_ok(gate_up) and gate_up.shape[-1] % 16 == 0:
        return _SwiGLUFn.apply(gate_up)
    g, u = gate_up.float().chunk(2, dim=-1)
    return (F.silu(g) * u).to(gate_up.dtype)
