"""Linear layer ``y = x W^T + b`` (reference `nn.Linear(20,1)` `ddp_gpus.py:77`,
the 4-layer MLP `01_multi_gpus_data_parallelism.ipynb` raw lines 94-107, ResNet `fc`).

GPU, bf16 with in/out features multiples of 8: the MFMA GEMM (forward K-major x K-major, dgrad
K-major x MN-major, wgrad MN-major x MN-major via LDS transpose reads, split-K when the tile grid is
small).  GPU otherwise (fp32 models, odd widths): the general-stride SIMT GEMM kernel.

Every bf16 GEMM runs on the native kernels: the pipelined 256x256 tile (csrc/kernels/gemm_pp.hip) takes
the large ones in all three operand layouts — on the GPT-2-medium / Llama-3-8B training shapes it is
within 85-95 % of hipBLASLt on the forward (both operands K-major), at parity on the data gradient and
1.1-2.7x faster on the weight gradient, whose bias gradient it produces in the same pass
(profiles/r4_gpt2_gemm_shapes_pp.jsonl, r4_llama_gemm_shapes_pp.jsonl); whole steps: GPT-2-medium 300k
vs 286k tok/s, Llama-3-8B FSDP 18.8k vs 18.6k (profiles/r4_gpt2_native_ab.jsonl, r4_llama_native_ab.jsonl).
There is no vendor-library path.
"""
from __future__ import annotations

import contextlib
import os

import torch
import torch.nn.functional as F

from .._native import C
from ..parallel.flat import grad_target
from . import streams as _streams


def _mfma_ok(x2, w):
    return (x2.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and w.shape[0] % 8 == 0 and w.shape[1] % 8 == 0)


_SIDE_MAX_NUMEL = 256 * 256 * 256  # 256 CUs x one 256x256 tile


def _gemm_fwd(x2, w, b, relu):
    M, K = x2.shape
    N = w.shape[0]
    if _mfma_ok(x2, w):
        y = torch.empty(M, N, device=x2.device, dtype=x2.dtype)
        if M > 0:
            C().gemm(x2, True, K, w, True, K, y, N, M, N, K, b, relu, True)
        return y
    y = torch.empty(M, N, device=x2.device, dtype=x2.dtype)
    if M > 0:
        bias = b.float() if b is not None else None
        # A(m,k) = x[m*K+k], B(k,n) = W[n*K+k]
        C().simt_gemm(x2, K, 1, w, 1, K, y, N, 1, M, N, K, bias, relu, 0.0)
    return y


def _gemm_dgrad(dy, w):
    M, N = dy.shape
    K = w.shape[1]
    dx = torch.empty(M, K, device=dy.device, dtype=dy.dtype)
    if M == 0:
        return dx
    if _mfma_ok(dy, w):
        # dx[M,K] = dy[M,N] W[N,K]:  A = dy (K-major, lda N), B(k=n, col=kk) = W[n*K + kk] (MN-major, ldb K)
        C().gemm(dy, True, N, w, False, K, dx, K, M, K, N, None, False, True)
    else:
        C().simt_gemm(dy, N, 1, w, K, 1, dx, K, 1, M, K, N, None, False, 0.0)
    return dx


def _gemm_wgrad(dy, x2, out_dtype, target=None):
    M, N = dy.shape
    K = x2.shape[1]
    dw = target if target is not None else torch.empty(N, K, device=dy.device, dtype=out_dtype)
    if M == 0:
        return dw.zero_()
    if dy.dtype == torch.bfloat16 and x2.dtype == torch.bfloat16 and N % 8 == 0 and K % 8 == 0:
        # dw[N,K] = dy^T x: A(m=n, k=r) = dy[r*N + n] (MN-major), B(k=r, col) = x[r*K + col] (MN-major)
        C().gemm(dy, False, N, x2, False, K, dw, K, N, K, M, None, False, True)
    else:
        C().simt_gemm(dy, 1, N, x2, K, 1, dw, K, 1, N, K, M, None, False, 0.0)
    return dw


def _fused_wgrad_db(dy2, x2, wparam, bparam, target, tb):
    """dW and db from ONE pipelined GEMM (db = row sums of its A operand dY^T), or None when
    the shape does not take that kernel (the caller falls back to GEMM + column sum).  ``target`` / ``tb``
    are the flat-buffer slots the caller claimed (each slot is claimed exactly once per backward)."""
    if os.environ.get("PDA_WGRAD_DB_FUSED", "1") != "1":
        return None
    if not (dy2.dtype == x2.dtype == torch.bfloat16 and dy2.shape[1] % 8 == 0 and x2.shape[1] % 8 == 0):
        return None
    N, K = dy2.shape[1], x2.shape[1]
    dw = target if target is not None else torch.empty(N, K, device=dy2.device, dtype=wparam.dtype)
    db = tb if tb is not None else torch.empty(N, device=dy2.device, dtype=bparam.dtype)
    if db.dtype not in (torch.bfloat16, torch.float32) or dw.dtype not in (torch.bfloat16, torch.float32):
        return None
    if not C().gemm_wgrad_db(dy2, x2, dw, db):
        return dw, None  # dw written; the bias gradient still needs its column sum
    return dw, db


def _param_grads(dy2, x2, wparam, bparam, need_w, need_b):
    """Weight and bias gradients of ``y = x W^T + b`` (dy2 [M, N], x2 [M, K]), written into the flat
    gradient buffers when the parameters have them.  With both needed, the native weight-gradient GEMM
    also produces the bias gradient (its A operand's row sums) when it runs on the pipelined tile."""
    dw = db = None
    # claim each flat slot ONCE: a second grad_target() on the same parameter reads as a tied weight
    # (flat.py), which would push the parameter off the side stream for good
    target = grad_target(wparam) if need_w else None
    tb = grad_target(bparam) if need_b else None
    side = target is not None and _streams.side_ok(wparam) and target.numel() < _SIDE_MAX_NUMEL
    if need_w and need_b and dy2.shape[0] > 0:
        with (_streams.wgrad_stream(dy2.device, dy2, x2) if side else contextlib.nullcontext()):
            r = _fused_wgrad_db(dy2, x2, wparam, bparam, target, tb)
        if r is not None:
            dw, db = r
            if db is None:
                db = C().colsum(dy2, out=tb, out_bf16=bparam.dtype == torch.bfloat16)
                if db.dtype != bparam.dtype:
                    db = db.to(bparam.dtype)
            return dw, db
    if need_w:
        if side:
            # written straight into the flat gradient slot: run it beside the critical path
            # (ops/streams.py; same contract as the conv weight gradient).  A dW with a full wave
            # of 256x256 output tiles per CU fills the chip by itself; beside other work it only
            # adds interference (Llama-3-8B FSDP: -2.4 %; GPT-2-medium DDP, 1-16 tiles + split-K:
            # +9.9 %, profiles/r2_wgrad_stream_transformers.jsonl)
            # (the bias gradient stays on the compute stream: as a side-stream column sum its
            # hundreds of memory-bound workgroups delayed the critical-path dgrad GEMMs — GPT-2-medium
            # 55.7 -> 57.0 ms/step, profiles/r2_gpt2_addnorm_ab.md)
            with _streams.wgrad_stream(dy2.device, dy2, x2):
                dw = _gemm_wgrad(dy2, x2, wparam.dtype, target)
        else:
            dw = _gemm_wgrad(dy2, x2, wparam.dtype, target)
    if need_b:
        # written in the parameter dtype, straight into its flat-buffer slot when it has one
        db = C().colsum(dy2, out=tb, out_bf16=bparam.dtype == torch.bfloat16)
        if db.dtype != bparam.dtype:
            db = db.to(bparam.dtype)
    return dw, db


class _LinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, relu):
        shape = x.shape
        x2 = x.reshape(-1, shape[-1]).contiguous()
        w = w.contiguous()
        y = _gemm_fwd(x2, w, b, relu)
        ctx.save_for_backward(x2, w, y if relu else None)
        ctx.relu = relu
        ctx.has_bias = b is not None
        ctx.shape = shape
        ctx.wparam, ctx.bparam = w, b
        return y.reshape(*shape[:-1], w.shape[0])

    @staticmethod
    def backward(ctx, dy):
        x2, w, y = ctx.saved_tensors
        dy2 = dy.reshape(-1, w.shape[0]).contiguous()
        if ctx.relu:
            dy2 = C().relu_bwd(dy2, y)
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = _gemm_dgrad(dy2, w).reshape(ctx.shape)
        dw, db = _param_grads(dy2, x2, ctx.wparam, ctx.bparam if ctx.has_bias else None,
                              ctx.needs_input_grad[1], ctx.has_bias and ctx.needs_input_grad[2])
        return dx, dw, db, None


class _MlpGeluFn(torch.autograd.Function):
    """``fc2(gelu_tanh(fc1(x)))`` with the activation inside the GEMM epilogues: the fc1 forward writes
    the pre-activation h and g = gelu(h) in one pass, and the fc2 data gradient is produced as
    ``(dy W2) * gelu'(h)`` (gemm_conv.hip Epi::act) — no elementwise pass over the two [tokens, 4d]
    tensors in either direction."""

    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2):
        ctx.params = (w1, b1, w2, b2)  # the parameters themselves: grad_target finds their flat slots
        shape = x.shape
        x2 = x.reshape(-1, shape[-1]).contiguous()
        w1, w2 = w1.contiguous(), w2.contiguous()
        M, K = x2.shape
        F_ = w1.shape[0]
        h = torch.empty(M, F_, device=x.device, dtype=x.dtype)
        g = torch.empty_like(h)
        if M > 0:
            C().gemm_act(x2, True, K, w1, True, K, g, F_, M, F_, K, b1, 1, h)
        y = _gemm_fwd(g, w2, b2, False)
        ctx.save_for_backward(x2, w1, h, g, w2)
        ctx.shape = shape
        return y.reshape(*shape[:-1], w2.shape[0])

    @staticmethod
    def backward(ctx, dy):
        x2, w1, h, g, w2 = ctx.saved_tensors
        pw1, pb1, pw2, pb2 = ctx.params
        N = w2.shape[0]
        dy2 = dy.reshape(-1, N).contiguous()
        M, F_ = h.shape
        # fc2 data gradient fused with the GELU backward: dh = (dy W2) * gelu'(h), W2 read in place as the
        # MN-major B operand (B(k, f) = W2[k * F + f]): the pipelined tile runs that layout at the K-major
        # rate (profiles/r4_gpt2_gemm_shapes_pp.jsonl dgrad rows), so no per-step transposed copy
        dh = torch.empty_like(h)
        if M > 0:
            C().gemm_act(dy2, True, N, w2, False, F_, dh, F_, M, F_, N, None, 2, h)
        dw2, db2 = _param_grads(dy2, g, pw2, pb2, ctx.needs_input_grad[3], pb2 is not None and ctx.needs_input_grad[4])
        dx = _gemm_dgrad(dh, w1).reshape(ctx.shape) if ctx.needs_input_grad[0] else None
        dw1, db1 = _param_grads(dh, x2, pw1, pb1, ctx.needs_input_grad[1], pb1 is not None and ctx.needs_input_grad[2])
        return dx, dw1, db1, dw2, db2


def mlp_fused_ok(x, w1, w2) -> bool:
    """The fused GELU MLP applies: GPU bf16, widths multiples of 8, ``PDA_MLP_FUSED`` not ``0``.  On by
    default since the pipelined tile carries the forward / backward GEMMs: GPT-2-medium 308.7k vs 300.4k
    tok/s unfused (profiles/r4_gpt2_native_ab.jsonl; it lost to hipBLASLt + two elementwise passes while
    the GEMMs were the 2-stage wide tile, r2_gpt2_mlp_fused_ab.jsonl / r3_gpt2_mlp_fused_wt_DROPPED.jsonl)."""
    return (x.is_cuda and x.dtype == torch.bfloat16 and _mfma_ok(x, w1) and _mfma_ok(x, w2)
            and os.environ.get("PDA_MLP_FUSED", "1") != "0")


def mlp_gelu(x, w1, b1, w2, b2):
    """``linear(gelu_tanh(linear(x, w1, b1)), w2, b2)`` — GPT-2's MLP.  GPU bf16: :class:`_MlpGeluFn`
    (activation fused into the GEMM epilogues); otherwise the unfused composition."""
    if mlp_fused_ok(x, w1, w2):
        return _MlpGeluFn.apply(x, w1, b1, w2, b2)
    from .act import gelu_tanh

    return linear(gelu_tanh(linear(x, w1, b1)), w2, b2)


def linear(x: torch.Tensor, weight: torch.Tensor, bias=None, relu: bool = False) -> torch.Tensor:
    if x.is_cuda:
        return _LinearFn.apply(x, weight, bias, relu)
    y = F.linear(x, weight, bias)
    return torch.relu(y) if relu else y
