"""Linear layer ``y = x W^T + b`` (reference `nn.Linear(20,1)` `ddp_gpus.py:77`,
the 4-layer MLP `01_multi_gpus_data_parallelism.ipynb` raw lines 94-107, ResNet `fc`).

GPU, bf16 with in/out features multiples of 8: the MFMA GEMM (forward K-major x K-major, dgrad
K-major x MN-major, wgrad MN-major x MN-major via LDS transpose reads, split-K when the tile grid is
small).  GPU otherwise (fp32 models, odd widths): the general-stride SIMT GEMM kernel.

Plain (epilogue-free) large GEMMs go to the vendor library (hipBLASLt through ``torch.mm``) under
``PDA_GEMM=auto`` (default): on the 4096^3 bf16 probe it runs 1.47 PF/s against 0.67 PF/s for the
native 128x128 MFMA tile (profiles/r1_conv_gemm_microbench.md), and a plain GEMM is exactly the case
the library is tuned for.  Fused cases (ReLU epilogue) and everything else stay native;
``PDA_GEMM=native`` forces the native kernel everywhere, ``PDA_GEMM=blas`` the library.
"""
from __future__ import annotations

import os

import torch
import torch.nn.functional as F

from .._native import C
from ..parallel.flat import grad_target
from . import streams as _streams


def _mfma_ok(x2, w):
    return (x2.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and w.shape[0] % 8 == 0 and w.shape[1] % 8 == 0)


_SIDE_MAX_NUMEL = 256 * 256 * 256  # 256 CUs x one 256x256 tile
_BLAS_MIN_WORK = 1 << 27  # M*N*K below this: launch-latency bound, the native kernel is as good


def _use_blas(a, b, M, N, K) -> bool:
    mode = os.environ.get("PDA_GEMM", "auto")
    if mode == "native" or a.dtype != torch.bfloat16 or b.dtype != torch.bfloat16:
        return False
    return mode == "blas" or M * N * K >= _BLAS_MIN_WORK


def _gemm_fwd(x2, w, b, relu):
    M, K = x2.shape
    N = w.shape[0]
    if not relu and M > 0 and _use_blas(x2, w, M, N, K):
        if b is not None:
            return torch.addmm(b.to(x2.dtype), x2, w.t())
        return torch.mm(x2, w.t())
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
    if _use_blas(dy, w, M, N, K):
        return torch.mm(dy, w, out=dx)
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
    if dw.dtype == dy.dtype and _use_blas(dy, x2, M, N, K):
        return torch.mm(dy.t(), x2, out=dw)
    if dy.dtype == torch.bfloat16 and x2.dtype == torch.bfloat16 and N % 8 == 0 and K % 8 == 0:
        # dw[N,K] = dy^T x: A(m=n, k=r) = dy[r*N + n] (MN-major), B(k=r, col) = x[r*K + col] (MN-major)
        C().gemm(dy, False, N, x2, False, K, dw, K, N, K, M, None, False, True)
    else:
        C().simt_gemm(dy, 1, N, x2, K, 1, dw, K, 1, N, K, M, None, False, 0.0)
    return dw


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
        if ctx.needs_input_grad[1]:
            target = grad_target(ctx.wparam)
            if target is not None and _streams.enabled() and target.numel() < _SIDE_MAX_NUMEL:
                # written straight into the flat gradient slot: run it beside the critical path
                # (ops/streams.py; same contract as the conv weight gradient).  A dW with a full wave
                # of 256x256 output tiles per CU fills the chip by itself; beside other work it only
                # adds interference (Llama-3-8B FSDP: -2.4 %; GPT-2-medium DDP, 1-16 tiles + split-K:
                # +9.9 %, profiles/r2_wgrad_stream_transformers.jsonl)
                # (the bias gradient stays on the compute stream: as a side-stream column sum its
                # hundreds of memory-bound workgroups delayed the critical-path dgrad GEMMs — GPT-2-medium
                # 55.7 -> 57.0 ms/step, profiles/r2_gpt2_addnorm_ab.md)
                with _streams.wgrad_stream(dy2.device, dy2, x2):
                    dw = _gemm_wgrad(dy2, x2, w.dtype, target)
            else:
                dw = _gemm_wgrad(dy2, x2, w.dtype, target)
        if ctx.has_bias and ctx.needs_input_grad[2]:
            tb = grad_target(ctx.bparam)
            db = C().colsum(dy2)
            db = tb.copy_(db) if tb is not None else db.to(ctx.bparam.dtype)
        return dx, dw, db, None


def linear(x: torch.Tensor, weight: torch.Tensor, bias=None, relu: bool = False) -> torch.Tensor:
    if x.is_cuda:
        return _LinearFn.apply(x, weight, bias, relu)
    y = F.linear(x, weight, bias)
    return torch.relu(y) if relu else y
