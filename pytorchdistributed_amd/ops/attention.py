"""Flash attention, token embedding (K24) and rotary embedding (K23).

``attention_qkv`` consumes the fused QKV projection output ``[B, T, Hq + 2*Hkv, D]`` in place (the
kernels take arbitrary batch/time/head strides) and its backward writes dQ, dK, dV straight into one
fused gradient buffer, so neither direction materialises separate q/k/v copies.

RoPE: one rotary pass over the Q and K heads before the forward kernel (and the inverse rotation of
dQ/dK, written straight into the fused gradient, after the backward kernels).  The kernels can
also rotate while loading (``rope_cos``/``rope_sin`` arguments) but that re-rotates every K tile for
every query block — T/64 times per element, measured 2.9 ms per Llama-3 layer for dK/dV at T = 4096 —
while the separate pass costs one read + write of Q and K.
"""
from __future__ import annotations

import math
from typing import Optional, Tuple

import torch
import torch.nn.functional as F

from .._native import C
from ..parallel.flat import grad_target


# ---------------------------------------------------------------- reference (CPU / oracle)
def _rope_ref(x, cos, sin):
    # x [B, T, H, D]; rotate-half convention
    d2 = x.shape[-1] // 2
    x1, x2 = x[..., :d2].float(), x[..., d2:].float()
    c = cos[: x.shape[1]].view(1, x.shape[1], 1, d2)
    s = sin[: x.shape[1]].view(1, x.shape[1], 1, d2)
    return torch.cat([x1 * c - x2 * s, x2 * c + x1 * s], -1).to(x.dtype)


def attention_ref(q, k, v, causal=True, scale=None, rope=None):
    """[B,T,H,D] reference via PyTorch SDPA math (fp32)."""
    if rope is not None:
        q, k = _rope_ref(q, *rope), _rope_ref(k, *rope)
    hq, hk = q.shape[2], k.shape[2]
    qf, kf, vf = (t.float().transpose(1, 2) for t in (q, k, v))
    if hq != hk:
        kf = kf.repeat_interleave(hq // hk, dim=1)
        vf = vf.repeat_interleave(hq // hk, dim=1)
    scale = scale if scale is not None else 1.0 / math.sqrt(q.shape[-1])
    s = (qf @ kf.transpose(-1, -2)) * scale
    if causal:
        T = q.shape[1]
        s = s.masked_fill(torch.triu(torch.ones(T, T, dtype=torch.bool, device=s.device), 1), float("-inf"))
    o = torch.softmax(s, -1) @ vf
    return o.transpose(1, 2).to(q.dtype)


def rope_tables(T: int, D: int, theta: float = 10000.0, device=None) -> Tuple[torch.Tensor, torch.Tensor]:
    inv = 1.0 / (theta ** (torch.arange(0, D, 2, dtype=torch.float64) / D))
    t = torch.arange(T, dtype=torch.float64)
    f = torch.outer(t, inv)
    return f.cos().float().contiguous().to(device), f.sin().float().contiguous().to(device)


# ---------------------------------------------------------------- autograd functions
class _AttnQKVFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, qkv, hq, hkv, causal, scale, rcos, rsin):
        v = qkv[:, :, hq + hkv:]
        qk = qkv[:, :, : hq + hkv]
        if rcos is not None:
            qk = C().rope(qk, rcos, rsin, False, None)  # rotated Q|K, [B, T, hq + hkv, D]
        o, lse = C().attn_fwd(qk[:, :, :hq], qk[:, :, hq:], v, scale, causal, None, None)
        ctx.save_for_backward(qkv, qk if rcos is not None else None, o, lse, rcos, rsin)
        ctx.cfg = (hq, hkv, causal, scale)
        return o

    @staticmethod
    def backward(ctx, do):
        qkv, qk, o, lse, rcos, rsin = ctx.saved_tensors
        hq, hkv, causal, scale = ctx.cfg
        dqkv = torch.empty_like(qkv)
        if qk is None:
            qk = qkv[:, :, : hq + hkv]
            dqk = dqkv[:, :, : hq + hkv]
        else:
            dqk = torch.empty_like(qk)
        C().attn_bwd(do.contiguous(), qk[:, :, :hq], qk[:, :, hq:], qkv[:, :, hq + hkv:], o, lse,
                     dqk[:, :, :hq], dqk[:, :, hq:], dqkv[:, :, hq + hkv:], scale, causal, None, None)
        if rcos is not None:
            C().rope(dqk, rcos, rsin, True, dqkv[:, :, : hq + hkv])  # gradient w.r.t. the unrotated Q|K
        return dqkv, None, None, None, None, None, None


def attention_qkv(qkv: torch.Tensor, n_heads: int, n_kv_heads: Optional[int] = None, causal: bool = True,
                  scale: Optional[float] = None, rope: Optional[Tuple[torch.Tensor, torch.Tensor]] = None):
    """qkv: ``[B, T, Hq + 2*Hkv, D]`` (view of the fused projection). Returns ``[B, T, Hq, D]``."""
    hkv = n_kv_heads or n_heads
    D = qkv.shape[-1]
    scale = scale if scale is not None else 1.0 / math.sqrt(D)
    if qkv.is_cuda and qkv.dtype == torch.bfloat16 and D in (64, 128):
        rc, rs = rope if rope is not None else (None, None)
        return _AttnQKVFn.apply(qkv, n_heads, hkv, causal, scale, rc, rs)
    q, k, v = qkv[:, :, :n_heads], qkv[:, :, n_heads: n_heads + hkv], qkv[:, :, n_heads + hkv:]
    return attention_ref(q, k, v, causal, scale, rope)


class _EmbeddingFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, idx, table):
        ctx.save_for_backward(idx)
        ctx.V = table.shape[0]
        ctx.table = table
        return C().embedding_fwd(idx.contiguous(), table.contiguous())

    @staticmethod
    def backward(ctx, dy):
        (idx,) = ctx.saved_tensors
        return None, C().embedding_bwd(idx.contiguous(), dy.contiguous(), ctx.V, grad_target(ctx.table))


def embedding(idx: torch.Tensor, table: torch.Tensor) -> torch.Tensor:
    if table.is_cuda and table.dtype == torch.bfloat16 and table.shape[1] % 8 == 0:
        return _EmbeddingFn.apply(idx, table)
    return F.embedding(idx, table)
