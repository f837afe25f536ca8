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


# ---------------------------------------------------------------- serving (KV cache, no autograd)
def _rope_at(x, cos, sin, pos):
    """Reference rotation of x [B, T, H, D] at absolute positions pos..pos+T-1."""
    return _rope_ref(x, cos[pos: pos + x.shape[1]], sin[pos: pos + x.shape[1]])


def decode_attention(q, k_cache, v_cache, L: int, scale: Optional[float] = None, splits: int = 0):
    """One query token per sequence against the first ``L`` rows of a KV cache.

    q ``[B, 1, Hq, D]``, caches ``[B, Tmax, Hkv, D]`` (GQA: Hq a multiple of Hkv).  GPU bf16: the
    split-sequence HIP kernel (`csrc/kernels/decode_attn.hip`); otherwise reference math."""
    D = q.shape[-1]
    scale = scale if scale is not None else 1.0 / math.sqrt(D)
    if q.is_cuda and q.dtype == torch.bfloat16 and D in (64, 128):
        return C().decode_attn(q, k_cache, v_cache, L, scale, splits)
    return attention_ref(q, k_cache[:, :L], v_cache[:, :L], causal=False, scale=scale)


@torch.no_grad()
def attention_cached(qkv: torch.Tensor, n_heads: int, n_kv_heads: int, k_cache: torch.Tensor, v_cache: torch.Tensor,
                     pos, rope: Optional[Tuple[torch.Tensor, torch.Tensor]] = None,
                     scale: Optional[float] = None) -> torch.Tensor:
    """Inference attention over a KV cache (SURVEY §2.4 W8 serving path).

    ``qkv`` ``[B, T, Hq + 2*Hkv, D]`` holds the new tokens at positions ``pos .. pos+T-1``; their
    (rotated) K and V are written into ``k_cache``/``v_cache`` ``[B, Tmax, Hkv, D]`` rows
    ``pos .. pos+T-1``.  ``T > 1`` is a prefill from position 0 (causal flash attention over the
    prompt); ``T == 1`` is a decode step (split-sequence decode kernel over ``pos + 1`` rows).
    ``rope`` = full-length (cos, sin) tables, indexed by absolute position.  Returns ``[B, T, Hq, D]``.
    ``pos`` may be a device int32 tensor (decode only): the position is then read by the kernels at
    run time, so the whole step can be captured once in a HIP graph and replayed every token.
    """
    B, T, _, D = qkv.shape
    hq, hkv = n_heads, n_kv_heads
    native = qkv.is_cuda and qkv.dtype == torch.bfloat16 and D in (64, 128)
    scale = scale if scale is not None else 1.0 / math.sqrt(D)
    if isinstance(pos, torch.Tensor):
        # device-resident position (HIP-graph replayable decode step): one append + one attention launch
        if T != 1:
            raise ValueError("a device position drives single-token decode steps only")
        if native:
            cs, sn = rope if rope is not None else (None, None)
            q = C().kv_append(qkv, k_cache, v_cache, pos, hq, hkv, cs, sn)
            return C().decode_attn(q, k_cache, v_cache, k_cache.shape[1], scale, 0, pos)
        pos = int(pos.item())
    if pos + T > k_cache.shape[1]:
        raise ValueError(f"KV cache holds {k_cache.shape[1]} positions, step needs {pos + T}")
    if T > 1 and pos != 0:
        raise ValueError("multi-token steps are prefills from position 0 (decode one token at a time)")
    q, k, v = qkv[:, :, :hq], qkv[:, :, hq: hq + hkv], qkv[:, :, hq + hkv:]
    kc, vc = k_cache[:, pos: pos + T], v_cache[:, pos: pos + T]
    if rope is not None:
        cs, sn = rope[0][pos: pos + T], rope[1][pos: pos + T]
        if native:
            q = C().rope(q, cs, sn, False, None)
            C().rope(k, cs, sn, False, kc)  # rotated K straight into the cache rows
        else:
            q = _rope_at(q, rope[0], rope[1], pos)
            kc.copy_(_rope_at(k, rope[0], rope[1], pos))
    else:
        kc.copy_(k)
    vc.copy_(v)
    if T == 1:
        return decode_attention(q, k_cache, v_cache, pos + 1, scale)
    if native:
        return C().attn_fwd(q, kc, vc, scale, True, None, None)[0]
    return attention_ref(q, kc, vc, causal=True, scale=scale)


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
