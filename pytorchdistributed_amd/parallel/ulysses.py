"""Ulysses sequence parallelism (the long-context option that fits the xGMI
full mesh — one all-to-all drives all 7 links of every GPU at once, where ring attention streams K/V
over one link at a time).

Each rank of the SP group holds a contiguous sequence shard ``[B, T/P, H, D]`` of Q, K and V.  One
all-to-all re-partitions them to ``[B, T, H/P, D]`` (full sequence, a head slice), the unchanged
flash-attention kernel (K22, causal, GQA) runs on the local heads, and a second all-to-all returns
the output to the sequence layout.  Backward is the mirror image (the all-to-all is its own adjoint
up to the inverse permutation).  Communication per layer: 3 + 1 tensors of B·T·H·D/P elements per
rank forward, the same backward — independent of P, so it scales with the mesh.

    o = ulysses_attention(q, k, v, group, causal=True)          # q/k/v: local sequence shards
"""
from __future__ import annotations

import math
from typing import Optional

import torch
import torch.distributed as dist

from ..ops.attention import attention_ref
from .._native import C


def _all_to_all(send: torch.Tensor, group) -> torch.Tensor:
    recv = torch.empty_like(send)
    if send.is_cuda and dist.get_backend(group) == "gloo":  # rehearsal (ranks sharing a GPU): stage on host
        host = torch.empty_like(send, device="cpu")
        dist.all_to_all_single(host, send.cpu(), group=group)
        recv.copy_(host)
    else:
        dist.all_to_all_single(recv, send, group=group)  # RCCL: all 7 xGMI links at once
    return recv


def _a2a_seq_to_heads(x: torch.Tensor, group) -> torch.Tensor:
    """[B, T/P, H, D] (sequence shard) -> [B, T, H/P, D] (head shard)."""
    P = dist.get_world_size(group)
    B, Ts, H, D = x.shape
    # split heads into P groups; chunk p goes to rank p
    send = x.reshape(B, Ts, P, H // P, D).permute(2, 0, 1, 3, 4).contiguous()  # [P, B, Ts, H/P, D]
    recv = _all_to_all(send, group)  # recv[p] = rank p's sequence shard of my heads
    return recv.permute(1, 0, 2, 3, 4).reshape(B, P * Ts, H // P, D)


def _a2a_heads_to_seq(x: torch.Tensor, group) -> torch.Tensor:
    """[B, T, H/P, D] (head shard) -> [B, T/P, H, D] (sequence shard)."""
    P = dist.get_world_size(group)
    B, T, Hs, D = x.shape
    send = x.reshape(B, P, T // P, Hs, D).permute(1, 0, 2, 3, 4).contiguous()  # [P, B, T/P, H/P, D]
    recv = _all_to_all(send, group)  # recv[p] = my sequence shard of rank p's heads
    return recv.permute(1, 2, 0, 3, 4).reshape(B, T // P, P * Hs, D)


class _SeqToHeads(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        return _a2a_seq_to_heads(x, group)

    @staticmethod
    def backward(ctx, g):
        return _a2a_heads_to_seq(g.contiguous(), ctx.group), None


class _HeadsToSeq(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        return _a2a_heads_to_seq(x, group)

    @staticmethod
    def backward(ctx, g):
        return _a2a_seq_to_heads(g.contiguous(), ctx.group), None


class _LocalAttn(torch.autograd.Function):
    """Flash attention (K22) on the local heads with an autograd backward (q, k, v separate tensors)."""

    @staticmethod
    def forward(ctx, q, k, v, causal, scale):
        o, lse = C().attn_fwd(q, k, v, scale, causal, None, None)
        ctx.save_for_backward(q, k, v, o, lse)
        ctx.cfg = (causal, scale)
        return o

    @staticmethod
    def backward(ctx, do):
        q, k, v, o, lse = ctx.saved_tensors
        causal, scale = ctx.cfg
        dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
        C().attn_bwd(do.contiguous(), q, k, v, o, lse, dq, dk, dv, scale, causal, None, None)
        return dq, dk, dv, None, None


def ulysses_attention(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, group=None, causal: bool = True,
                      scale: Optional[float] = None) -> torch.Tensor:
    """Sequence-parallel attention over the SP ``group``.  q ``[B, T/P, Hq, D]``, k/v ``[B, T/P, Hkv, D]``
    (rank r holds positions [r·T/P, (r+1)·T/P)); Hq and Hkv must be multiples of P.  Returns this
    rank's output shard ``[B, T/P, Hq, D]``."""
    P = dist.get_world_size(group)
    if q.shape[2] % P or k.shape[2] % P:
        raise ValueError(f"heads ({q.shape[2]}/{k.shape[2]}) must be divisible by the SP size {P}")
    D = q.shape[-1]
    scale = scale if scale is not None else 1.0 / math.sqrt(D)
    qh, kh, vh = (_SeqToHeads.apply(t.contiguous(), group) for t in (q, k, v))
    if qh.is_cuda and qh.dtype == torch.bfloat16 and D in (64, 128):
        oh = _LocalAttn.apply(qh, kh, vh, causal, scale)
    else:
        oh = attention_ref(qh, kh, vh, causal=causal, scale=scale)
    return _HeadsToSeq.apply(oh.contiguous(), group)
