"""Ring attention / context parallelism: every rank keeps its sequence shard of
Q and passes K/V shards around a ring of the CP group, merging blockwise flash-attention results with
their log-sum-exp.  Not in the reference; provided for completeness next to Ulysses
(`parallel/ulysses.py`), which is the better fit for the xGMI full mesh (one all-to-all drives all 7
links, a ring step drives one) — ring attention is the option when heads do not divide by the
parallel degree, and its per-step traffic (one K/V shard) is independent of the head count.

Forward on rank r, step s = 0..P-1 with the K/V shard of rank j = (r - s) mod P:
  j == r: causal flash attention (K22 kernel) on the diagonal block; j < r: full block; j > r: skipped
  (causal) — partial (o_j, lse_j) merged as o = Σ o_j·exp(lse_j − lse), lse = logsumexp_j lse_j.
Backward: the FA2 backward kernel on every visited block with the FINAL o / lse gives exact block
gradients; dQ accumulates locally, dK/dV accumulate in buffers that travel with their K/V shard and
arrive home after P hops.  (Causal load is unbalanced across ranks; a zig-zag shard order would fix
that and is left as a further step.)
"""
from __future__ import annotations

import math
from typing import Optional

import torch
import torch.distributed as dist

from .._native import C


# ---------------------------------------------------------------- block kernels (native or reference)
def _native(t: torch.Tensor) -> bool:
    return t.is_cuda and t.dtype == torch.bfloat16 and t.shape[-1] in (64, 128)


def _block_fwd(q, k, v, causal: bool, scale: float):
    """(o [B,T,H,D], lse [B,H,T] natural log of Σ exp(scale·qk))."""
    if _native(q):
        o, lse = C().attn_fwd(q, k, v, scale, causal, None, None)
        return o, lse
    G = q.shape[2] // k.shape[2]
    qf = q.float().transpose(1, 2)
    kf = k.float().transpose(1, 2).repeat_interleave(G, 1)
    vf = v.float().transpose(1, 2).repeat_interleave(G, 1)
    s = (qf @ kf.transpose(-1, -2)) * scale
    if causal:
        T = q.shape[1]
        s = s.masked_fill(torch.triu(torch.ones(T, T, dtype=torch.bool, device=s.device), 1), float("-inf"))
    lse = torch.logsumexp(s, -1)
    o = torch.softmax(s, -1) @ vf
    return o.transpose(1, 2).to(q.dtype), lse


def _block_bwd(do, q, k, v, o, lse, causal: bool, scale: float):
    if _native(q):
        dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
        C().attn_bwd(do.contiguous(), q, k, v, o, lse, dq, dk, dv, scale, causal, None, None)
        return dq, dk, dv
    B, T, Hq, D = q.shape
    Hkv = k.shape[2]
    G = Hq // Hkv
    qf, dof, of = (t.float().transpose(1, 2) for t in (q, do, o))
    kf = k.float().transpose(1, 2).repeat_interleave(G, 1)
    vf = v.float().transpose(1, 2).repeat_interleave(G, 1)
    s = (qf @ kf.transpose(-1, -2)) * scale
    if causal:
        s = s.masked_fill(torch.triu(torch.ones(T, T, dtype=torch.bool, device=s.device), 1), float("-inf"))
    p = torch.exp(s - lse.unsqueeze(-1))
    dv = p.transpose(-1, -2) @ dof
    dp = dof @ vf.transpose(-1, -2)
    delta = (dof * of).sum(-1, keepdim=True)
    ds = p * (dp - delta)
    dq = (ds @ kf) * scale
    dk = (ds.transpose(-1, -2) @ qf) * scale
    dk = dk.view(B, Hkv, G, T, D).sum(2)
    dv = dv.view(B, Hkv, G, T, D).sum(2)
    return (dq.transpose(1, 2).to(q.dtype), dk.transpose(1, 2).to(k.dtype), dv.transpose(1, 2).to(v.dtype))


# ---------------------------------------------------------------- ring exchange
def _ring_pass(tensors, group):
    """Send ``tensors`` to the next rank of the ring, receive the previous rank's."""
    P = dist.get_world_size(group)
    r = dist.get_rank(group)
    nxt = dist.get_global_rank(group, (r + 1) % P) if group is not None else (r + 1) % P
    prv = dist.get_global_rank(group, (r - 1) % P) if group is not None else (r - 1) % P
    stage = tensors[0].is_cuda and dist.get_backend(group) == "gloo"  # rehearsal: gloo moves host tensors
    send = [t.contiguous().cpu() if stage else t.contiguous() for t in tensors]
    recv = [torch.empty_like(t) for t in send]
    ops = [dist.P2POp(dist.isend, t, nxt, group) for t in send] + [dist.P2POp(dist.irecv, t, prv, group) for t in recv]
    for w in dist.batch_isend_irecv(ops):
        w.wait()
    return [t.to(tensors[0].device) for t in recv] if stage else recv


class _RingAttn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, group, causal, scale):
        P = dist.get_world_size(group)
        r = dist.get_rank(group)
        o_acc, lse_acc = None, None
        kc, vc = k, v
        for s in range(P):
            j = (r - s) % P
            if not (causal and j > r):
                o_j, lse_j = _block_fwd(q, kc, vc, causal and j == r, scale)
                if o_acc is None:
                    o_acc, lse_acc = o_j.float(), lse_j
                else:
                    lse_new = torch.logaddexp(lse_acc, lse_j)
                    a = torch.exp(lse_acc - lse_new).transpose(1, 2).unsqueeze(-1)
                    b = torch.exp(lse_j - lse_new).transpose(1, 2).unsqueeze(-1)
                    o_acc = o_acc * a + o_j.float() * b
                    lse_acc = lse_new
            if s < P - 1:
                kc, vc = _ring_pass([kc, vc], group)
        o = o_acc.to(q.dtype)
        ctx.save_for_backward(q, k, v, o, lse_acc.contiguous())
        ctx.cfg = (group, causal, scale)
        return o

    @staticmethod
    def backward(ctx, do):
        q, k, v, o, lse = ctx.saved_tensors
        group, causal, scale = ctx.cfg
        P = dist.get_world_size(group)
        r = dist.get_rank(group)
        dq = torch.zeros_like(q, dtype=torch.float32)
        kc, vc = k, v
        dkc = torch.zeros_like(k, dtype=torch.float32)
        dvc = torch.zeros_like(v, dtype=torch.float32)
        for s in range(P):
            j = (r - s) % P
            if not (causal and j > r):
                dq_j, dk_j, dv_j = _block_bwd(do, q, kc, vc, o, lse, causal and j == r, scale)
                dq += dq_j.float()
                dkc += dk_j.float()
                dvc += dv_j.float()
            # K/V travel on; their gradient buffers travel with them and are home after P hops
            if s < P - 1:
                kc, vc, dkc, dvc = _ring_pass([kc, vc, dkc, dvc], group)
            else:
                dkc, dvc = _ring_pass([dkc, dvc], group)
        return dq.to(q.dtype), dkc.to(k.dtype), dvc.to(v.dtype), None, None, None


def ring_attention(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, group=None, causal: bool = True,
                   scale: Optional[float] = None) -> torch.Tensor:
    """Context-parallel attention: q ``[B, T/P, Hq, D]``, k/v ``[B, T/P, Hkv, D]`` = this rank's
    contiguous sequence shard (rank r holds positions [r·T/P, (r+1)·T/P)).  Returns the output shard."""
    scale = scale if scale is not None else 1.0 / math.sqrt(q.shape[-1])
    return _RingAttn.apply(q.contiguous(), k.contiguous(), v.contiguous(), group, causal, scale)
