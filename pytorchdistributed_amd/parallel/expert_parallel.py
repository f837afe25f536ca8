"""Expert parallelism: a top-k routed mixture-of-experts layer whose experts are sharded over an EP
group (SURVEY §2.2 P18 — not in the reference or the BASELINE configs; provided because on an
MI355X node the token exchange is one all-to-all, which drives all 7 xGMI links of every GPU at once).

Forward, per rank (tokens are this rank's data-parallel shard):
  1. router logits -> top-k experts and their softmax weights (replicated router);
  2. the (token, expert) assignments are sorted by destination rank and exchanged with ONE uneven
     all-to-all of the token rows (plus one of the expert ids; the split sizes go first);
  3. each local expert (SwiGLU FFN on the native GEMM / SwiGLU kernels) runs on its received rows;
  4. the reverse all-to-all returns the outputs, which are scaled by the routing weights and summed
     per token.
Backward mirrors it: the all-to-all's adjoint is the reverse all-to-all with the splits swapped.
Expert weights live on exactly one rank, so their gradients are complete after backward; the
replicated router's gradients are summed over the group like any data-parallel parameter
(:func:`sync_router_grads`).

    moe = ExpertParallelMoE(dim=4096, ffn_dim=14336, n_experts=8, top_k=2, group=ep_group)
    y = moe(x)               # x [tokens, dim] -> [tokens, dim]
"""
from __future__ import annotations

import math
from typing import List

import torch
import torch.distributed as dist
import torch.nn as tnn

from .. import ops


def _a2a(x: torch.Tensor, out_splits: List[int], in_splits: List[int], group) -> torch.Tensor:
    out = x.new_empty((sum(out_splits),) + tuple(x.shape[1:]))
    if x.is_cuda and dist.get_backend(group) == "gloo":  # rehearsal with ranks sharing a GPU
        host = out.cpu()
        dist.all_to_all_single(host, x.cpu(), out_splits, in_splits, group=group)
        return host.to(x.device)
    dist.all_to_all_single(out, x.contiguous(), out_splits, in_splits, group=group)
    return out


class _AllToAll(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, out_splits, in_splits, group):
        ctx.meta = (out_splits, in_splits, group)
        return _a2a(x, out_splits, in_splits, group)

    @staticmethod
    def backward(ctx, g):
        out_splits, in_splits, group = ctx.meta
        return _a2a(g.contiguous(), in_splits, out_splits, group), None, None, None


class ExpertParallelMoE(tnn.Module):
    def __init__(self, dim: int, ffn_dim: int, n_experts: int, top_k: int = 2, group=None, device=None,
                 dtype=None, seed: int = 0):
        super().__init__()
        self.group = group
        self.P = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        if n_experts % self.P:
            raise ValueError(f"{n_experts} experts do not divide over {self.P} ranks")
        self.E, self.k, self.El = n_experts, top_k, n_experts // self.P
        kw = dict(device=device, dtype=dtype)
        g = torch.Generator().manual_seed(seed)  # identical full init on every rank, then keep the shard
        std = 1.0 / math.sqrt(dim)
        self.router = tnn.Parameter((torch.randn(n_experts, dim, generator=g) * std).to(**kw))
        w13 = torch.randn(n_experts, 2 * ffn_dim, dim, generator=g) * std
        w2 = torch.randn(n_experts, dim, ffn_dim, generator=g) / math.sqrt(ffn_dim)
        lo = self.rank * self.El
        self.w13 = tnn.Parameter(w13[lo: lo + self.El].to(**kw).contiguous())  # [El, 2F, d] gate | up
        self.w2 = tnn.Parameter(w2[lo: lo + self.El].to(**kw).contiguous())    # [El, d, F]

    def _expert(self, e: int, x: torch.Tensor) -> torch.Tensor:
        return ops.linear(ops.swiglu(ops.linear(x, self.w13[e])), self.w2[e])

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        N, d = x.shape
        logits = ops.linear(x, self.router).float()
        top_v, top_i = torch.topk(logits, self.k, dim=-1)
        gate = torch.softmax(top_v, -1).to(x.dtype)                        # [N, k]
        flat_e = top_i.reshape(-1)                                         # [N*k]
        order = torch.argsort(flat_e, stable=True)                         # grouped by expert = by rank
        tok = order // self.k
        send_e = flat_e[order]
        send_x = x[tok]
        per_rank = torch.bincount(send_e // self.El, minlength=self.P)
        in_splits = per_rank.tolist()
        if self.P > 1:
            # split sizes first (device tensors on RCCL, host tensors on gloo)
            cdev = x.device if dist.get_backend(self.group) == "nccl" else torch.device("cpu")
            cnt = torch.tensor(in_splits, dtype=torch.long, device=cdev)
            recv_cnt = torch.empty_like(cnt)
            dist.all_to_all_single(recv_cnt, cnt, group=self.group)
            out_splits = recv_cnt.tolist()
            recv_x = _AllToAll.apply(send_x, out_splits, in_splits, self.group)
            recv_e = _a2a(send_e, out_splits, in_splits, self.group)
        else:
            out_splits, recv_x, recv_e = in_splits, send_x, send_e
        local_e = recv_e - self.rank * self.El
        y = torch.zeros_like(recv_x)
        for e in range(self.El):
            sel = (local_e == e).nonzero(as_tuple=True)[0]
            if sel.numel():
                y = y.index_copy(0, sel, self._expert(e, recv_x[sel]))
        back = _AllToAll.apply(y, in_splits, out_splits, self.group) if self.P > 1 else y
        w = gate.reshape(-1)[order].unsqueeze(1)
        return torch.zeros_like(x).index_add(0, tok, back * w)

    @torch.no_grad()
    def sync_router_grads(self):
        """Sum the replicated router's gradient over the group (each rank routed its own tokens)."""
        if self.P > 1 and self.router.grad is not None:
            dist.all_reduce(self.router.grad, group=self.group)


def sync_router_grads(moe: ExpertParallelMoE):
    moe.sync_router_grads()


def dense_moe_reference(x, router, w13, w2, top_k, top=None):
    """All experts on one device, plain PyTorch math (the oracle of the EP tests).  ``top`` = given
    (values, indices) routing, so a bf16 run can be checked without near-tie routing flips."""
    if top is None:
        top = torch.topk(x.float() @ router.float().t(), top_k, dim=-1)
    top_v, top_i = top[0].float(), top[1]
    gate = torch.softmax(top_v, -1)
    out = torch.zeros_like(x, dtype=torch.float32)
    F = w2.shape[-1]
    for j in range(top_k):
        for e in range(router.shape[0]):
            sel = top_i[:, j] == e
            if sel.any():
                h = x[sel].float() @ w13[e].float().t()
                a = torch.nn.functional.silu(h[:, :F]) * h[:, F:]
                out[sel] += gate[sel, j: j + 1] * (a @ w2[e].float().t())
    return out.to(x.dtype)
