"""Tensor parallelism (Megatron-style) for the transformer models — training and serving.

Not in the reference (SURVEY §2.2 P14/P15 list TP/SP as out of its scope); provided because on an
MI355X node TP is how a model is spread over the xGMI mesh when one GPU's 288 GB or its decode
latency is not enough.  Design for xGMI:

* one all-reduce per sub-layer and direction (after the row-parallel ``wo`` and ``w2``; their
  mirror in backward before the column-parallel ``wqkv`` / ``w13``) — 2 collectives per block
  forward, 2 backward, each of B·T·d bf16 elements;
* heads are split, never head dimensions: rank r owns query heads [r·Hq/tp, …) and the KV heads they
  read ([r·Hkv/tp, …)), so attention (training flash kernel, serving decode kernel + KV cache) runs
  unchanged on the local heads and the KV cache shrinks by tp on every rank;
* the fused ``w13 = [gate | up]`` projection is split so that each rank holds matching gate and up
  rows: the SwiGLU kernel runs on local data;
* ``sequence_parallel=True`` replaces each all-reduce by reduce-scatter (forward) / all-gather
  (backward) over the sequence dimension, so norms and residual adds run on T/tp rows per rank
  (activation memory / tp); the norm / embedding gradients are then summed once per step by
  :func:`tp_sync_replicated_grads`;
* embeddings and the LM head stay replicated (vocab-parallel CE is a further step; a 128k x 4096
  table is 1 GB, small against 288 GB).

    tp_group = dist.new_group([...])
    model = tensor_parallel_llama(full_llama, tp_group)        # shards the weights in place
    logits = model(idx)                                         # identical to the full model
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.distributed as dist
import torch.nn as tnn

from .. import ops


# ------------------------------------------------------------------ communication autograd functions
class _CopyToTP(torch.autograd.Function):
    """Identity forward; all-reduce of the gradient backward (input of a column-parallel layer)."""

    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        return x

    @staticmethod
    def backward(ctx, g):
        g = g.contiguous()
        dist.all_reduce(g, group=ctx.group)
        return g, None


class _ReduceFromTP(torch.autograd.Function):
    """All-reduce forward (output of a row-parallel layer); identity backward."""

    @staticmethod
    def forward(ctx, x, group):
        x = x.contiguous()
        dist.all_reduce(x, group=group)
        return x

    @staticmethod
    def backward(ctx, g):
        return g, None


class _GatherSeq(torch.autograd.Function):
    """Sequence parallel: all-gather over dim 1 forward, reduce-scatter backward."""

    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        tp = dist.get_world_size(group)
        parts = [torch.empty_like(x) for _ in range(tp)]
        dist.all_gather(parts, x.contiguous(), group=group)
        return torch.cat(parts, 1)

    @staticmethod
    def backward(ctx, g):
        return _reduce_scatter_seq(g, ctx.group), None


class _ScatterSeq(torch.autograd.Function):
    """Sequence parallel: reduce-scatter over dim 1 forward, all-gather backward."""

    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        return _reduce_scatter_seq(x, group)

    @staticmethod
    def backward(ctx, g):
        tp = dist.get_world_size(ctx.group)
        parts = [torch.empty_like(g) for _ in range(tp)]
        dist.all_gather(parts, g.contiguous(), group=ctx.group)
        return torch.cat(parts, 1), None


def _reduce_scatter_seq(x, group):
    tp = dist.get_world_size(group)
    chunks = [c.contiguous() for c in x.chunk(tp, 1)]
    out = torch.empty_like(chunks[0])
    if x.is_cuda and dist.get_backend(group) == "nccl":
        dist.reduce_scatter(out, chunks, group=group)
    else:  # gloo has no reduce_scatter: all-reduce then keep the own chunk
        full = x.contiguous().clone()
        dist.all_reduce(full, group=group)
        out.copy_(full.chunk(tp, 1)[dist.get_rank(group)])
    return out


def copy_to_tp(x, group):
    return _CopyToTP.apply(x, group)


def reduce_from_tp(x, group):
    return _ReduceFromTP.apply(x, group)


def gather_seq(x, group):
    return _GatherSeq.apply(x, group)


def scatter_seq(x, group):
    return _ScatterSeq.apply(x, group)


# ------------------------------------------------------------------ generic layers
class ColumnParallelLinear(tnn.Module):
    """``y_local = x W_r^T`` with W split along the output rows.  ``weight`` given = this rank's rows."""

    def __init__(self, weight: torch.Tensor, bias: Optional[torch.Tensor], group, sequence_parallel=False):
        super().__init__()
        self.weight = tnn.Parameter(weight.detach().clone())
        self.bias = tnn.Parameter(bias.detach().clone()) if bias is not None else None
        self.group, self.sp = group, sequence_parallel

    def forward(self, x):
        x = gather_seq(x, self.group) if self.sp else copy_to_tp(x, self.group)
        return ops.linear(x, self.weight, self.bias)


class RowParallelLinear(tnn.Module):
    """``y = sum_r x_r W_r^T`` with W split along the input columns (bias added once, after the sum)."""

    def __init__(self, weight: torch.Tensor, bias: Optional[torch.Tensor], group, sequence_parallel=False):
        super().__init__()
        self.weight = tnn.Parameter(weight.detach().clone())
        self.bias = tnn.Parameter(bias.detach().clone()) if bias is not None else None
        self.group, self.sp = group, sequence_parallel

    def forward(self, x):
        y = ops.linear(x, self.weight)
        y = scatter_seq(y, self.group) if self.sp else reduce_from_tp(y, self.group)
        return y + self.bias if self.bias is not None else y


def _local(mod, x):
    """This rank's part of a TP projection without its collective (serving); int8-quantised projections
    (``ops.quantize_linears`` replaces the TP layers by ``Int8Linear``) run their own kernel."""
    if isinstance(mod, (ColumnParallelLinear, RowParallelLinear)):
        return ops.linear(x, mod.weight, mod.bias if isinstance(mod, ColumnParallelLinear) else None)
    return mod(x)


def _rows(w: torch.Tensor, lo: int, hi: int) -> torch.Tensor:
    return w[lo:hi]


# ------------------------------------------------------------------ Llama
class TPLlamaBlock(tnn.Module):
    """One Llama block's shard: local heads / FFN columns, two all-reduces per direction."""

    def __init__(self, blk, tp: int, rank: int, group, sequence_parallel: bool = False):
        super().__init__()
        c = blk.cfg
        if c.n_heads % tp or c.n_kv_heads % tp or c.ffn_dim % tp:
            raise ValueError(f"tp={tp} must divide heads ({c.n_heads}/{c.n_kv_heads}) and ffn_dim ({c.ffn_dim})")
        self.cfg, self.group, self.sp = c, group, sequence_parallel
        hd = c.head_dim
        self.hq, self.hkv, self.hd = c.n_heads // tp, c.n_kv_heads // tp, hd
        w = blk.wqkv.weight
        q = _rows(w, rank * self.hq * hd, (rank + 1) * self.hq * hd)
        k0 = c.n_heads * hd
        k = _rows(w, k0 + rank * self.hkv * hd, k0 + (rank + 1) * self.hkv * hd)
        v0 = k0 + c.n_kv_heads * hd
        v = _rows(w, v0 + rank * self.hkv * hd, v0 + (rank + 1) * self.hkv * hd)
        self.attention_norm = blk.attention_norm
        self.ffn_norm = blk.ffn_norm
        self.wqkv = ColumnParallelLinear(torch.cat([q, k, v], 0), None, group, sequence_parallel)
        self.wo = RowParallelLinear(blk.wo.weight[:, rank * self.hq * hd:(rank + 1) * self.hq * hd], None, group,
                                    sequence_parallel)
        f = c.ffn_dim // tp
        w13 = blk.w13.weight
        gate = _rows(w13, rank * f, (rank + 1) * f)
        up = _rows(w13, c.ffn_dim + rank * f, c.ffn_dim + (rank + 1) * f)
        self.w13 = ColumnParallelLinear(torch.cat([gate, up], 0), None, group, sequence_parallel)
        self.w2 = RowParallelLinear(blk.w2.weight[:, rank * f:(rank + 1) * f], None, group, sequence_parallel)

    def forward(self, x, rope, res=None, pending: bool = False):
        # x: [B, T, d] replicated (or [B, T/tp, d] with sequence parallelism); pending-residual
        # convention of LlamaBlock.forward (residual adds fused into the RMSNorms)
        an, fn = self.attention_norm, self.ffn_norm
        h, n = ops.add_norm_train(x, res, an.weight, eps=an.eps)
        a_in = self.wqkv(n)
        B, T = a_in.shape[:2]
        qkv = a_in.view(B, T, self.hq + 2 * self.hkv, self.hd)
        a = ops.attention_qkv(qkv, self.hq, self.hkv, causal=True, rope=rope)
        h, n = ops.add_norm_train(h, self.wo(a.reshape(B, T, self.hq * self.hd)), fn.weight, eps=fn.eps)
        y = self.w2(ops.swiglu(self.w13(n)))
        return (h, y) if pending else h + y

    @torch.no_grad()
    def forward_cached(self, x, k_cache, v_cache, pos, rope, res=None):
        """Serving step (pending-residual convention of LlamaBlock.forward_cached)."""
        B, T, _ = x.shape
        if res is None:
            h, n = x, self.attention_norm(x)
        else:
            h, n = ops.add_norm(x, res, self.attention_norm.weight, eps=self.attention_norm.eps)
        qkv = _local(self.wqkv, n).view(B, T, self.hq + 2 * self.hkv, self.hd)
        a = ops.attention_cached(qkv, self.hq, self.hkv, k_cache, v_cache, pos, rope)
        o = _local(self.wo, a.reshape(B, T, self.hq * self.hd))
        dist.all_reduce(o, group=self.group)
        h, n = ops.add_norm(h, o, self.ffn_norm.weight, eps=self.ffn_norm.eps)
        y = _local(self.w2, ops.swiglu(_local(self.w13, n)))
        dist.all_reduce(y, group=self.group)
        return h, y


def tensor_parallel_llama(model, group=None, sequence_parallel: bool = False):
    """Replace every block of ``model`` (a :class:`~..models.llama.Llama`) by its TP shard for this
    rank of ``group``.  Every rank must pass the same full weights (same seed or a broadcast); the
    result computes exactly the full model.  ``kv_shape()`` then reports the local KV heads, so
    :class:`~..serving.KVCache` allocates 1/tp of the cache per rank.  With ``sequence_parallel``
    the caller feeds the block stack a sequence shard (see :func:`scatter_seq`)."""
    tp = dist.get_world_size(group)
    rank = dist.get_rank(group)
    model.layers = tnn.ModuleList([TPLlamaBlock(b, tp, rank, group, sequence_parallel) for b in model.layers])
    model.tp_group, model.tp, model.tp_sp = group, tp, sequence_parallel
    cfg = model.cfg
    model.kv_shape = lambda: (cfg.n_layers, cfg.n_kv_heads // tp, cfg.head_dim)
    if sequence_parallel:
        model.forward = _sp_forward.__get__(model)
    return model


def tp_sync_replicated_grads(model):
    """Sequence parallelism only: parameters replicated over the TP group but applied to a sequence
    shard (RMSNorm weights inside the blocks, the token embedding) hold partial gradients — sum them
    over the group (one flat all-reduce).  Without sequence parallelism every rank already holds the
    full gradient of those parameters."""
    if not getattr(model, "tp_sp", False):
        return
    ps = [model.tok_embeddings] + [p for blk in model.layers for p in (blk.attention_norm.weight, blk.ffn_norm.weight)]
    gs = [p.grad for p in ps if p.grad is not None]
    if not gs:
        return
    flat = torch.cat([g.reshape(-1).float() for g in gs])
    dist.all_reduce(flat, group=model.tp_group)
    off = 0
    for g in gs:
        g.copy_(flat[off: off + g.numel()].view_as(g))
        off += g.numel()


def _sp_forward(self, idx, targets=None):
    """Sequence-parallel Llama forward: embedding replicated, blocks on T/tp rows, gathered before the head."""
    T = idx.shape[1]
    rope = self.rope(T, idx.device)
    x = ops.embedding(idx, self.tok_embeddings)
    tp, r = self.tp, dist.get_rank(self.tp_group)
    x = x.chunk(tp, 1)[r].contiguous()
    for blk in self.layers:
        x = blk(x, rope)
    x = _GatherSeqNoReduce.apply(x, self.tp_group)
    logits = self.output(self.norm(x))
    if targets is None:
        return logits
    return ops.cross_entropy(logits.reshape(-1, logits.shape[-1]), targets.reshape(-1))


class _GatherSeqNoReduce(torch.autograd.Function):
    """All-gather of the sequence shards before the replicated head; backward keeps the own rows
    (every rank computes the same head gradient for all rows, so no reduction is needed)."""

    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        tp = dist.get_world_size(group)
        parts = [torch.empty_like(x) for _ in range(tp)]
        dist.all_gather(parts, x.contiguous(), group=group)
        return torch.cat(parts, 1)

    @staticmethod
    def backward(ctx, g):
        tp = dist.get_world_size(ctx.group)
        return g.chunk(tp, 1)[dist.get_rank(ctx.group)].contiguous(), None
