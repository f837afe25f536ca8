"""Llama-3 (BASELINE config 4 — Llama-3 8B FSDP full-shard on 8 x MI355X; the reference's
``LlamaForCausalLM`` load at `03_model_parallel.ipynb` raw lines 85-89), on the native layers.

Llama-3-8B: d 4096, 32 layers, 32 query / 8 KV heads (GQA) of 128, SwiGLU FFN 14336, RMSNorm
(eps 1e-5), RoPE theta 500000, vocab 128256, untied output head.  MI355X choices: Q, K, V are one fused
projection (one GEMM, consumed in place by attention), gate/up are one fused projection feeding the
SwiGLU kernel, and RoPE is applied inside the attention kernels (no rotary pass over HBM).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, replace

import torch
import torch.nn as tnn

from .. import nn as pnn
from .. import ops


@dataclass
class LlamaConfig:
    vocab_size: int = 128256
    dim: int = 4096
    n_layers: int = 32
    n_heads: int = 32
    n_kv_heads: int = 8
    ffn_dim: int = 14336
    norm_eps: float = 1e-5
    rope_theta: float = 500000.0
    max_seq_len: int = 8192

    @property
    def head_dim(self) -> int:
        return self.dim // self.n_heads


PRESETS = {
    "llama3-8b": LlamaConfig(),
    "llama3-70b": LlamaConfig(dim=8192, n_layers=80, n_heads=64, n_kv_heads=8, ffn_dim=28672),
    "llama3-tiny": LlamaConfig(vocab_size=1024, dim=256, n_layers=2, n_heads=2, n_kv_heads=1, ffn_dim=512,
                               max_seq_len=512),
}


def config(name: str, **overrides) -> LlamaConfig:
    return replace(PRESETS[name], **overrides)


class LlamaBlock(tnn.Module):
    def __init__(self, cfg: LlamaConfig, device=None, dtype=None):
        super().__init__()
        kw = dict(device=device, dtype=dtype)
        self.cfg = cfg
        hd = cfg.head_dim
        self.attention_norm = pnn.RMSNorm(cfg.dim, cfg.norm_eps, **kw)
        self.wqkv = pnn.Linear(cfg.dim, (cfg.n_heads + 2 * cfg.n_kv_heads) * hd, bias=False, **kw)
        self.wo = pnn.Linear(cfg.n_heads * hd, cfg.dim, bias=False, **kw)
        self.ffn_norm = pnn.RMSNorm(cfg.dim, cfg.norm_eps, **kw)
        self.w13 = pnn.Linear(cfg.dim, 2 * cfg.ffn_dim, bias=False, **kw)  # gate | up
        self.w2 = pnn.Linear(cfg.ffn_dim, cfg.dim, bias=False, **kw)

    def forward(self, x, rope, res=None, pending: bool = False):
        """``pending=True``: input ``x + res``, output the pair ``(h, y)`` (see GPT2Block.forward) — the
        residual adds run inside the RMSNorms (:func:`ops.add_norm_train`)."""
        B, T, d = x.shape
        c = self.cfg
        an, fn = self.attention_norm, self.ffn_norm
        h, n = ops.add_norm_train(x, res, an.weight, eps=an.eps)
        qkv = self.wqkv(n).view(B, T, c.n_heads + 2 * c.n_kv_heads, c.head_dim)
        a = ops.attention_qkv(qkv, c.n_heads, c.n_kv_heads, causal=True, rope=rope)
        h, n = ops.add_norm_train(h, self.wo(a.reshape(B, T, d)), fn.weight, eps=fn.eps)
        y = self.w2(ops.swiglu(self.w13(n)))
        return (h, y) if pending else h + y

    @torch.no_grad()
    def forward_cached(self, x, k_cache, v_cache, pos, rope, res=None):
        """Inference step over a KV cache (prefill at pos 0 or one decode token; see
        ops.attention_cached).  The residual stream is carried as a pending pair: the block's input
        is ``x + res`` and it returns ``(h, y)`` whose sum is its output, so every residual add is
        fused into the following norm (one pass, `add_rownorm_fwd_kernel`)."""
        B, T, d = x.shape
        c = self.cfg
        if res is None:
            h, n = x, self.attention_norm(x)
        else:
            h, n = ops.add_norm(x, res, self.attention_norm.weight, eps=self.attention_norm.eps)
        qkv = self.wqkv(n).view(B, T, c.n_heads + 2 * c.n_kv_heads, c.head_dim)
        a = ops.attention_cached(qkv, c.n_heads, c.n_kv_heads, k_cache, v_cache, pos, rope)
        h, n = ops.add_norm(h, self.wo(a.reshape(B, T, d)), self.ffn_norm.weight, eps=self.ffn_norm.eps)
        return h, self.w2(ops.swiglu(self.w13(n)))


class Llama(tnn.Module):
    def __init__(self, cfg: LlamaConfig, device=None, dtype=None, seed=None):
        """``device="meta"``: no storage is allocated — FSDP then builds each unit directly as a shard
        (:meth:`init_unit` fills one unit at a time, parallel/fsdp.py).  ``seed``: base of the per-unit
        initialisation streams (default: drawn from the global RNG, so ``torch.manual_seed`` fixes it)."""
        super().__init__()
        self.cfg = cfg
        kw = dict(device=device, dtype=dtype)
        self.init_seed = int(torch.randint(0, 2 ** 31 - 1, (1,)).item()) if seed is None else int(seed)
        self.tok_embeddings = tnn.Parameter(torch.empty(cfg.vocab_size, cfg.dim, **kw))
        self.layers = tnn.ModuleList([LlamaBlock(cfg, **kw) for _ in range(cfg.n_layers)])
        self.norm = pnn.RMSNorm(cfg.dim, cfg.norm_eps, **kw)
        self.output = pnn.Linear(cfg.dim, cfg.vocab_size, bias=False, **kw)
        self._rope_cache = {}
        self.reset_parameters()

    @torch.no_grad()
    def reset_parameters(self):
        if self.tok_embeddings.is_meta:
            return
        for i, blk in enumerate(self.layers):
            self.init_unit(blk, i)
        self.init_unit(self, len(self.layers))

    @torch.no_grad()
    def init_unit(self, module: tnn.Module, index: int):
        """Initialise one FSDP unit's parameters — block ``index``, or (``module`` is the model, index =
        n_layers) the embedding, final norm and head — from its own generator seeded by (init_seed, index).
        Eager construction and FSDP's deferred one run exactly this, unit by unit, so they produce the same
        bits (test_fsdp_cpu.py::test_fsdp_deferred_init_matches_eager)."""
        std = 0.02
        std_out = std / math.sqrt(2 * self.cfg.n_layers)

        def gen(t):
            g = torch.Generator(device=t.device)
            g.manual_seed(self.init_seed * 1000003 + index)
            return g

        if isinstance(module, LlamaBlock):
            g = gen(module.wqkv.weight)
            module.attention_norm.weight.fill_(1.0)
            module.wqkv.weight.normal_(0, std, generator=g)
            module.wo.weight.normal_(0, std_out, generator=g)
            module.ffn_norm.weight.fill_(1.0)
            module.w13.weight.normal_(0, std, generator=g)
            module.w2.weight.normal_(0, std_out, generator=g)
        else:
            g = gen(self.tok_embeddings)
            self.tok_embeddings.normal_(0, std, generator=g)
            self.norm.weight.fill_(1.0)
            self.output.weight.normal_(0, std, generator=g)

    def rope(self, T: int, device):
        key = (T, str(device))
        if key not in self._rope_cache:
            self._rope_cache[key] = ops.rope_tables(T, self.cfg.head_dim, self.cfg.rope_theta, device=device)
        return self._rope_cache[key]

    def forward(self, idx, targets=None):
        T = idx.shape[1]
        rope = self.rope(T, idx.device)
        x, res = ops.embedding(idx, self.tok_embeddings), None
        for blk in self.layers:
            x, res = blk(x, rope, res, pending=True)
        _, n = ops.add_norm_train(x, res, self.norm.weight, eps=self.norm.eps)
        logits = self.output(n)
        if targets is None:
            return logits
        return ops.cross_entropy(logits.reshape(-1, logits.shape[-1]), targets.reshape(-1))

    # ---------------------------------------------------------------- serving (serving/generate.py)
    def kv_shape(self):
        """(n_layers, n_kv_heads, head_dim) of the KV cache this model needs."""
        return self.cfg.n_layers, self.cfg.n_kv_heads, self.cfg.head_dim

    @torch.no_grad()
    def forward_cached(self, idx, cache, pos: int, last_only: bool = True):
        """Logits for tokens ``idx`` [B, T] at positions pos..pos+T-1, reading/extending ``cache``
        (:class:`~pytorchdistributed_amd.serving.KVCache`).  Layers may live on different devices
        (``serving.place``): the hidden state follows them."""
        dev0 = self.tok_embeddings.device
        x, res = ops.embedding(idx.to(dev0), self.tok_embeddings), None
        for i, blk in enumerate(self.layers):
            dev = blk.attention_norm.weight.device  # (wqkv may be an Int8Linear)
            x = x.to(dev, non_blocking=True)
            res = res.to(dev, non_blocking=True) if res is not None else None
            rope = self.rope(cache.max_len, dev)
            x, res = blk.forward_cached(x, cache.k[i], cache.v[i], pos, rope, res)
        if last_only:
            x, res = x[:, -1:], res[:, -1:]
        dev = self.norm.weight.device
        _, n = ops.add_norm(x.to(dev, non_blocking=True), res.to(dev, non_blocking=True), self.norm.weight,
                            eps=self.norm.eps)
        return self.output(n)


def llama(name: str = "llama3-8b", device=None, dtype=None, seed=None, **overrides) -> Llama:
    return Llama(config(name, **overrides), device=device, dtype=dtype, seed=seed)
