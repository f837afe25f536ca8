"""GPT-2 (BASELINE configs 3 — GPT-2-medium DDP — and 5 — GPT-2-XL PP4 x DP2), on the native layers.

Architecture as OpenAI GPT-2: learned token + position embeddings, pre-LN blocks (LN -> fused QKV ->
causal attention -> proj; LN -> 4x MLP with tanh-GELU), final LN, LM head tied to the token embedding.
MI355X-specific choices: the vocabulary table is padded to a multiple of 64 rows (50257 -> 50304) so the
LM-head GEMMs tile cleanly, and the padded logits are excluded from the softmax by the cross-entropy
kernel (``num_valid_classes``), so the loss equals the unpadded model's; attention consumes the fused
QKV output in place.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, replace
from typing import List, Optional

import torch
import torch.nn as tnn

from .. import nn as pnn
from .. import ops


@dataclass
class GPT2Config:
    vocab_size: int = 50257
    n_positions: int = 1024
    n_embd: int = 1024
    n_layer: int = 24
    n_head: int = 16
    layer_norm_eps: float = 1e-5
    pad_vocab_multiple: int = 64

    @property
    def padded_vocab(self) -> int:
        m = self.pad_vocab_multiple
        return (self.vocab_size + m - 1) // m * m


PRESETS = {
    "gpt2": GPT2Config(n_embd=768, n_layer=12, n_head=12),
    "gpt2-medium": GPT2Config(n_embd=1024, n_layer=24, n_head=16),
    "gpt2-large": GPT2Config(n_embd=1280, n_layer=36, n_head=20),
    "gpt2-xl": GPT2Config(n_embd=1600, n_layer=48, n_head=25),
}


def config(name: str, **overrides) -> GPT2Config:
    return replace(PRESETS[name], **overrides)


class GPT2Block(tnn.Module):
    def __init__(self, cfg: GPT2Config, device=None, dtype=None):
        super().__init__()
        d, kw = cfg.n_embd, dict(device=device, dtype=dtype)
        self.n_head = cfg.n_head
        self.ln_1 = pnn.LayerNorm(d, cfg.layer_norm_eps, **kw)
        self.c_attn = pnn.Linear(d, 3 * d, **kw)
        self.attn_proj = pnn.Linear(d, d, **kw)
        self.ln_2 = pnn.LayerNorm(d, cfg.layer_norm_eps, **kw)
        self.c_fc = pnn.Linear(d, 4 * d, **kw)
        self.mlp_proj = pnn.Linear(4 * d, d, **kw)

    def forward(self, x, res=None, pending: bool = False):
        """``pending=False``: the block output.  ``pending=True``: the residual stream is carried as a
        pair — the input is ``x + res`` (``res=None``: just ``x``) and the block returns ``(h, y)`` whose
        sum is its output, so each residual add runs inside the next LayerNorm, forward and backward
        (:func:`ops.add_norm_train`)."""
        B, T, d = x.shape
        h, n = ops.add_norm_train(x, res, self.ln_1.weight, self.ln_1.bias, self.ln_1.eps, rms=False)
        qkv = self.c_attn(n).view(B, T, 3 * self.n_head, d // self.n_head)
        a = ops.attention_qkv(qkv, self.n_head, self.n_head, causal=True)
        h, n = ops.add_norm_train(h, self.attn_proj(a.reshape(B, T, d)), self.ln_2.weight, self.ln_2.bias,
                                  self.ln_2.eps, rms=False)
        y = ops.mlp_gelu(n, self.c_fc.weight, self.c_fc.bias, self.mlp_proj.weight, self.mlp_proj.bias)
        return (h, y) if pending else h + y

    @torch.no_grad()
    def forward_cached(self, x, k_cache, v_cache, pos, res=None):
        """Serving step; pending-residual convention of LlamaBlock.forward_cached (input x + res,
        returns (h, y) with output h + y) so each residual add is fused into the next LayerNorm."""
        B, T, d = x.shape
        ln1, ln2 = self.ln_1, self.ln_2
        if res is None:
            h, n = x, ln1(x)
        else:
            h, n = ops.add_norm(x, res, ln1.weight, ln1.bias, eps=ln1.eps, rms=False)
        qkv = self.c_attn(n).view(B, T, 3 * self.n_head, d // self.n_head)
        a = ops.attention_cached(qkv, self.n_head, self.n_head, k_cache, v_cache, pos)
        h, n = ops.add_norm(h, self.attn_proj(a.reshape(B, T, d)), ln2.weight, ln2.bias, eps=ln2.eps, rms=False)
        return h, self.mlp_proj(ops.gelu_tanh(self.c_fc(n)))


class GPT2(tnn.Module):
    def __init__(self, cfg: GPT2Config, device=None, dtype=None):
        super().__init__()
        self.cfg = cfg
        kw = dict(device=device, dtype=dtype)
        self.wte = tnn.Parameter(torch.empty(cfg.padded_vocab, cfg.n_embd, **kw))
        self.wpe = tnn.Parameter(torch.empty(cfg.n_positions, cfg.n_embd, **kw))
        self.h = tnn.ModuleList([GPT2Block(cfg, **kw) for _ in range(cfg.n_layer)])
        self.ln_f = pnn.LayerNorm(cfg.n_embd, cfg.layer_norm_eps, **kw)
        self.reset_parameters()

    @torch.no_grad()
    def reset_parameters(self):
        std = 0.02
        self.wte.normal_(0, std)
        self.wpe.normal_(0, std / 2)
        for blk in self.h:
            for lin in (blk.c_attn, blk.c_fc):
                lin.weight.normal_(0, std)
                lin.bias.zero_()
            for lin in (blk.attn_proj, blk.mlp_proj):  # residual projections, GPT-2 scaling
                lin.weight.normal_(0, std / math.sqrt(2 * self.cfg.n_layer))
                lin.bias.zero_()

    def embed(self, idx):
        T = idx.shape[1]
        pos = torch.arange(T, device=idx.device)
        return ops.embedding(idx, self.wte) + ops.embedding(pos, self.wpe).unsqueeze(0)

    def head(self, x, targets=None, res=None):
        """LN_f (fused with a pending residual ``res``) + tied LM head (+ loss)."""
        _, n = ops.add_norm_train(x, res, self.ln_f.weight, self.ln_f.bias, self.ln_f.eps, rms=False)
        logits = ops.linear(n, self.wte)
        if targets is None:
            return logits[..., : self.cfg.vocab_size]
        return ops.cross_entropy(logits.reshape(-1, logits.shape[-1]), targets.reshape(-1),
                                 num_valid_classes=self.cfg.vocab_size)

    def forward(self, idx, targets=None):
        x, res = self.embed(idx), None
        for blk in self.h:
            x, res = blk(x, res, pending=True)
        return self.head(x, targets, res)

    # ---------------------------------------------------------------- serving (serving/generate.py)
    def kv_shape(self):
        return self.cfg.n_layer, self.cfg.n_head, self.cfg.n_embd // self.cfg.n_head

    @property
    def layers(self):
        return self.h

    @torch.no_grad()
    def forward_cached(self, idx, cache, pos: int, last_only: bool = True):
        """Logits for tokens ``idx`` [B, T] at positions pos..pos+T-1 over ``cache`` (see Llama)."""
        dev0 = self.wte.device
        idx = idx.to(dev0)
        T = idx.shape[1]
        if isinstance(pos, torch.Tensor):  # device position (graph-replayed decode step)
            positions = pos.to(dev0, torch.long).view(1)
        else:
            positions = torch.arange(pos, pos + T, device=dev0)
        x = ops.embedding(idx, self.wte) + ops.embedding(positions, self.wpe).unsqueeze(0)
        res = None
        for i, blk in enumerate(self.h):
            dev = blk.ln_1.weight.device  # (c_attn may be an Int8Linear)
            x = x.to(dev, non_blocking=True)
            res = res.to(dev, non_blocking=True) if res is not None else None
            x, res = blk.forward_cached(x, cache.k[i], cache.v[i], pos, res)
        if last_only:
            x, res = x[:, -1:], res[:, -1:]
        # tied head: LM projection with the embedding table (final LN fused with the last residual add)
        _, n = ops.add_norm(x.to(dev0, non_blocking=True), res.to(dev0, non_blocking=True), self.ln_f.weight,
                            self.ln_f.bias, eps=self.ln_f.eps, rms=False)
        return ops.linear(n, self.wte)[..., : self.cfg.vocab_size]

    def num_params(self, exclude_padding=True) -> int:
        n = sum(p.numel() for p in self.parameters())
        if exclude_padding:
            n -= (self.cfg.padded_vocab - self.cfg.vocab_size) * self.cfg.n_embd
        return n


class GPT2Stage(tnn.Module):
    """Blocks [lo, hi) of a GPT-2, plus the embedding on the first stage and LN_f + LM head + loss on
    the last (pipeline parallel, BASELINE config 5).  The last stage's forward takes (x, targets)."""

    def __init__(self, cfg: GPT2Config, lo: int, hi: int, first: bool, last: bool, device=None, dtype=None):
        super().__init__()
        self.cfg, self.first, self.last = cfg, first, last
        kw = dict(device=device, dtype=dtype)
        if first:
            self.wte = tnn.Parameter(torch.empty(cfg.padded_vocab, cfg.n_embd, **kw).normal_(0, 0.02))
            self.wpe = tnn.Parameter(torch.empty(cfg.n_positions, cfg.n_embd, **kw).normal_(0, 0.01))
        self.h = tnn.ModuleList([GPT2Block(cfg, **kw) for _ in range(lo, hi)])
        if last:
            self.ln_f = pnn.LayerNorm(cfg.n_embd, cfg.layer_norm_eps, **kw)
            # untied head on the last stage (the embedding lives on stage 0)
            self.lm_head = tnn.Parameter(torch.empty(cfg.padded_vocab, cfg.n_embd, **kw).normal_(0, 0.02))

    def forward(self, x):
        if self.first:
            T = x.shape[1]
            x = ops.embedding(x, self.wte) + ops.embedding(torch.arange(T, device=x.device), self.wpe).unsqueeze(0)
        res = None
        for blk in self.h:
            x, res = blk(x, res, pending=True)
        if self.last:
            _, n = ops.add_norm_train(x, res, self.ln_f.weight, self.ln_f.bias, self.ln_f.eps, rms=False)
            return ops.linear(n, self.lm_head)
        return x + res if res is not None else x

    def loss(self, logits, targets):
        return ops.cross_entropy(logits.reshape(-1, logits.shape[-1]), targets.reshape(-1),
                                 num_valid_classes=self.cfg.vocab_size)


def gpt2(name: str = "gpt2-medium", device=None, dtype=None, **overrides) -> GPT2:
    return GPT2(config(name, **overrides), device=device, dtype=dtype)
