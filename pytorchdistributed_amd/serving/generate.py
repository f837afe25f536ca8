"""KV cache, layer placement and the generation loop.

MI355X-first choices:
* the KV cache is preallocated once per layer as ``[B, max_len, Hkv, D]`` bf16 on the layer's GPU —
  288 GB of HBM3E holds e.g. Llama-3-8B weights (16 GB) plus a 128-sequence x 8192-token cache
  (128 GiB) on ONE device, so placement over several GPUs is only needed for bigger models;
* prefill runs the training flash-attention kernel over the prompt and writes the rotated K/V rows
  straight into the cache (the RoPE kernel's output is the cache slice, no extra copy of K);
* each decode step is one new token per sequence: the split-sequence decode kernel
  (`csrc/kernels/decode_attn.hip`) streams K/V once for all query heads of a KV group;
* placement (``place``) follows accelerate's ``device_map="auto"`` semantics: layers fill GPUs in
  order up to a byte budget (then CPU); the hidden state follows the layers during the forward.
  Peer copies between layers ride xGMI.

Static batching: every sequence of a batch has the same prompt length (synthetic serving benches and
the reference's single-prompt use).  Sampling: greedy (``temperature=0``) or temperature + top-k.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence

import torch
import torch.nn as tnn


def _dev(d) -> torch.device:
    if isinstance(d, int):
        return torch.device("cuda", d)
    return torch.device(d)


class KVCache:
    """Per-layer K/V buffers ``[B, max_len, Hkv, D]`` on each layer's device."""

    def __init__(self, model: tnn.Module, batch: int, max_len: int, dtype: Optional[torch.dtype] = None):
        n_layers, hkv, hd = model.kv_shape()
        self.batch, self.max_len = batch, max_len
        self.k: List[torch.Tensor] = []
        self.v: List[torch.Tensor] = []
        for blk in model.layers:
            w = next(blk.parameters())
            dt = dtype or w.dtype
            self.k.append(torch.zeros(batch, max_len, hkv, hd, device=w.device, dtype=dt))
            self.v.append(torch.zeros(batch, max_len, hkv, hd, device=w.device, dtype=dt))
        self.pos = 0

    def nbytes(self) -> int:
        return sum(t.numel() * t.element_size() for t in self.k + self.v)

    @staticmethod
    def bytes_per_token(model: tnn.Module, dtype=torch.bfloat16) -> int:
        n_layers, hkv, hd = model.kv_shape()
        return 2 * n_layers * hkv * hd * torch.empty((), dtype=dtype).element_size()


def _sample(logits: torch.Tensor, temperature: float, top_k: Optional[int], gen: Optional[torch.Generator]):
    logits = logits[:, -1].float()
    if temperature <= 0:
        return logits.argmax(-1, keepdim=True)
    logits = logits / temperature
    if top_k is not None and top_k < logits.shape[-1]:
        kth = torch.topk(logits, top_k, dim=-1).values[:, -1:]
        logits = logits.masked_fill(logits < kth, float("-inf"))
    probs = torch.softmax(logits, -1)
    return torch.multinomial(probs, 1, generator=gen)


class _GraphedDecode:
    """One decode step (embedding -> all blocks -> head) captured in a HIP graph.  The token and the
    position live in static device buffers; the append / attention kernels read the position at run
    time, so replaying the graph after ``tok.copy_(next); pos += 1`` is a real next step."""

    def __init__(self, model, cache: KVCache, pos0: int):
        dev = next(model.parameters()).device
        self.tok = torch.zeros(cache.batch, 1, dtype=torch.long, device=dev)
        self.pos = torch.full((1,), pos0, dtype=torch.int32, device=dev)
        side = torch.cuda.Stream(dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):  # warm-up outside capture (plans, rope tables); row pos0 is rewritten later
            model.forward_cached(self.tok, cache, self.pos)
        torch.cuda.current_stream(dev).wait_stream(side)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self.logits = model.forward_cached(self.tok, cache, self.pos)

    def __call__(self, tok):
        self.tok.copy_(tok)
        self.graph.replay()
        self.pos += 1
        return self.logits


def _single_device(model) -> bool:
    devs = {p.device for p in model.parameters()}
    return len(devs) == 1 and next(iter(devs)).type == "cuda"


@torch.no_grad()
def generate(model: tnn.Module, prompt: torch.Tensor, max_new_tokens: int, temperature: float = 0.0,
             top_k: Optional[int] = None, eos_token: Optional[int] = None, cache: Optional[KVCache] = None,
             generator: Optional[torch.Generator] = None, return_logits: bool = False, graph: bool = False):
    """Autoregressive generation: ``prompt`` [B, T0] token ids -> [B, T0 + max_new_tokens].

    One prefill over the prompt, then ``max_new_tokens - 1`` single-token decode steps over the KV cache.
    With ``eos_token``, finished sequences keep emitting ``eos_token`` (static batch shape).  With
    ``return_logits`` the per-step last-position logits are returned too (tests compare them with the
    uncached forward).  ``graph=True`` (one-GPU bf16 models) replays every decode step from one HIP
    graph: no per-kernel launch cost, the step is bound by HBM traffic only."""
    B, T0 = prompt.shape
    if cache is None:
        cache = KVCache(model, B, T0 + max_new_tokens)
    out_dev = prompt.device
    logits = model.forward_cached(prompt, cache, 0)
    cache.pos = T0
    seq = [prompt]
    all_logits = [logits[:, -1].float().to(out_dev)] if return_logits else None
    done = torch.zeros(B, 1, dtype=torch.bool, device=out_dev)
    step = None
    if graph and max_new_tokens > 1 and _single_device(model):
        step = _GraphedDecode(model, cache, T0)
    for i in range(max_new_tokens):
        nxt = _sample(logits, temperature, top_k, generator).to(out_dev)
        if eos_token is not None:
            nxt = torch.where(done, torch.full_like(nxt, eos_token), nxt)
            done = done | (nxt == eos_token)
        seq.append(nxt)
        if i == max_new_tokens - 1:
            break
        logits = step(nxt) if step is not None else model.forward_cached(nxt, cache, cache.pos)
        cache.pos += 1
        if return_logits:
            all_logits.append(logits[:, -1].float().to(out_dev))
    tokens = torch.cat(seq, 1)
    return (tokens, torch.stack(all_logits, 1)) if return_logits else tokens


def place(model: tnn.Module, max_memory: Optional[Dict] = None, devices: Optional[Sequence] = None,
          kv_tokens: int = 0) -> Dict[str, torch.device]:
    """Budget-driven placement of a Llama / GPT-2 for inference (``device_map="auto"`` semantics):
    embeddings on the first device, transformer blocks fill each device up to its byte budget
    (weights + ``kv_tokens`` tokens of KV cache per block), the final norm / head go with the last
    block (GPT-2's tied head stays with the embedding).  Returns the device map {module name: device}.
    Default budget: 90 % of each visible GPU's free memory, then CPU."""
    if devices is None:
        devices = list(range(torch.cuda.device_count())) + ["cpu"]
    devs = [_dev(d) for d in devices]
    if max_memory is None:
        max_memory = {}
        for d in devs:
            max_memory[d] = int(torch.cuda.mem_get_info(d)[0] * 0.9) if d.type == "cuda" else 1 << 62
    budget = {_dev(k): v for k, v in max_memory.items()}
    n_layers, hkv, hd = model.kv_shape()

    def size(m):
        return sum(p.numel() * p.element_size() for p in m.parameters()) + sum(
            b.numel() * b.element_size() for b in m.buffers())

    dmap: Dict[str, torch.device] = {}
    di, used = 0, 0
    emb_names = [n for n in ("tok_embeddings", "wte", "wpe") if hasattr(model, n)]
    for n in emb_names:
        p = getattr(model, n)
        used += p.numel() * p.element_size()
        dmap[n] = devs[0]
    elt = next(model.parameters()).element_size()
    for i, blk in enumerate(model.layers):
        need = size(blk) + 2 * kv_tokens * hkv * hd * elt
        while di < len(devs) - 1 and used + need > budget.get(devs[di], 0):
            di, used = di + 1, 0
        dmap[f"layers.{i}"] = devs[di]
        used += need
    last = devs[di]
    for n in ("norm", "output", "ln_f"):
        if hasattr(model, n):
            dmap[n] = last
    if hasattr(model, "wte"):
        dmap["ln_f"] = devs[0]  # GPT-2: final LN + tied head run next to the embedding table
    # move
    with torch.no_grad():
        for n in emb_names:
            p = getattr(model, n)
            p.data = p.data.to(dmap[n])
        for i, blk in enumerate(model.layers):
            blk.to(dmap[f"layers.{i}"])
        for n in ("norm", "output", "ln_f"):
            if hasattr(model, n):
                getattr(model, n).to(dmap[n])
    if hasattr(model, "_rope_cache"):
        model._rope_cache.clear()
    return dmap
