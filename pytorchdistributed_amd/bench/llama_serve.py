"""Serving benchmark (the reference's Llama inference): KV-cached generation on one
MI355X, random-init Llama-3 weights, synthetic prompts.  Reports prefill tokens/s, decode tokens/s
(new tokens of the whole batch per second over the decode steps) and per-step latency.

    python -m pytorchdistributed_amd.bench.llama_serve --batch 32 --prompt 1024 --new 128
"""
from __future__ import annotations

import argparse
import json
import time

import torch

from ..models.llama import Llama, config
from ..serving import KVCache, generate


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--prompt", type=int, default=1024)
    ap.add_argument("--new", type=int, default=128)
    ap.add_argument("--repeat", type=int, default=2)
    ap.add_argument("--layers", type=int, default=None, help="override depth (smoke runs only)")
    ap.add_argument("--graph", action="store_true", help="replay each decode step from one HIP graph")
    ap.add_argument("--int8", action="store_true", help="weight-only int8 block projections (w8_gemm kernel)")
    ap.add_argument("--int8-head", action="store_true", help="also quantise the LM head")
    ap.add_argument("--int8-names", default="w13", help="block projections to quantise with --int8 (w13: the measured win; the split-K shapes wqkv/wo/w2 run slower in int8 today)")
    a = ap.parse_args(argv)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    over = {} if a.layers is None else {"n_layers": a.layers}
    torch.manual_seed(0)
    model = Llama(config(a.model, **over), device=dev, dtype=torch.bfloat16).eval()
    if a.int8 or a.int8_head:
        from ..ops import quantize_linears

        quantize_linears(model, names=a.int8_names.split(",") if a.int8 else (), head=a.int8_head)
        torch.cuda.empty_cache()
    prompt = torch.randint(0, model.cfg.vocab_size, (a.batch, a.prompt), device=dev)
    cache = KVCache(model, a.batch, a.prompt + a.new)

    def prefill():
        cache.pos = 0
        model.forward_cached(prompt, cache, 0)

    prefill()  # warm-up: kernels, GEMM plans, rope tables
    generate(model, prompt, 4, cache=cache, graph=a.graph)
    torch.cuda.synchronize()
    pre, tot = [], []
    for _ in range(a.repeat):
        t0 = time.perf_counter()
        prefill()
        torch.cuda.synchronize()
        pre.append(time.perf_counter() - t0)
        t0 = time.perf_counter()
        generate(model, prompt, a.new, cache=cache, graph=a.graph)
        torch.cuda.synchronize()
        tot.append(time.perf_counter() - t0)
    t_pre, t_tot = min(pre), min(tot)
    t_dec = max(t_tot - t_pre, 1e-9)  # graph mode: includes the one-time capture of the decode step
    steps = a.new - 1
    print(json.dumps({
        "metric": "Llama-3 KV-cached generation (1 GPU)", "model": a.model + ("" if a.layers is None else f"-{a.layers}L"),
        "batch": a.batch, "decode_graph": a.graph, "weights": f"int8 (per-row scale): {a.int8_names}" if a.int8 else "bf16",
        "int8_head": a.int8_head, "prompt": a.prompt, "new_tokens": a.new, "dtype": "bf16",
        "data": "synthetic prompts, random-init weights",
        "prefill_ms": round(t_pre * 1e3, 2), "prefill_tokens_per_s": round(a.batch * a.prompt / t_pre, 1),
        "decode_ms_per_step": round(t_dec / steps * 1e3, 3),
        "decode_tokens_per_s": round(a.batch * steps / t_dec, 1),
        "kv_cache_gb": round(cache.nbytes() / 1e9, 2)}), flush=True)


if __name__ == "__main__":
    main()
