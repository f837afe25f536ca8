"""Chapter 03's big-model inference cell (reference `03 模型并行/03_model_parallel.ipynb` raw lines 85-89:
``LlamaForCausalLM.from_pretrained(..., device_map="auto", load_in_8bit=True)`` then generation), done
the MI355X way: random-init Llama-3 weights (no checkpoint download here), budget-driven placement of
the blocks over the visible GPUs (``serving.place`` — one MI355X holds Llama-3-8B plus a large KV cache,
so by default everything lands on GPU 0), a preallocated KV cache, and KV-cached generation with the
split-sequence decode kernel; ``--graph`` replays each decode step from one HIP graph.

    python examples/05_llama_generate.py --model llama3-8b --batch 4 --prompt 128 --new 32 [--graph]
    python examples/05_llama_generate.py --model llama3-tiny --cpu          # CPU reference math
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorchdistributed_amd.models.llama import llama  # noqa: E402
from pytorchdistributed_amd.serving import KVCache, generate, place  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--batch", type=int, default=4)
    ap.add_argument("--prompt", type=int, default=128)
    ap.add_argument("--new", type=int, default=32)
    ap.add_argument("--max-memory-gb", type=float, default=None, help="per-GPU budget (forces multi-GPU placement)")
    ap.add_argument("--graph", action="store_true")
    ap.add_argument("--temperature", type=float, default=0.0)
    ap.add_argument("--top-k", type=int, default=None)
    ap.add_argument("--cpu", action="store_true")
    a = ap.parse_args()
    gpu = torch.cuda.is_available() and not a.cpu
    torch.manual_seed(0)
    model = llama(a.model, device="cpu", dtype=torch.bfloat16 if gpu else torch.float32).eval()
    if gpu:
        mm = None
        if a.max_memory_gb is not None:
            mm = {i: int(a.max_memory_gb * 2**30) for i in range(torch.cuda.device_count())}
            mm["cpu"] = 1 << 62
        dmap = place(model, max_memory=mm, kv_tokens=a.batch * (a.prompt + a.new))
    else:
        dmap = place(model, devices=["cpu"], max_memory={"cpu": 1 << 62})
    print("device_map:", {k: str(v) for k, v in dmap.items() if not k.startswith("layers.")},
          "layers:", sorted({str(v) for k, v in dmap.items() if k.startswith("layers.")}))
    first = next(iter(dmap.values()))
    prompt = torch.randint(0, model.cfg.vocab_size, (a.batch, a.prompt), device=first)
    cache = KVCache(model, a.batch, a.prompt + a.new)
    print(f"KV cache: {cache.nbytes() / 2**30:.2f} GiB ({KVCache.bytes_per_token(model) // 1024} KiB/token)")
    t0 = time.perf_counter()
    out = generate(model, prompt, a.new, temperature=a.temperature, top_k=a.top_k, cache=cache, graph=a.graph)
    if gpu:
        torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(f"generated {a.batch}x{a.new} tokens in {dt:.2f} s ({a.batch * a.new / dt:.1f} tok/s incl. prefill)")
    print("first sequence, new tokens:", out[0, a.prompt:].tolist())


if __name__ == "__main__":
    main()
