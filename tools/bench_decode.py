"""Decode-attention microbench (csrc/kernels/decode_attn.hip) on Llama-3 shapes: one query token per
sequence vs a bf16 KV cache.  Reports time and effective HBM bandwidth (K+V bytes read / time), and
PyTorch SDPA (math/flash backends as ROCm PyTorch picks them, GQA expanded) on the same inputs."""
import json
import math
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorchdistributed_amd.ops.attention import decode_attention  # noqa: E402


def timeit(fn, iters=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    torch.manual_seed(0)
    dev = "cuda"
    for (B, L, Hq, Hkv, D) in [(1, 8192, 32, 8, 128), (16, 4096, 32, 8, 128), (64, 2048, 32, 8, 128),
                               (128, 1024, 32, 8, 128), (32, 8192, 32, 8, 128), (64, 1024, 16, 16, 64),
                               (32, 4096, 64, 8, 128)]:
        k = torch.randn(B, L, Hkv, D, device=dev, dtype=torch.bfloat16)
        v = torch.randn_like(k)
        q = torch.randn(B, 1, Hq, D, device=dev, dtype=torch.bfloat16)
        ms = timeit(lambda: decode_attention(q, k, v, L))
        gb = 2 * k.numel() * 2 / 1e9
        rec = {"B": B, "L": L, "Hq": Hq, "Hkv": Hkv, "D": D, "ms": round(ms, 4), "GBps": round(gb / (ms * 1e-3), 1)}
        try:
            qt, kt, vt = q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2)
            fn = lambda: F.scaled_dot_product_attention(qt, kt, vt, scale=1 / math.sqrt(D), enable_gqa=Hq != Hkv)  # noqa: E731
            tms = timeit(fn, 20)
            rec["torch_sdpa_ms"] = round(tms, 4)
            rec["torch_sdpa_GBps"] = round(gb / (tms * 1e-3), 1)
        except Exception as e:  # noqa: BLE001
            rec["torch_sdpa"] = f"unavailable: {type(e).__name__}"
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
