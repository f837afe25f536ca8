"""Flash-attention microbenchmark: native fwd / bwd kernels (csrc/kernels/attention.hip) at the
GPT-2-medium and Llama-3-8B training shapes, TFLOP/s (causal FLOPs = half of dense; backward counted as
2.5x forward), next to PyTorch-ROCm SDPA on the same tensors.  One JSON line per shape.

    python tools/bench_attn.py [--iters 20]
"""
import argparse
import json
import math
import os
import sys

import torch

# PDA_AB_ROOT: import another build of the package (tools/ab_build.sh) for an A/B on the same box
sys.path.insert(0, os.environ.get("PDA_AB_ROOT") or os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorchdistributed_amd._native import C  # noqa: E402

SHAPES = {"gpt2-medium": (16, 1024, 16, 16, 64), "llama3-8b": (1, 4096, 32, 8, 128)}


def timeit(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--no-torch", action="store_true")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    for name, (B, T, Hq, Hkv, D) in SHAPES.items():
        torch.manual_seed(0)
        q = torch.randn(B, T, Hq, D, device=dev, dtype=torch.bfloat16)
        k = torch.randn(B, T, Hkv, D, device=dev, dtype=torch.bfloat16)
        v = torch.randn(B, T, Hkv, D, device=dev, dtype=torch.bfloat16)
        do = torch.randn_like(q)
        scale = 1.0 / math.sqrt(D)
        o, lse = C().attn_fwd(q, k, v, scale, True, None, None)
        dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
        fwd_ms = timeit(lambda: C().attn_fwd(q, k, v, scale, True, None, None), a.iters)
        bwd_ms = timeit(lambda: C().attn_bwd(do, q, k, v, o, lse, dq, dk, dv, scale, True, None, None), a.iters)
        flop = 4.0 * B * Hq * T * T * D * 0.5
        rec = {"shape": name, "B": B, "T": T, "Hq": Hq, "Hkv": Hkv, "D": D, "causal": True,
               "fwd_ms": round(fwd_ms, 4), "fwd_tflops": round(flop / fwd_ms / 1e9, 1),
               "bwd_ms": round(bwd_ms, 4), "bwd_tflops": round(2.5 * flop / bwd_ms / 1e9, 1)}
        if not a.no_torch:
            try:
                import torch.nn.functional as F

                qt, kt, vt = (t.transpose(1, 2).contiguous() for t in (q, k, v))
                if Hq != Hkv:
                    kt = kt.repeat_interleave(Hq // Hkv, 1)
                    vt = vt.repeat_interleave(Hq // Hkv, 1)
                qt.requires_grad_(); kt.requires_grad_(); vt.requires_grad_()
                ot = F.scaled_dot_product_attention(qt, kt, vt, is_causal=True)
                dot = torch.randn_like(ot)
                tf = timeit(lambda: F.scaled_dot_product_attention(qt, kt, vt, is_causal=True), a.iters)
                tb = timeit(lambda: torch.autograd.grad(ot, (qt, kt, vt), dot, retain_graph=True), a.iters)
                rec.update({"torch_sdpa_fwd_ms": round(tf, 4), "torch_sdpa_fwd_tflops": round(flop / tf / 1e9, 1),
                            "torch_sdpa_bwd_ms": round(tb, 4), "torch_sdpa_bwd_tflops": round(2.5 * flop / tb / 1e9, 1)})
            except Exception as e:  # noqa: BLE001
                rec["torch_sdpa"] = f"unavailable: {type(e).__name__}"
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
