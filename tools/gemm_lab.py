"""A/B lab for the pipelined GEMM (csrc/kernels/gemm_pp.hip) against the production native kernel and
hipBLASLt (torch.mm), interleaved rounds in one process on uniform [-1, 1) bf16 operands
(cdna_hip_programming.md §5.4 rules 24/25).  Prints one JSON line per shape.

    python tools/gemm_lab.py [--variants 0,1,2,3] [--iters 20] [--rounds 3] [--shapes ...]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorchdistributed_amd._native import C  # noqa: E402

SHAPES = [
    (4096, 4096, 4096),
    (8192, 8192, 8192),
    (32768, 3072, 1024),   # GPT-2-medium qkv
    (32768, 1024, 1024),   # attn proj
    (32768, 4096, 1024),   # fc1
    (32768, 1024, 4096),   # fc2
    (16384, 4096, 4096),   # Llama-3-8B q / o
    (16384, 14336, 4096),  # gate / up
    (16384, 4096, 14336),  # down
    (16384, 4800, 1600),   # GPT-2-XL qkv (K = 25 tiles)
]
EDGE = [(1000, 264, 136), (257, 520, 72), (300, 256, 1600), (1, 8, 8)]


def timed(fn, iters):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="0,1,2,3")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--shapes", default="")
    ap.add_argument("--no-native", action="store_true")
    args = ap.parse_args()
    variants = [int(v) for v in args.variants.split(",") if v != ""]
    shapes = SHAPES
    if args.shapes:
        shapes = [tuple(int(x) for x in s.split("x")) for s in args.shapes.split(",")]
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    # correctness on edge shapes first (fp32 reference of the bf16 operands)
    for (M, N, K) in EDGE:
        a = (torch.rand(M, K, device=dev) * 2 - 1).bfloat16()
        b = (torch.rand(N, K, device=dev) * 2 - 1).bfloat16()
        bias = (torch.rand(N, device=dev) - 0.5).bfloat16()
        ref = a.float() @ b.float().t() + bias.float()
        for v in variants:
            c = torch.full((M, N), float("nan"), device=dev, dtype=torch.bfloat16)
            C().gemm_pp_lab(a, b, c, bias, v)
            err = ((c.float() - ref).abs().max() / ref.abs().max().clamp_min(1e-6)).item()
            print(json.dumps({"check": [M, N, K], "variant": v, "max_rel_err": err, "ok": err < 2e-2}), flush=True)
    for (M, N, K) in shapes:
        a = (torch.rand(M, K, device=dev) * 2 - 1).bfloat16()
        b = (torch.rand(N, K, device=dev) * 2 - 1).bfloat16()
        cref = torch.mm(a, b.t())
        arms = {}
        outs = {}
        for v in variants:
            outs[f"pp{v}"] = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            arms[f"pp{v}"] = (lambda v=v, o=outs[f"pp{v}"]: C().gemm_pp_lab(a, b, o, None, v))
        if not args.no_native:
            outs["native"] = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            arms["native"] = lambda o=outs["native"]: C().gemm(a, True, K, b, True, K, o, N, M, N, K, None, False, True)
        outs["blas"] = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        arms["blas"] = lambda o=outs["blas"]: torch.mm(a, b.t(), out=o)
        times = {k: [] for k in arms}
        for _ in range(args.rounds):
            for k, fn in arms.items():
                times[k].append(timed(fn, args.iters))
        flop = 2.0 * M * N * K
        rec = {"M": M, "N": N, "K": K}
        for k, ts in times.items():
            t = sorted(ts)[len(ts) // 2]
            rec[f"{k}_tflops"] = round(flop / t / 1e9, 1)
            if k != "blas":
                d = (outs[k].float() - cref.float()).abs().max().item()
                rec[f"{k}_maxdiff"] = round(d, 4)
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
