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
EDGE = [(1000, 264, 136), (256, 520, 72), (296, 256, 1600), (8, 8, 8), (512, 512, 4096)]
LAYOUTS = ("nt", "nn", "tn")


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
    ap.add_argument("--layouts", default="nt,tn")
    args = ap.parse_args()
    variants = [int(v) for v in args.variants.split(",") if v != ""]
    shapes = SHAPES
    if args.shapes:
        shapes = [tuple(int(x) for x in s.split("x")) for s in args.shapes.split(",")]
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    # correctness on edge shapes first (fp32 reference of the bf16 operands), every operand layout
    for (M, N, K) in EDGE:
        for lay in LAYOUTS:
            a, b, ak, lda, bk, ldb, ref = operands(lay, M, N, K, dev)
            bias = (torch.rand(N, device=dev) - 0.5).bfloat16()
            ref = ref + bias.float()
            for v in variants:
                c = torch.full((M, N), float("nan"), device=dev, dtype=torch.bfloat16)
                C().gemm_pp_lab(a, ak, lda, b, bk, ldb, c, N, M, N, K, bias, v)
                err = ((c.float() - ref).abs().max() / ref.abs().max().clamp_min(1e-6)).item()
                print(json.dumps({"check": [M, N, K], "layout": lay, "variant": v, "max_rel_err": err,
                                  "ok": err < 2e-2}), flush=True)
    for lay in args.layouts.split(","):
        for (M, N, K) in shapes:
            a, b, ak, lda, bk, ldb, ref = operands(lay, M, N, K, dev, want_ref=False)
            arms, outs = {}, {}
            for v in variants:
                o = outs[f"pp{v}"] = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
                arms[f"pp{v}"] = (lambda v=v, o=o: C().gemm_pp_lab(a, ak, lda, b, bk, ldb, o, N, M, N, K, None, v))
            if not args.no_native:
                o = outs["native"] = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
                arms["native"] = lambda o=o: C().gemm(a, ak, lda, b, bk, ldb, o, N, M, N, K, None, False, False)
            o = outs["blas"] = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            arms["blas"] = lambda o=o: torch.mm(torch_view(a, ak, M, K), torch_view_b(b, bk, N, K), out=o)
            times = {k: [] for k in arms}
            for _ in range(args.rounds):
                for k, fn in arms.items():
                    times[k].append(timed(fn, args.iters))
            flop = 2.0 * M * N * K
            rec = {"layout": lay, "M": M, "N": N, "K": K}
            cref = outs["blas"].float()
            for k, ts in times.items():
                t = sorted(ts)[len(ts) // 2]
                rec[f"{k}_tflops"] = round(flop / t / 1e9, 1)
                if k != "blas":
                    rec[f"{k}_maxdiff"] = round((outs[k].float() - cref).abs().max().item(), 4)
            print(json.dumps(rec), flush=True)


def torch_view(a, ak, M, K):
    return a if ak else a.t()  # A(m,k): [M,K] K-major, or stored [K,M]


def torch_view_b(b, bk, N, K):
    return b.t() if bk else b  # B(k,n): stored [N,K] (K-major) or [K,N]


def operands(lay, M, N, K, dev, want_ref=True):
    """nt: A [M,K], B [N,K] (Linear forward); nn: A [M,K], B [K,N] (dgrad); tn: A [K,M], B [K,N] (wgrad)."""
    ak = lay in ("nt", "nn")
    bk = lay == "nt"
    a = ((torch.rand(M, K, device=dev) if ak else torch.rand(K, M, device=dev)) * 2 - 1).bfloat16()
    b = ((torch.rand(N, K, device=dev) if bk else torch.rand(K, N, device=dev)) * 2 - 1).bfloat16()
    lda = K if ak else M
    ldb = K if bk else N
    ref = None
    if want_ref:
        ref = torch_view(a, ak, M, K).float() @ torch_view_b(b, bk, N, K).float()
    return a, b, ak, lda, bk, ldb, ref


if __name__ == "__main__":
    main()
