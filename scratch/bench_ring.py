"""A/B of the wide-tile GEMM schedules: the 2-stage kernel (ring=0) vs the 4-slot ring of 32-deep K
tiles (ring=1), interleaved in one process (min of `--rounds` per arm), on plain GEMMs (squares, the
GPT-2-medium / Llama-3-8B projections in all three layouts) and on every ResNet-50 conv that takes the
wide tile.  Both schedules accumulate every output in the same K order, so their outputs must be
bit-identical: each case also reports the max |ring - 2stage| (expected 0).

    python tools/bench_ring.py [--batch 640] [--rounds 3] [--iters 10] > out.jsonl
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorchdistributed_amd._native import C  # noqa: E402
from tools.bench_conv import COUNT, RESNET_CONVS, time_fn  # noqa: E402


def ab(c, fn, out, rounds, iters):
    best = {0: 1e9, 1: 1e9}
    res = {}
    for _ in range(rounds):
        for ring in (0, 1):
            c.set_gemm_paths(-1, ring)
            best[ring] = min(best[ring], time_fn(fn, iters))
    for ring in (0, 1):
        c.set_gemm_paths(-1, ring)
        fn()
        torch.cuda.synchronize()
        res[ring] = out.float().clone()
    c.set_gemm_paths(-1, -1)
    diff = (res[0] - res[1]).abs().max().item()
    return best, diff


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=640)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--no-conv", action="store_true")
    a = ap.parse_args()
    c = C()
    dev = "cuda"
    gemms = [(4096, 4096, 4096), (8192, 8192, 8192)]
    for T, d, f in ((32768, 1024, 4096), (16384, 4096, 14336)):
        for N, K in ((3 * d if d == 1024 else 6144, d), (d, d), (f, d), (d, f)):
            gemms.append((T, N, K))
    tot = {0: 0.0, 1: 0.0}
    for M, N, K in gemms:
        for lay in ("fwd", "dgrad", "wgrad"):
            if lay == "fwd":  # y[M,N] = x[M,K] W[N,K]^T
                A = torch.randn(M, K, device=dev).to(torch.bfloat16)
                B = torch.randn(N, K, device=dev).to(torch.bfloat16)
                out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
                fn = lambda: c.gemm(A, True, K, B, True, K, out, N, M, N, K, None, False, False)  # noqa: E731
                mm, nn, kk = M, N, K
            elif lay == "dgrad":  # dx[M,K] = dy[M,N] W[N,K]
                A = torch.randn(M, N, device=dev).to(torch.bfloat16)
                B = torch.randn(N, K, device=dev).to(torch.bfloat16)
                out = torch.empty(M, K, device=dev, dtype=torch.bfloat16)
                fn = lambda: c.gemm(A, True, N, B, False, K, out, K, M, K, N, None, False, False)  # noqa: E731
                mm, nn, kk = M, K, N
            else:  # dW[N,K] = dy[M,N]^T x[M,K]
                if M == N == K:
                    continue
                A = torch.randn(M, N, device=dev).to(torch.bfloat16)
                B = torch.randn(M, K, device=dev).to(torch.bfloat16)
                out = torch.empty(N, K, device=dev, dtype=torch.bfloat16)
                fn = lambda: c.gemm(A, False, N, B, False, K, out, K, N, K, M, None, False, False)  # noqa: E731
                mm, nn, kk = N, K, M
            best, diff = ab(c, fn, out, a.rounds, a.iters)
            fl = 2.0 * mm * nn * kk
            print(json.dumps({"op": "gemm", "layout": lay, "M": mm, "N": nn, "K": kk,
                              "two_stage_ms": round(best[0], 4), "ring_ms": round(best[1], 4),
                              "two_stage_tflops": round(fl / best[0] / 1e9, 1),
                              "ring_tflops": round(fl / best[1] / 1e9, 1),
                              "speedup": round(best[0] / best[1], 3), "max_abs_diff": diff}), flush=True)
            del A, B, out
    if a.no_conv:
        return
    for (H, Ci, Co, R, st), cnt in zip(RESNET_CONVS, COUNT):
        pad = 0 if R == 4 else R // 2
        P = (H + 2 * pad - R) // st + 1
        x = torch.randn(a.batch, H, H, Ci, device=dev, dtype=torch.bfloat16)
        w = torch.randn(Co, R, R, Ci, device=dev, dtype=torch.bfloat16) * 0.05
        dy = torch.randn(a.batch, P, P, Co, device=dev, dtype=torch.bfloat16)
        dwo = torch.empty(Co, R, R, Ci, device=dev, dtype=torch.float32)
        holder = {}

        def fwd():
            holder["o"] = c.conv_fwd(x, w, st, pad, 1, None, False)

        def dgrad():
            holder["o"] = c.conv_dgrad(dy, w, H, H, st, pad, 1, None)

        def wgrad():
            c.conv_wgrad(dy, x, R, R, st, pad, 1, True, dwo)
            holder["o"] = dwo

        fns = {"fwd": fwd, "dgrad": dgrad, "wgrad": wgrad}
        if R == 4:
            del fns["dgrad"]
        rec = {"op": "conv", "H": H, "Cin": Ci, "Cout": Co, "R": R, "stride": st, "count": cnt}
        for k, fn in fns.items():
            best = {0: 1e9, 1: 1e9}
            outs = {}
            for _ in range(a.rounds):
                for ring in (0, 1):
                    c.set_gemm_paths(-1, ring)
                    best[ring] = min(best[ring], time_fn(fn, a.iters))
            for ring in (0, 1):
                c.set_gemm_paths(-1, ring)
                fn()
                torch.cuda.synchronize()
                outs[ring] = holder["o"].float().clone()
            c.set_gemm_paths(-1, -1)
            rec[f"{k}_two_stage_ms"] = round(best[0], 4)
            rec[f"{k}_ring_ms"] = round(best[1], 4)
            rec[f"{k}_diff"] = (outs[0] - outs[1]).abs().max().item()
            tot[0] += best[0] * cnt
            tot[1] += best[1] * cnt
        print(json.dumps(rec), flush=True)
    print(json.dumps({"op": "conv_total_per_forward_set_ms", "two_stage": round(tot[0], 3), "ring": round(tot[1], 3)}))


if __name__ == "__main__":
    main()
