"""Per-shape TFLOP/s of the native MFMA GEMM / implicit-GEMM conv kernels vs the vendor libraries
(hipBLASLt through torch.matmul, MIOpen through F.conv2d channels-last) on the ResNet-50 bs-256
layer shapes.  Prints one JSON line per (shape, op).

    python tools/bench_conv.py [--batch 256] [--iters 20] [--torch]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F

# PDA_AB_ROOT: import another build of the package (tools/ab_build.sh) for an A/B on the same box
sys.path.insert(0, os.environ.get("PDA_AB_ROOT") or os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorchdistributed_amd._native import C  # noqa: E402

# (H, Cin, Cout, R, stride) for every distinct ResNet-50 conv (input spatial size H)
RESNET_CONVS = [
    (115, 16, 64, 4, 1),  # the 7x7/2 stem as run: 4x4/1 valid conv over the 2x2 space-to-depth image
    (56, 64, 64, 1, 1), (56, 64, 64, 3, 1), (56, 64, 256, 1, 1), (56, 256, 64, 1, 1),
    (56, 256, 128, 1, 1), (56, 128, 128, 3, 2), (28, 128, 512, 1, 1), (56, 256, 512, 1, 2),
    (28, 512, 128, 1, 1), (28, 128, 128, 3, 1),
    (28, 512, 256, 1, 1), (28, 256, 256, 3, 2), (14, 256, 1024, 1, 1), (28, 512, 1024, 1, 2),
    (14, 1024, 256, 1, 1), (14, 256, 256, 3, 1),
    (14, 1024, 512, 1, 1), (14, 512, 512, 3, 2), (7, 512, 2048, 1, 1), (14, 1024, 2048, 1, 2),
    (7, 2048, 512, 1, 1), (7, 512, 512, 3, 1),
]
# how many times each shape appears in one ResNet-50 forward
COUNT = [1, 1, 3, 4, 2, 1, 1, 4, 1, 3, 3, 1, 1, 6, 1, 5, 5, 1, 1, 3, 1, 2, 2]


ROOF_PF = 2.2e15  # dense bf16 MFMA at the ~2.1 GHz the chip holds under MFMA load (1024 FLOP/clk/SIMD)
ROOF_BW = 5.5e12  # HBM bytes/s a streaming kernel sustains (the BN kernels reach 5-6 TB/s)


def time_fn(fn, iters):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--torch", action="store_true", help="also time MIOpen / hipBLASLt")
    ap.add_argument("--blas", action="store_true", help="1x1 stride-1 convs: also time the same GEMM on hipBLASLt")
    ap.add_argument("--wide", type=int, default=-1, help="wide-tile GEMM path: -1 env, 0 off, 1 auto, 2 force")
    ap.add_argument("--compare", action="store_true",
                    help="per shape and op, time the auto / 128-tile / wide-tile paths interleaved (min of 3)")
    a = ap.parse_args()
    c = C()
    c.set_gemm_paths(a.wide)
    dev = "cuda"
    for M, N, K in [(4096, 4096, 4096), (8192, 8192, 8192), (50176, 256, 2304), (12544, 512, 4608)]:
        A = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
        B = torch.randn(N, K, device=dev, dtype=torch.bfloat16)
        out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        ms = time_fn(lambda: c.gemm(A, True, K, B, True, K, out, N, M, N, K, None, False, False), a.iters)
        rec = {"op": "gemm", "shape": [M, N, K], "ms": round(ms, 4), "tflops": round(2 * M * N * K / ms / 1e9, 1)}
        if a.torch:
            mt = time_fn(lambda: torch.matmul(A, B.t()), a.iters)
            rec["torch_ms"] = round(mt, 4)
            rec["torch_tflops"] = round(2 * M * N * K / mt / 1e9, 1)
        print(json.dumps(rec), flush=True)
    tot = {"fwd": 0.0, "dgrad": 0.0, "wgrad": 0.0}
    tot_t = {"fwd": 0.0, "dgrad": 0.0, "wgrad": 0.0}
    tot_roof = {"fwd": 0.0, "dgrad": 0.0, "wgrad": 0.0}
    for (H, Ci, Co, R, st), cnt in zip(RESNET_CONVS, COUNT):
        pad = 0 if R == 4 else R // 2
        P = (H + 2 * pad - R) // st + 1
        x = torch.randn(a.batch, H, H, Ci, device=dev, dtype=torch.bfloat16)
        w = torch.randn(Co, R, R, Ci, device=dev, dtype=torch.bfloat16) * 0.05
        dy = torch.randn(a.batch, P, P, Co, device=dev, dtype=torch.bfloat16)
        dwo = torch.empty(Co, R, R, Ci, device=dev, dtype=torch.float32)
        flops = 2.0 * a.batch * P * P * Co * R * R * Ci
        fns = {"fwd": lambda: c.conv_fwd(x, w, st, pad, 1, None, False),
               "dgrad": lambda: c.conv_dgrad(dy, w, H, H, st, pad, 1, None),
               "wgrad": lambda: c.conv_wgrad(dy, x, R, R, st, pad, 1, True, dwo)}
        if R == 4:
            del fns["dgrad"]  # the stem's input needs no gradient
        rec = {"op": "conv", "H": H, "Cin": Ci, "Cout": Co, "R": R, "stride": st, "count": cnt}
        if a.compare:
            for k, fn in fns.items():
                best = {}
                for _ in range(3):
                    for mode, name in ((-1, "auto"), (0, "narrow"), (2, "wide")):
                        c.set_gemm_paths(mode)
                        ms = time_fn(fn, a.iters)
                        best[name] = min(best.get(name, 1e9), ms)
                c.set_gemm_paths(a.wide)
                for name, ms in best.items():
                    rec[f"{k}_{name}_ms"] = round(ms, 4)
            print(json.dumps(rec), flush=True)
            continue
        # roofline: minimum bytes (every operand read once, the output written once; bf16 activations,
        # fp32 weight gradient) at ROOF_BW vs FLOPs at ROOF_PF — the lower bound on each launch
        act_in, act_out = a.batch * H * H * Ci * 2, a.batch * P * P * Co * 2
        wbytes = Co * R * R * Ci * 2
        nbytes = {"fwd": act_in + act_out + wbytes, "dgrad": act_out + act_in + wbytes,
                  "wgrad": act_in + act_out + 2 * wbytes}
        for k, fn in fns.items():
            ms = time_fn(fn, a.iters)
            tot[k] += ms * cnt
            rec[k + "_ms"] = round(ms, 4)
            rec[k + "_tflops"] = round(flops / ms / 1e9, 1)
            roof = max(flops / ROOF_PF, nbytes[k] / ROOF_BW) * 1e3
            rec[k + "_roof_ms"] = round(roof, 4)
            rec[k + "_bound"] = "mfma" if flops / ROOF_PF > nbytes[k] / ROOF_BW else "hbm"
            rec[k + "_of_roof"] = round(roof / ms, 3)
            tot_roof[k] += roof * cnt
        if a.blas and R == 1 and st == 1:
            # the identical GEMMs on hipBLASLt (a 1x1 stride-1 conv IS a GEMM in NHWC): library class check
            x2, w2, dy2 = x.view(-1, Ci), w.view(Co, Ci), dy.view(-1, Co)
            bl = {"fwd": lambda: torch.mm(x2, w2.t()), "dgrad": lambda: torch.mm(dy2, w2),
                  "wgrad": lambda: torch.mm(dy2.t(), x2)}
            for k, fn in bl.items():
                ms = time_fn(fn, a.iters)
                rec["blas_" + k + "_ms"] = round(ms, 4)
        if a.torch:
            xt = x.permute(0, 3, 1, 2)
            wt = w.permute(0, 3, 1, 2)
            dyt = dy.permute(0, 3, 1, 2)
            tf = {"fwd": lambda: F.conv2d(xt, wt, None, st, pad),
                  "dgrad": lambda: torch.nn.grad.conv2d_input(xt.shape, wt, dyt, st, pad),
                  "wgrad": lambda: torch.nn.grad.conv2d_weight(xt, wt.shape, dyt, st, pad)}
            for k, fn in tf.items():
                ms = time_fn(fn, a.iters)
                tot_t[k] += ms * cnt
                rec["torch_" + k + "_ms"] = round(ms, 4)
        print(json.dumps(rec), flush=True)
    print(json.dumps({"op": "total_per_step_ms", "ours": {k: round(v, 3) for k, v in tot.items()},
                      "roofline": {k: round(v, 3) for k, v in tot_roof.items()},
                      "torch": {k: round(v, 3) for k, v in tot_t.items()} if a.torch else None}), flush=True)


if __name__ == "__main__":
    main()
