"""A/B the wide-tile GEMM main-loop schedules (3: one barrier per K step with setprio + MFMA/ds_read
interleave; 4: ping-pong wave groups) on plain GEMMs (vs hipBLASLt through torch.mm) and on the
ResNet-50 batch-640 convs (auto routing, so the split-K / 128-tile choices stay as in training).
Interleaved rounds in one process; prints one JSON line per shape with the median TFLOP/s per arm.

    python tools/bench_wide_variants.py [--variants 3,4] [--rounds 5] [--convs]
"""
import argparse
import json
import statistics
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from pytorchdistributed_amd._native import C  # noqa: E402

SHAPES = [(4096, 4096, 4096), (8192, 8192, 8192), (32768, 3072, 1024), (32768, 1024, 4096), (32768, 4096, 1024),
          (16384, 4096, 1024), (50176, 256, 2304), (50176, 1024, 256)]
# (batch, H, Cin, Cout, R, stride) — the heaviest ResNet-50 conv families at batch 640
CONVS = [(640, 56, 64, 256, 1, 1), (640, 56, 256, 64, 1, 1), (640, 56, 64, 64, 3, 1), (640, 28, 128, 128, 3, 1),
         (640, 28, 512, 128, 1, 1), (640, 14, 1024, 256, 1, 1), (640, 14, 256, 1024, 1, 1), (640, 7, 512, 2048, 1, 1)]


def t(fn, it=10):
    for _ in range(2):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="3,4,5,6")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--convs", action="store_true")
    ap.add_argument("--no-gemm", action="store_true")
    a = ap.parse_args()
    vs = [int(v) for v in a.variants.split(",")]
    c = C()
    if not a.no_gemm:
        for M, N, K in SHAPES:
            A = torch.randn(M, K, device="cuda").to(torch.bfloat16)
            B = torch.randn(N, K, device="cuda").to(torch.bfloat16)
            out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
            arms = {f"v{v}": (lambda v=v: (c.set_gemm_paths(2, v),
                                           c.gemm(A, True, K, B, True, K, out, N, M, N, K, None, False, False)))
                    for v in vs}
            arms["blas"] = lambda: torch.mm(A, B.t(), out=out)
            ms = {k: [] for k in arms}
            for _ in range(a.rounds):
                for k, fn in arms.items():
                    ms[k].append(t(fn))
            rec = {"M": M, "N": N, "K": K}
            for k, v in ms.items():
                rec[f"{k}_tflops"] = round(2 * M * N * K / statistics.median(v) / 1e9, 1)
            outs = []
            for v in vs:
                c.set_gemm_paths(2, v)
                c.gemm(A, True, K, B, True, K, out, N, M, N, K, None, False, False)
                outs.append(out.clone())
            rec["identical"] = all(torch.equal(outs[0], o) for o in outs[1:])
            print(json.dumps(rec), flush=True)
            del A, B, out, outs
    if a.convs:
        for n, H, Cin, Cout, R, st in CONVS:
            pad = R // 2
            x = torch.randn(n, H, H, Cin, device="cuda").to(torch.bfloat16)
            w = (torch.randn(Cout, R, R, Cin, device="cuda") * 0.05).to(torch.bfloat16)
            P = (H + 2 * pad - R) // st + 1
            dy = torch.randn(n, P, P, Cout, device="cuda").to(torch.bfloat16)
            flop = 2 * n * P * P * Cout * Cin * R * R
            ops = {"fwd": lambda: c.conv_fwd(x, w, st, pad, 1, None, False),
                   "dgrad": lambda: c.conv_dgrad(dy, w, H, H, st, pad, 1, None),
                   "wgrad": lambda: c.conv_wgrad(dy, x, R, R, st, pad, 1, False, None)}
            for op, fn in ops.items():
                ms = {v: [] for v in vs}
                for _ in range(a.rounds):
                    for v in vs:
                        c.set_gemm_paths(-1, v)
                        ms[v].append(t(fn))
                rec = {"conv": [n, H, Cin, Cout, R, st], "op": op}
                for v in vs:
                    rec[f"v{v}_ms"] = round(statistics.median(ms[v]), 4)
                    rec[f"v{v}_tflops"] = round(flop / statistics.median(ms[v]) / 1e9, 1)
                print(json.dumps(rec), flush=True)
            del x, w, dy
    c.set_gemm_paths(-1, 3)


if __name__ == "__main__":
    main()
