"""Time one conv data gradient with and without the BN-backward-sums epilogue (bst_*), the way the
ResNet-50 backward calls it, on the 256 x 256 tile and on the streaming short-K kernel (dgrad_stream.hip).

    python tools/dgrad_bst_probe.py N H Cin Cout R stride [iters] [--mask ss|bits|dual] [--addend] [--json]

``--mask ss``: ReLU mask recomputed from z and the BN's scale / shift (a bn1 / bn2 output);  ``bits``: the
residual block's 1-bit mask (block output, with ``--addend``: the shortcut gradient); ``dual``: a
downsample block's output (two BNs).  Prints one line per arm (``--json``: JSON lines with the achieved
HBM bandwidth from the bytes each arm must move).
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorchdistributed_amd._native import C  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dims", nargs=6, type=int)
    ap.add_argument("iters", nargs="?", type=int, default=20)
    ap.add_argument("--mask", default="ss", choices=["ss", "bits", "dual"])
    ap.add_argument("--addend", action="store_true")
    ap.add_argument("--json", action="store_true")
    a = ap.parse_args()
    N, H, Cin, Cout, R, st = a.dims
    pad = R // 2
    P = (H + 2 * pad - R) // st + 1
    dev = "cuda"
    dy = torch.randn(N, P, P, Cout, device=dev, dtype=torch.bfloat16)
    w = torch.randn(Cout, R, R, Cin, device=dev, dtype=torch.bfloat16) * 0.05
    z = torch.randn(N, H, H, Cin, device=dev, dtype=torch.bfloat16)
    add = torch.randn(N, H, H, Cin, device=dev, dtype=torch.bfloat16) if a.addend else None
    kw = dict(bst_z=z, bst_mean=torch.zeros(Cin, device=dev), bst_table=torch.zeros(64, 2, Cin, device=dev))
    out_b = N * H * H * Cin * 2
    extra = out_b  # z
    if a.mask == "ss":
        kw["bst_ss"] = torch.cat([torch.ones(Cin), torch.zeros(Cin)]).to(dev)
    else:
        kw["bst_bits"] = torch.randint(0, 256, (N * H * H * Cin // 8,), dtype=torch.uint8, device=dev)
        extra += out_b // 16
        if a.mask == "dual":
            kw.update(bst_z2=torch.randn_like(z), bst_mean2=torch.zeros(Cin, device=dev),
                      bst_table2=torch.zeros(64, 2, Cin, device=dev))
            extra += out_b
    add_b = out_b if a.addend else 0
    base_b = dy.numel() * 2 + out_b + add_b
    arms = (("plain", {}, 0, base_b), ("plain_stream", {}, 2, base_b), ("bst_tile", kw, 0, base_b + extra),
            ("bst_stream", kw, 1, base_b + extra))
    for name, k, mode, nbytes in arms:
        C().set_dgrad_stream(mode)
        for _ in range(3):
            C().conv_dgrad(dy, w, H, H, st, pad, 1, add, None, **k)
        torch.cuda.synchronize()
        t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0.record()
        for _ in range(a.iters):
            C().conv_dgrad(dy, w, H, H, st, pad, 1, add, None, **k)
        t1.record()
        torch.cuda.synchronize()
        ms = t0.elapsed_time(t1) / a.iters
        shape = f"N{N} H{H} {Cin}<-{Cout} {R}x{R}/{st} mask={a.mask} addend={int(a.addend)}"
        if a.json:
            print(json.dumps({"shape": shape, "arm": name, "ms": round(ms, 4), "GBps": round(nbytes / ms / 1e6, 1)}))
        else:
            print(f"{name}: {shape}: {ms:.4f} ms ({nbytes / ms / 1e6:.0f} GB/s)")
    C().set_dgrad_stream(-1)


if __name__ == "__main__":
    main()
