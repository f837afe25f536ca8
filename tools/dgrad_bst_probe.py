"""Time one conv data gradient with and without the BN-backward-sums epilogue (bst_*), the way the
ResNet-50 backward calls it (ReLU mask recomputed from z and the BN's scale / shift).

    python tools/dgrad_bst_probe.py N H Cin Cout R stride [iters]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorchdistributed_amd._native import C  # noqa: E402


def main():
    N, H, Cin, Cout, R, st = map(int, sys.argv[1:7])
    iters = int(sys.argv[7]) if len(sys.argv) > 7 else 20
    pad = R // 2
    P = (H + 2 * pad - R) // st + 1
    dev = "cuda"
    dy = torch.randn(N, P, P, Cout, device=dev, dtype=torch.bfloat16)
    w = torch.randn(Cout, R, R, Cin, device=dev, dtype=torch.bfloat16) * 0.05
    z = torch.randn(N, H, H, Cin, device=dev, dtype=torch.bfloat16)
    kw = dict(bst_z=z, bst_mean=torch.zeros(Cin, device=dev), bst_table=torch.zeros(64, 2, Cin, device=dev),
              bst_ss=torch.cat([torch.ones(Cin), torch.zeros(Cin)]).to(dev))
    for name, k in (("plain", {}), ("bst", kw)):
        for _ in range(3):
            C().conv_dgrad(dy, w, H, H, st, pad, 1, None, None, **k)
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(iters):
            C().conv_dgrad(dy, w, H, H, st, pad, 1, None, None, **k)
        b.record()
        torch.cuda.synchronize()
        print(f"{name}: N{N} H{H} {Cin}<-{Cout} {R}x{R}/{st}: {a.elapsed_time(b) / iters:.4f} ms")


if __name__ == "__main__":
    main()
