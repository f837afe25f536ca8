"""Time the 1x1 stride-1 conv forward with its BN statistics epilogue at ResNet-50 bs-640 shapes on the 256 x 256
tile (mode 0) and on the streaming kernel (fwd_stream.hip; mode 2 admits K = 256), with the HBM bandwidth the
launch reaches from the bytes it must move (x + w + y).

    python tools/fwd_stream_probe.py [iters] [--json]
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.environ.get("PDA_AB_ROOT") or os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorchdistributed_amd._native import C  # noqa: E402

SHAPES = [(56, 64, 256), (56, 64, 64), (28, 128, 512), (14, 256, 1024), (7, 512, 2048), (56, 256, 64),
          (28, 512, 128), (14, 1024, 256)]


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 20
    dev, N = "cuda", 640
    for H, Cin, Cout in SHAPES:
        x = torch.randn(N, H, H, Cin, device=dev, dtype=torch.bfloat16)
        w = torch.randn(Cout, 1, 1, Cin, device=dev, dtype=torch.bfloat16) * 0.05
        shift = torch.zeros(Cout, device=dev)
        table = torch.zeros(64, 2, Cout, device=dev)
        nbytes = x.numel() * 2 + w.numel() * 2 + N * H * H * Cout * 2
        for mode in (0, 2):
            C().set_fwd_stream(mode)
            for _ in range(3):
                C().conv_fwd_stats(x, w, 1, 0, 1, shift, table)
            torch.cuda.synchronize()
            t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            t0.record()
            for _ in range(iters):
                C().conv_fwd_stats(x, w, 1, 0, 1, shift, table)
            t1.record()
            torch.cuda.synchronize()
            ms = t0.elapsed_time(t1) / iters
            print(json.dumps({"shape": f"N{N} H{H} {Cin}->{Cout} 1x1", "arm": "tile" if mode == 0 else "stream",
                              "ms": round(ms, 4), "GBps": round(nbytes / ms / 1e6, 1)}), flush=True)
        C().set_fwd_stream(-1)


if __name__ == "__main__":
    main()
