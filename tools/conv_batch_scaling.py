"""Per-image cost of the native conv kernels vs batch size (does a layer stop scaling linearly once its
activations outgrow the 256 MB Infinity Cache?), and the same batch run as two half-batch launches.

    python tools/conv_batch_scaling.py
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorchdistributed_amd._native import C  # noqa: E402

SHAPES = [(56, 64, 64, 3, 1), (56, 128, 128, 3, 2), (56, 64, 64, 1, 1), (56, 64, 256, 1, 1), (28, 128, 128, 3, 1)]
BATCHES = [128, 256, 384, 512, 640]


def time_fn(fn, iters=10):
    for _ in range(2):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3  # us


def main():
    c = C()
    for H, Ci, Co, R, st in SHAPES:
        pad = R // 2
        P = (H + 2 * pad - R) // st + 1
        nmax = max(BATCHES)
        x = torch.randn(nmax, H, H, Ci, device="cuda").to(torch.bfloat16)
        w = (torch.randn(Co, R, R, Ci, device="cuda") * 0.05).to(torch.bfloat16)
        dy = torch.randn(nmax, P, P, Co, device="cuda").to(torch.bfloat16)
        rec = {"shape": [H, Ci, Co, R, st]}
        for n in BATCHES:
            xs, dys = x[:n], dy[:n]
            rec[f"fwd_us_per_img_b{n}"] = round(time_fn(lambda: c.conv_fwd(xs, w, st, pad, 1, None, False)) / n, 3)
            rec[f"dgrad_us_per_img_b{n}"] = round(time_fn(lambda: c.conv_dgrad(dys, w, H, H, st, pad, 1, None)) / n, 3)
        h = nmax // 2
        x0, x1, d0, d1 = x[:h], x[h:], dy[:h], dy[h:]
        rec["fwd_us_per_img_2x_half"] = round(time_fn(lambda: (c.conv_fwd(x0, w, st, pad, 1, None, False),
                                                                c.conv_fwd(x1, w, st, pad, 1, None, False))) / nmax, 3)
        rec["dgrad_us_per_img_2x_half"] = round(time_fn(lambda: (c.conv_dgrad(d0, w, H, H, st, pad, 1, None),
                                                                  c.conv_dgrad(d1, w, H, H, st, pad, 1, None))) / nmax, 3)
        print(json.dumps(rec), flush=True)
        del x, dy


if __name__ == "__main__":
    main()
