"""Microbenchmark of the BatchNorm kernels on ResNet-50 bs256 shapes: forward (stats+apply) and
backward with the ReLU mask from y (16-bit), from the bit mask, or recomputed from x (scale/shift).
Prints JSON lines with ms and effective TB/s."""
import json
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from pytorchdistributed_amd._native import C  # noqa: E402

SHAPES = [(256 * 56 * 56, 256), (256 * 28 * 28, 512), (256 * 14 * 14, 1024), (256 * 56 * 56, 64),
          (256 * 7 * 7, 2048)]


def timeit(fn, it=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it


def main():
    dev = "cuda"
    for M, Cc in SHAPES:
        x = torch.randn(M, Cc, device=dev).to(torch.bfloat16)
        r = torch.randn(M, Cc, device=dev).to(torch.bfloat16)
        dy = torch.randn(M, Cc, device=dev).to(torch.bfloat16)
        g = torch.ones(Cc, device=dev)
        b = torch.zeros(Cc, device=dev)
        rm, rv = torch.zeros(Cc, device=dev), torch.ones(Cc, device=dev)
        n = M * Cc
        y, mean, invstd, ss, bits = C().bn_fwd_train(x, r, g, b, rm, rv, 0.1, 1e-5, True, True, None)
        res = {"M": M, "C": Cc}
        t = timeit(lambda: C().bn_fwd_train(x, r, g, b, rm, rv, 0.1, 1e-5, True, True, None))
        res["fwd_res_relu_ms"] = round(t, 4)
        res["fwd_TBps"] = round(n * 2 * (1 + 3) / t / 1e9, 2)
        y2 = torch.empty_like(x)
        t = timeit(lambda: y2.copy_(x))
        res["copy_TBps"] = round(n * 2 * 2 / t / 1e9, 2)
        for name, saved, ssv in (("y", y, None), ("bits", bits, None), ("ss", None, ss)):
            t = timeit(lambda: C().bn_bwd(dy, x, saved, ssv, mean, invstd, g, True, True, None, None))
            res[f"bwd_{name}_ms"] = round(t, 4)
            per = {"y": 16, "bits": 12.25, "ss": 12}[name]  # bytes per element over both passes
            res[f"bwd_{name}_TBps"] = round(n * per / t / 1e9, 2)
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
