"""1x1-conv weight gradients (dW[Cout, Cin] = dy[NPQ, Cout]^T x[NPQ, Cin]) of the ResNet-50 small-spatial
layers: the native split-K MFMA path vs hipBLASLt (torch.matmul on the same bf16 operands).

    python tools/bench_1x1_wgrad.py [--batch 512]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorchdistributed_amd._native import C  # noqa: E402

SHAPES = [(14, 256, 1024), (14, 1024, 256), (7, 512, 2048), (7, 2048, 512), (14, 1024, 512), (28, 512, 128),
          (28, 128, 512), (56, 64, 256), (56, 256, 64)]


def t(fn, it=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=512)
    a = ap.parse_args()
    for H, ci, co in SHAPES:
        x = torch.randn(a.batch, H, H, ci, device="cuda", dtype=torch.bfloat16)
        dy = torch.randn(a.batch, H, H, co, device="cuda", dtype=torch.bfloat16)
        dw = torch.empty(co, 1, 1, ci, device="cuda", dtype=torch.bfloat16)
        native = t(lambda: C().conv_wgrad(dy, x, 1, 1, 1, 0, 1, False, dw))
        dy2, x2 = dy.view(-1, co), x.view(-1, ci)
        out = torch.empty(co, ci, device="cuda", dtype=torch.bfloat16)
        blas = t(lambda: torch.matmul(dy2.t(), x2, out=out))
        ref = torch.matmul(dy2.t().float(), x2.float())
        err = ((dw.view(co, ci).float() - ref).norm() / ref.norm()).item()
        print(json.dumps({"H": H, "Cin": ci, "Cout": co, "native_us": round(native, 1), "hipblaslt_us": round(blas, 1),
                          "native_rel_err": err}), flush=True)


if __name__ == "__main__":
    main()
