"""Decode-GEMM microbench: weight-only int8 (csrc/kernels/w8_gemm.hip) vs bf16 hipBLASLt (torch.matmul)
on the Llama-3-8B projections at decode batch sizes.  Reports time and weight-stream bandwidth."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorchdistributed_amd import _native  # noqa: E402
from pytorchdistributed_amd.ops.quant import _workspace, quantize_int8  # noqa: E402


def timeit(fn, iters=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    C = _native.C()
    for name, N, K in [("wqkv", 6144, 4096), ("wo", 4096, 4096), ("w13", 28672, 4096), ("w2", 4096, 14336),
                       ("head", 128256, 4096)]:
        w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16)
        q, s = quantize_int8(w)
        ws, tk = _workspace(torch.device("cuda", 0), N)
        for M in (1, 16, 32, 64):
            x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
            t8 = timeit(lambda: C.w8_gemm(x, q, s, ws, tk))
            tb = timeit(lambda: x @ w.t())
            print(json.dumps({"proj": name, "M": M, "N": N, "K": K, "int8_ms": round(t8, 4),
                              "int8_GBps": round(N * K / (t8 * 1e-3) / 1e9, 1), "bf16_ms": round(tb, 4),
                              "bf16_GBps": round(2 * N * K / (tb * 1e-3) / 1e9, 1),
                              "speedup": round(tb / t8, 2)}), flush=True)


if __name__ == "__main__":
    main()
