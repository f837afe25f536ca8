"""w8_gemm split-K sweep on the small-N Llama-3-8B projections (M = 32): time per split count."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorchdistributed_amd import _native  # noqa: E402
from pytorchdistributed_amd.ops.quant import _workspace, quantize_int8  # noqa: E402
from bench_w8 import timeit  # noqa: E402

C = _native.C()
for name, N, K in [("wqkv", 6144, 4096), ("wo", 4096, 4096), ("w2", 4096, 14336)]:
    q, s = quantize_int8(torch.randn(N, K, device="cuda"))
    ws, tk = _workspace(torch.device("cuda", 0), N)
    x = torch.randn(32, K, device="cuda", dtype=torch.bfloat16)
    rec = {"proj": name}
    for S in (1, 2, 4, 8):
        if K % (256 * S) == 0:
            rec[f"S{S}_us"] = round(timeit(lambda: C.w8_gemm(x, q, s, ws, tk, S)) * 1e3, 1)
    print(json.dumps(rec), flush=True)
