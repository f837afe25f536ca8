"""hipBLASLt (torch.mm) vs the native MFMA GEMM on square and conv-as-GEMM shapes (bf16)."""
import json
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from pytorchdistributed_amd._native import C  # noqa: E402

SHAPES = [(8192, 8192, 8192), (4096, 4096, 4096), (50176, 256, 2304), (200704, 128, 1152), (802816, 64, 576),
          (12544, 512, 4608), (16384, 4096, 1024), (16384, 1024, 4096)]


def t(fn, it=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it


for M, N, K in SHAPES:
    a = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    b = torch.randn(N, K, device="cuda").to(torch.bfloat16)
    fl = 2 * M * N * K
    tb = t(lambda: torch.mm(a, b.t()))
    out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    tn = t(lambda: C().gemm(a, True, K, b, True, K, out, N, M, N, K, None, False, False))
    print(json.dumps({"M": M, "N": N, "K": K, "blas_ms": round(tb, 4), "blas_tflops": round(fl / tb / 1e9, 1),
                      "native_ms": round(tn, 4), "native_tflops": round(fl / tn / 1e9, 1)}), flush=True)
