"""Time the wide-tile GEMM schedule variants (0: plain, 1: setprio, 2: MFMA/ds_read interleave, 3: both)."""
import json
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from pytorchdistributed_amd._native import C  # noqa: E402

SHAPES = [(8192, 8192, 8192), (4096, 4096, 4096), (50176, 256, 2304), (50176, 1024, 256), (16384, 4096, 1024)]


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
    out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    rec = {"M": M, "N": N, "K": K}
    ref = None
    for v in range(4):
        C().set_gemm_paths(2, v)
        ms = t(lambda: C().gemm(a, True, K, b, True, K, out, N, M, N, K, None, False, False))
        rec[f"v{v}_tflops"] = round(2 * M * N * K / ms / 1e9, 1)
        if ref is None:
            ref = out.clone()
        else:
            rec[f"v{v}_same"] = bool(torch.equal(ref, out))
    C().set_gemm_paths(0, 0)
    ms = t(lambda: C().gemm(a, True, K, b, True, K, out, N, M, N, K, None, False, False))
    rec["narrow_tflops"] = round(2 * M * N * K / ms / 1e9, 1)
    print(json.dumps(rec), flush=True)
