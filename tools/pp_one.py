"""Run one GEMM (pipelined kernel variant, or hipBLASLt with variant -1) repeatedly: the unit of work
for rocprofv3 PMC passes.   python tools/pp_one.py VARIANT LAYOUT M N K [iters]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorchdistributed_amd._native import C  # noqa: E402

v, lay = int(sys.argv[1]), sys.argv[2]
M, N, K = map(int, sys.argv[3:6])
iters = int(sys.argv[6]) if len(sys.argv) > 6 else 10
ak, bk = lay in ("nt", "nn"), lay == "nt"
a = (torch.rand(M, K, device="cuda") * 2 - 1).bfloat16() if ak else (torch.rand(K, M, device="cuda") * 2 - 1).bfloat16()
b = (torch.rand(N, K, device="cuda") * 2 - 1).bfloat16() if bk else (torch.rand(K, N, device="cuda") * 2 - 1).bfloat16()
out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
for _ in range(iters):
    if v < 0:
        torch.mm(a if ak else a.t(), b.t() if bk else b, out=out)
    else:
        C().gemm_pp_lab(a, ak, K if ak else M, b, bk, K if bk else N, out, N, M, N, K, None, v)
torch.cuda.synchronize()
