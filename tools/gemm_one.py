"""Run one native GEMM (M N K) repeatedly — the unit of work for rocprofv3 PMC collection."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorchdistributed_amd._native import C  # noqa: E402

M, N, K = map(int, sys.argv[1:4])
iters = int(sys.argv[4]) if len(sys.argv) > 4 else 5
a = torch.randn(M, K, device="cuda").to(torch.bfloat16)
b = torch.randn(N, K, device="cuda").to(torch.bfloat16)
out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
for _ in range(iters):
    C().gemm(a, True, K, b, True, K, out, N, M, N, K, None, False, False)
torch.cuda.synchronize()
