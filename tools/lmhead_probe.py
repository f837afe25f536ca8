"""Which kernel takes the LM-head weight gradient (MN-major x MN-major, K = tokens): run one Linear backward of
a GPT-2-medium / Llama-3-8B head shape; look at it under rocprofv3 --kernel-trace --stats."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorchdistributed_amd.ops.linear import linear  # noqa: E402

V, D, T = (int(a) for a in sys.argv[1:4]) if len(sys.argv) > 3 else (50304, 1024, 32768)
x = torch.randn(T, D, device="cuda", dtype=torch.bfloat16, requires_grad=True)
w = torch.nn.Parameter(torch.randn(V, D, device="cuda", dtype=torch.bfloat16) * 0.02)
dy = torch.randn(T, V, device="cuda", dtype=torch.bfloat16)
for _ in range(2):
    w.grad = None
    linear(x, w).backward(dy)
torch.cuda.synchronize()
print("ok", w.grad.dtype, w.grad.shape)
