"""Per-launch kernels of the strided conv dgrads (phase launches) at bs 640, for rocprofv3 --stats."""
import os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorchdistributed_amd._native import C
for (H, Ci, Co, R, st) in [(56, 256, 512, 1, 2), (56, 128, 128, 3, 2)]:
    pad = R // 2
    P = (H + 2 * pad - R) // st + 1
    dy = torch.randn(640, P, P, Co, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(Co, R, R, Ci, device="cuda", dtype=torch.bfloat16) * 0.05
    for _ in range(10):
        C().conv_dgrad(dy, w, H, H, st, pad, 1, None)
    torch.cuda.synchronize()
print("done")
