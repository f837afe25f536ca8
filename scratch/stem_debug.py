"""Stem forward kernel vs CPU fp32 reference at shapes with 1, 2 and 3 output rows per workgroup."""
import math, sys, os
import torch, torch.nn.functional as F
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorchdistributed_amd._native import C

def rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12)).item()

for (N, H) in [(2, 35), (16, 51), (8, 115), (13, 115), (40, 35)]:
    torch.manual_seed(1)
    x = torch.randn(N, H, H, 16).to(torch.bfloat16)
    w = (torch.randn(64, 4, 4, 16) / 16).to(torch.bfloat16)
    ref = F.conv2d(x.float().permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2)).permute(0, 2, 3, 1)
    outs = []
    for rep in range(3):
        y = C().conv_fwd(x.cuda(), w.cuda(), 1, 0, 1, None, False)
        torch.cuda.synchronize()
        outs.append(y.cpu())
    P = H - 3
    rows = N * P
    rps = (rows + 511) // 512
    bad = (outs[0].float() - ref).abs().reshape(N, P, P, 64).amax(dim=(2, 3))
    print(f"N={N} H={H} rows={rows} rps={rps} rel={rel(outs[0], ref):.3e} same_runs={all(torch.equal(outs[0], o) for o in outs)} worst_rows={[(int(i)//P, int(i)%P) for i in bad.flatten().topk(4).indices]} maxerr={bad.max().item():.3f}", flush=True)
