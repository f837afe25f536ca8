"""Run one conv op (fwd | dgrad | wgrad) of one ResNet shape repeatedly — the unit of work for
rocprofv3 PMC counter collection:

    rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS --kernel-trace -- python tools/conv_one.py wgrad 14 256 256 3 1
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorchdistributed_amd._native import C  # noqa: E402


def main():
    op, H, Ci, Co, R, st = sys.argv[1], *map(int, sys.argv[2:7])
    iters = int(sys.argv[7]) if len(sys.argv) > 7 else 10
    N, pad = 256, R // 2
    P = (H + 2 * pad - R) // st + 1
    x = torch.randn(N, H, H, Ci, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(Co, R, R, Ci, device="cuda", dtype=torch.bfloat16) * 0.05
    dy = torch.randn(N, P, P, Co, device="cuda", dtype=torch.bfloat16)
    dwo = torch.empty(Co, R, R, Ci, device="cuda", dtype=torch.float32)
    for _ in range(iters):
        if op == "fwd":
            C().conv_fwd(x, w, st, pad, 1, None, False)
        elif op == "dgrad":
            C().conv_dgrad(dy, w, H, H, st, pad, 1, None)
        else:
            C().conv_wgrad(dy, x, R, R, st, pad, 1, True, dwo)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
