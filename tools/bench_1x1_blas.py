"""ResNet-50 (bs 256) 1x1 stride-1 convolutions as plain GEMMs: hipBLASLt (torch.mm) vs the native
conv kernels, for fwd / dgrad / wgrad.  Decides which 1x1 convs may route to the library."""
import json
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from pytorchdistributed_amd._native import C  # noqa: E402

SHAPES = [(56, 64, 64), (56, 64, 256), (56, 256, 64), (28, 128, 512), (28, 512, 128), (14, 256, 1024),
          (14, 1024, 256), (7, 512, 2048), (7, 2048, 512)]


def t(fn, it=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it * 1000


for H, Ci, Co in SHAPES:
    M = 256 * H * H
    x = torch.randn(256, H, H, Ci, device="cuda").to(torch.bfloat16)
    w = (torch.randn(Co, 1, 1, Ci, device="cuda") * 0.05).to(torch.bfloat16)
    dy = torch.randn(256, H, H, Co, device="cuda").to(torch.bfloat16)
    x2, w2, dy2 = x.view(M, Ci), w.view(Co, Ci), dy.view(M, Co)
    dwo = torch.empty(Co, 1, 1, Ci, device="cuda", dtype=torch.float32)
    r = {"H": H, "Cin": Ci, "Cout": Co,
         "fwd_native_us": t(lambda: C().conv_fwd(x, w, 1, 0, 1, None, False)),
         "fwd_blas_us": t(lambda: torch.mm(x2, w2.t())),
         "dgrad_native_us": t(lambda: C().conv_dgrad(dy, w, H, H, 1, 0, 1, None)),
         "dgrad_blas_us": t(lambda: torch.mm(dy2, w2)),
         "wgrad_native_us": t(lambda: C().conv_wgrad(dy, x, 1, 1, 1, 0, 1, True, dwo)),
         "wgrad_blas_us": t(lambda: torch.mm(dy2.t(), x2, out_dtype=torch.float32)
                            if "out_dtype" in torch.mm.__doc__ else torch.mm(dy2.t(), x2))}
    print(json.dumps({k: (round(v, 1) if isinstance(v, float) else v) for k, v in r.items()}), flush=True)
