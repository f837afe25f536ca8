"""Debug: every Int8Linear call of a quantized tiny Llama generate vs dequantised fp32 math."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorchdistributed_amd.models.llama import llama  # noqa: E402
from pytorchdistributed_amd.ops import quant  # noqa: E402
from pytorchdistributed_amd.serving import generate  # noqa: E402

torch.manual_seed(0)
m = llama("llama3-tiny", n_heads=4, n_kv_heads=2, dim=256, ffn_dim=512, device="cuda", dtype=torch.bfloat16).eval()
quant.quantize_linears(m, head=True)
orig = quant.w8_linear


def checked(x, q, s, b=None):
    y = orig(x, q, s, b)
    ref = x.float().reshape(-1, q.shape[1]) @ (q.float() * s[:, None]).t()
    err = (y.float().reshape(ref.shape) - ref).abs().max().item() / (ref.abs().max().item() + 1e-6)
    print(f"M={x.numel() // q.shape[1]} N={q.shape[0]} K={q.shape[1]} stride={tuple(x.stride())} rel_err={err:.4f}")
    return y


quant.w8_linear = checked
prompt = torch.randint(0, 1024, (4, 24), device="cuda")
generate(m, prompt, 3)
