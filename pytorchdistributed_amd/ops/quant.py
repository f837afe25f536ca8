"""Weight-only int8 for serving (the reference's ``load_in_8bit=True``
Llama, `03 模型并行/03_model_parallel.ipynb` raw line 86).

Measured on MI355X (`profiles/r1_w8_gemm_microbench_v3.jsonl`, `r1_llama3_8b_serve_int8_v2.jsonl`): the
kernel streams int8 at 3-4.9 TB/s at M <= 16 (1.3-3.7x the bf16 GEMM on wqkv / wo / w13 / LM head;
w2 at 2.2-2.6 TB/s), falling off at M >= 32 where the activation re-reads from L2 grow.  Llama-3-8B
decode: bs 8 all-int8 4.29 ms/step vs 5.38 bf16 (+25 %); bs 32 w13 + head int8 5.34 vs 5.89 (+10 %),
all-int8 5.74.  Halving the resident weight bytes also lets 2x larger models (or KV caches) fit.

Per-output-row symmetric quantisation (``scale = absmax / 127``).  Decode steps (<= 64 token rows) run
the int8-streaming MFMA kernel `csrc/kernels/w8_gemm.hip` (half the weight bytes of bf16 — the decode
step is weight-bandwidth bound); prefills (many rows) dequantise the layer's weight to bf16 once and
take the regular GEMM path; CPU uses reference math.
"""
from __future__ import annotations

from typing import Dict, Iterable, Optional

import torch
import torch.nn as tnn

from .._native import C
from .linear import linear

_WS: Dict[torch.device, list] = {}  # device -> [fp32 split-K slabs, int32 tickets (zero between calls)]


def _workspace(device: torch.device, N: int):
    """Per-device scratch for w8_gemm (only used with explicit split-K): 8 x 64 x N fp32 partial slabs
    and N/16 tickets.  Grown (never
    during HIP-graph capture: the warm-up step allocates it) and shared by every call on the device —
    calls are stream-ordered and each leaves the tickets zeroed."""
    ent = _WS.get(device)
    if ent is None or ent[0].numel() < 8 * 64 * N:
        ent = _WS[device] = [torch.empty(8 * 64 * N, dtype=torch.float32, device=device),
                             torch.zeros((N + 15) // 16, dtype=torch.int32, device=device)]
    return ent


@torch.no_grad()
def quantize_int8(w: torch.Tensor):
    """[N, K] float weight -> (int8 [N, K], fp32 scale [N]) with w ~= q * scale[:, None]."""
    wf = w.float()
    scale = wf.abs().amax(1).clamp_min(1e-12) / 127.0
    q = torch.round(wf / scale[:, None]).clamp_(-127, 127).to(torch.int8)
    return q.contiguous(), scale.contiguous()


def w8_linear(x: torch.Tensor, q: torch.Tensor, scale: torch.Tensor, bias: Optional[torch.Tensor] = None):
    N, K = q.shape
    rows = x.numel() // K
    if (x.is_cuda and x.dtype == torch.bfloat16 and rows <= 64 and N % 16 == 0 and K % 256 == 0
            and x.stride(-1) == 1):
        ws, tk = _workspace(x.device, N)
        y = C().w8_gemm(x.contiguous(), q, scale, ws, tk)
        return y + bias if bias is not None else y
    if x.is_cuda:
        w = (q.to(x.dtype) * scale[:, None].to(x.dtype))
        return linear(x, w, bias)
    y = x.float() @ (q.float() * scale[:, None]).t()
    if bias is not None:
        y = y + bias.float()
    return y.to(x.dtype)


class Int8Linear(tnn.Module):
    """Inference-only replacement of a Linear: int8 weight + per-row scale (+ the original bias)."""

    def __init__(self, q: torch.Tensor, scale: torch.Tensor, bias: Optional[torch.Tensor] = None):
        super().__init__()
        self.register_buffer("q", q)
        self.register_buffer("scale", scale)
        self.bias = None if bias is None else tnn.Parameter(bias.detach(), requires_grad=False)
        self.out_features, self.in_features = q.shape

    @classmethod
    def from_linear(cls, lin: tnn.Module) -> "Int8Linear":
        q, s = quantize_int8(lin.weight)
        return cls(q, s, getattr(lin, "bias", None))

    @property
    def device(self) -> torch.device:
        return self.q.device

    @property
    def weight(self) -> torch.Tensor:
        """The DEQUANTISED weight (``q * scale``, bf16 on a GPU / fp32 on the CPU), computed on every
        access — for code that genuinely needs the float weight.  Hot paths use ``forward`` or
        ``q``/``scale``; placement code uses :attr:`device`."""
        dt = torch.bfloat16 if self.q.is_cuda else torch.float32
        return self.q.to(dt) * self.scale[:, None].to(dt)

    def forward(self, x):
        return w8_linear(x, self.q, self.scale, self.bias)


@torch.no_grad()
def quantize_linears(model: tnn.Module, names: Iterable[str] = ("wqkv", "wo", "w13", "w2", "c_attn", "attn_proj",
                                                                "c_fc", "mlp_proj"),
                     head: bool = False) -> int:
    """Replace the named Linear sub-modules of every transformer block (and the LM head ``output`` when
    ``head``) by :class:`Int8Linear`, in place.  Returns the number of layers quantised."""
    n = 0
    for blk in model.layers:
        for name in names:
            lin = getattr(blk, name, None)
            if lin is not None and hasattr(lin, "weight") and not isinstance(lin, Int8Linear):
                setattr(blk, name, Int8Linear.from_linear(lin))
                n += 1
    if head and hasattr(model, "output") and not isinstance(model.output, Int8Linear):
        model.output = Int8Linear.from_linear(model.output)
        n += 1
    return n
