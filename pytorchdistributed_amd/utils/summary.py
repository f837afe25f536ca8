"""Layer table with output shapes, parameter counts and memory estimate — the ``torchsummary.summary``
the reference calls on ResNet-50 (`03_model_parallel.ipynb` raw lines 107-110, 314-315; totals
25,557,032 params / 97.49 MB params / 93.59 MB fwd+bwd activations at 3x128x128, raw lines 301-308).

    from pytorchdistributed_amd.utils.summary import summary
    print(summary(resnet50(), (3, 128, 128)))          # NCHW input size, batch 1, like torchsummary

Forward hooks record every leaf module's output; the activation estimate follows torchsummary's
convention (sum of leaf outputs x 2 for forward + backward, fp32 bytes, batch of one).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List, Sequence, Tuple

import torch
import torch.nn as tnn


@dataclass
class SummaryRow:
    name: str
    kind: str
    out_shape: Tuple[int, ...]
    params: int


@dataclass
class Summary:
    rows: List[SummaryRow] = field(default_factory=list)
    total_params: int = 0
    trainable_params: int = 0
    input_mb: float = 0.0
    activations_mb: float = 0.0
    params_mb: float = 0.0

    @property
    def total_mb(self) -> float:
        return self.input_mb + self.activations_mb + self.params_mb

    def __str__(self) -> str:
        w = max([len(r.kind) + len(r.name) + 3 for r in self.rows] + [24])
        lines = ["-" * (w + 42), f"{'Layer (type)':>{w}}  {'Output Shape':>25}  {'Param #':>12}", "=" * (w + 42)]
        for r in self.rows:
            shape = "[-1, " + ", ".join(str(d) for d in r.out_shape[1:]) + "]"
            lines.append(f"{r.kind + '-' + r.name:>{w}}  {shape:>25}  {r.params:>12,}")
        lines += ["=" * (w + 42),
                  f"Total params: {self.total_params:,}",
                  f"Trainable params: {self.trainable_params:,}",
                  f"Non-trainable params: {self.total_params - self.trainable_params:,}",
                  "-" * (w + 42),
                  f"Input size (MB): {self.input_mb:.2f}",
                  f"Forward/backward pass size (MB): {self.activations_mb:.2f}",
                  f"Params size (MB): {self.params_mb:.2f}",
                  f"Estimated Total Size (MB): {self.total_mb:.2f}",
                  "-" * (w + 42)]
        return "\n".join(lines)


def summary(model: tnn.Module, input_size: Sequence[int], batch_size: int = 1, device=None,
            dtype=torch.float32) -> Summary:
    """``input_size`` excludes the batch dim (NCHW for image models, as torchsummary)."""
    device = device or next(model.parameters()).device
    out = Summary()
    hooks = []
    order = []

    def hook(mod, inp, outp):
        t = outp[0] if isinstance(outp, (tuple, list)) else outp
        if not isinstance(t, torch.Tensor):
            return
        shape = tuple(t.shape)
        if t.dim() == 4 and getattr(model, "nhwc", False):
            # the native ResNet runs NHWC; report NCHW like torchsummary
            shape = (shape[0], shape[3], shape[1], shape[2])
        n = sum(p.numel() for p in mod.parameters(recurse=False))
        order.append(SummaryRow(names[mod], type(mod).__name__, shape, n))

    names = {}
    for name, mod in model.named_modules():
        if len(list(mod.children())) == 0:
            names[mod] = name or type(mod).__name__
            hooks.append(mod.register_forward_hook(hook))
    x = torch.zeros(batch_size, *input_size, device=device, dtype=dtype)
    was_training = model.training
    model.eval()
    try:
        with torch.no_grad():
            model(x)
    finally:
        model.train(was_training)
        for h in hooks:
            h.remove()
    out.rows = order
    out.total_params = sum(p.numel() for p in model.parameters())
    out.trainable_params = sum(p.numel() for p in model.parameters() if p.requires_grad)
    fp32 = 4.0 / 2 ** 20
    out.input_mb = x.numel() / batch_size * fp32
    out.activations_mb = 2 * sum(int(torch.tensor(r.out_shape[1:]).prod()) for r in order) * fp32
    out.params_mb = out.total_params * fp32
    return out
