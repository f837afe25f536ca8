"""Fused optimizers (SURVEY §2.5 K09 SGD — reference `optim.SGD(lr=1e-3)` `ddp_gpus.py:78`;
K10 Adam — reference `optim.Adam(lr=1e-3)` `03_model_parallel.ipynb` raw line 383; K25 grad-norm clip).

Parameters that live in a :class:`~pytorchdistributed_amd.parallel.flat.FlatGroup` (DDP / FSDP
wrap them) are updated by ONE kernel launch per group: fp32 master + optimizer state are flat
buffers, gradients are read straight from the (already averaged) bucket buffer, and the bf16 working
copy is written in the same pass.  Other GPU parameters take the same kernel per tensor; CPU
parameters use the reference PyTorch math (identical update rule).
"""
from .fused import SGD, Adam, AdamW, clip_grad_norm_  # noqa: F401
