"""Flat parameter / gradient storage shared by DDP, FSDP and the fused optimizers.

Every parameter of a :class:`FlatGroup` is a view into ONE contiguous parameter buffer and its
``.grad`` a view into ONE contiguous gradient buffer laid out identically (DDP buckets are slices of
it).  The optimizer then updates the whole model with one kernel launch per group, and a gradient
bucket is all-reduced in place with no flatten/unflatten copies.  Views start on 16-byte boundaries
(offsets are multiples of ``ALIGN`` elements) so every kernel can use 16-byte vector accesses.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence

import torch

ALIGN = 8  # elements (16 B for bf16, 32 B for fp32)


def _round(n: int, a: int = ALIGN) -> int:
    return (n + a - 1) // a * a


class FlatGroup:
    """Parameters of one dtype/device materialised as views of a flat buffer."""

    def __init__(self, params: Sequence[torch.nn.Parameter], offsets: Optional[Sequence[int]] = None,
                 numel: Optional[int] = None, copy_data: bool = True):
        assert len(params) > 0
        self.params: List[torch.nn.Parameter] = list(params)
        self.dtype = params[0].dtype
        self.pending_comm = 0  # bucket collectives launched but not yet waited on by the compute stream (DDP)
        self.device = params[0].device
        if offsets is None:
            offsets, off = [], 0
            for p in self.params:
                offsets.append(off)
                off += _round(p.numel())
            numel = off
        self.offsets = list(offsets)
        self.numel = int(numel)
        self.param_buffer = torch.zeros(self.numel, dtype=self.dtype, device=self.device)
        self.grad_buffer = torch.zeros(self.numel, dtype=self.dtype, device=self.device)
        for p, off in zip(self.params, self.offsets):
            assert p.dtype == self.dtype and p.device == self.device, "FlatGroup params must share dtype/device"
            view = self.param_buffer[off: off + p.numel()].view_as(p)
            if copy_data:
                view.copy_(p.detach())
            p.data = view
            p._pda_flat = (self, off)
        self.index: Dict[int, int] = {id(p): i for i, p in enumerate(self.params)}

    def grad_view(self, i: int) -> torch.Tensor:
        p, off = self.params[i], self.offsets[i]
        return self.grad_buffer[off: off + p.numel()].view_as(p)

    def attach_grads(self):
        """Point every ``p.grad`` at its slot of the flat gradient buffer."""
        for i, p in enumerate(self.params):
            p.grad = self.grad_view(i)

    def zero_grad(self):
        self.grad_buffer.zero_()
        self.attach_grads()

    def covers(self, params: Sequence[torch.nn.Parameter]) -> bool:
        return len(params) == len(self.params) and all(id(p) in self.index for p in params)


def grad_target(param: torch.Tensor) -> Optional[torch.Tensor]:
    """Where a backward kernel should write ``param``'s gradient.

    For a parameter living in a :class:`FlatGroup` whose ``.grad`` is unset, this is its slot of the
    flat gradient buffer: the kernel writes there and autograd's AccumulateGrad adopts the returned
    view as ``.grad`` without a copy (so DDP's bucket is filled in place).  Otherwise ``None``
    (allocate normally; accumulation semantics are then autograd's).
    """
    info = getattr(param, "_pda_flat", None)
    if info is None or param.grad is not None or not param.requires_grad:
        return None
    if getattr(param, "_pda_claimed", False):
        # used more than once in this graph (tied weights): only the first backward writes in place,
        # the others allocate; autograd sums them on the compute stream before AccumulateGrad (DDP's
        # hook clears the claim).  The first use may still be writing the slot on the side stream:
        # the compute stream waits for it here, and the parameter is marked shared so later passes
        # keep all of its gradients on the compute stream (ops/streams.py:side_ok).
        param._pda_shared = True
        if param.is_cuda:
            from ..ops import streams as _streams

            _streams.wait_side(param.device)
        return None
    param._pda_claimed = True
    fg, off = info
    return fg.grad_buffer[off: off + param.numel()].view_as(param)


def flat_group_of(p: torch.Tensor) -> Optional[FlatGroup]:
    info = getattr(p, "_pda_flat", None)
    return info[0] if info is not None else None


def flatten_buffers(module: torch.nn.Module) -> Dict[torch.dtype, torch.Tensor]:
    """Re-home every buffer of ``module`` as a view of one flat buffer per dtype (for coalesced
    broadcasts).  Returns ``{dtype: flat}``."""
    owners = []
    for mod in module.modules():
        for name, b in list(mod._buffers.items()):
            if b is not None:
                owners.append((mod, name, b))
    by_dtype: Dict[torch.dtype, list] = {}
    for item in owners:
        by_dtype.setdefault(item[2].dtype, []).append(item)
    flats = {}
    for dt, items in by_dtype.items():
        total = sum(_round(b.numel(), 1) for _, _, b in items)
        flat = torch.empty(total, dtype=dt, device=items[0][2].device)
        off = 0
        for mod, name, b in items:
            n = b.numel()
            view = flat[off: off + n].view_as(b)
            view.copy_(b)
            mod._buffers[name] = view
            off += n
        flats[dt] = flat
    return flats
