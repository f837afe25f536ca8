"""Gradient joins: fuse the accumulation of a tensor's gradient from several consumers into the
kernel of the last consumer to run its backward.

Autograd sums the gradients a tensor receives from its consumers with a separate elementwise add
(read 2, write 1).  In a ResNet bottleneck the block input feeds conv1 and the shortcut, so every
block paid a full-activation add in backward (1.3 ms/step at bs 256, `profiles/`).  A
:class:`GradJoin` shared by the consumers' autograd Functions lets the earlier ones *stash* their
gradient (returning ``None`` = zero to autograd) and the last one fold the stash into its own
output — for conv1's dgrad, as the epilogue addend of the MFMA kernel.
"""
from __future__ import annotations

from typing import Optional

import torch


class GradJoin:
    def __init__(self, consumers: int = 2):
        self.consumers = consumers
        self.arrived = 0
        self.pending: Optional[torch.Tensor] = None

    def is_last(self) -> bool:
        """True when the calling consumer is the last one still to contribute."""
        return self.arrived == self.consumers - 1

    def take(self) -> Optional[torch.Tensor]:
        """Last contributor: the accumulated gradient of the others (None if they contributed zero)."""
        p = self.pending
        self.pending = None
        self.arrived = 0  # ready for a second backward over the same graph
        return p

    def stash(self, g: Optional[torch.Tensor]):
        """Non-last contributor: keep ``g`` for the last one; the caller returns None to autograd."""
        if g is not None:
            self.pending = g if self.pending is None else self.pending + g
        self.arrived += 1

    def contribute(self, g: Optional[torch.Tensor]) -> Optional[torch.Tensor]:
        """Generic contributor without a fused path: stash, or (last) return the total."""
        if not self.is_last():
            self.stash(g)
            return None
        p = self.take()
        if p is None:
            return g
        return p if g is None else g + p
