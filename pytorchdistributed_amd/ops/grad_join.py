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

from typing import Optional, Union

import torch


class MaskedGrad:
    """A gradient held as ``grad * mask`` without materialising it: ``grad`` (bf16) and the ReLU bit
    mask ``bits`` (uint8, bit j of byte v masks element 8v + j) written by the BN+residual+ReLU
    forward.  A bottleneck's residual-branch gradient is exactly this (dres = dz * relu_mask), so the
    BN backward skips writing dres and conv1's dgrad epilogue reads dz + the 1-bit mask instead
    (one full-activation store fewer per identity block)."""

    __slots__ = ("grad", "bits")

    def __init__(self, grad: torch.Tensor, bits: torch.Tensor):
        self.grad, self.bits = grad, bits

    def materialize(self) -> torch.Tensor:
        shifts = torch.arange(8, device=self.bits.device, dtype=torch.uint8)
        mask = ((self.bits.reshape(-1, 1) >> shifts) & 1).bool().reshape(self.grad.shape)
        return torch.where(mask, self.grad, torch.zeros((), dtype=self.grad.dtype, device=self.grad.device))


def _dense(g):
    return g.materialize() if isinstance(g, MaskedGrad) else g


class GradJoin:
    def __init__(self, consumers: int = 2):
        self.consumers = consumers
        self.arrived = 0
        self.pending: Optional[torch.Tensor] = None

    def is_last(self) -> bool:
        """True when the calling consumer is the last one still to contribute."""
        return self.arrived == self.consumers - 1

    def take(self) -> Optional[Union[torch.Tensor, MaskedGrad]]:
        """Last contributor: the accumulated gradient of the others (None if they contributed zero);
        a :class:`MaskedGrad` when a single masked contribution is pending."""
        p = self.pending
        self.pending = None
        self.arrived = 0  # ready for a second backward over the same graph
        return p

    def stash(self, g: Optional[Union[torch.Tensor, MaskedGrad]]):
        """Non-last contributor: keep ``g`` for the last one; the caller returns None to autograd."""
        if g is not None:
            self.pending = g if self.pending is None else _dense(self.pending) + _dense(g)
        self.arrived += 1

    def contribute(self, g: Optional[torch.Tensor]) -> Optional[torch.Tensor]:
        """Generic contributor without a fused path: stash, or (last) return the total."""
        if not self.is_last():
            self.stash(g)
            return None
        p = self.take()
        if p is None:
            return _dense(g)
        return _dense(p) if g is None else _dense(g) + _dense(p)


class BnBwdStats:
    """Hand-off of a BatchNorm's backward reduction to the data gradient of the conv that consumes the
    BN's ReLU output.  The BN forward creates it and attaches it to its output tensor
    (``y._pda_bnb``); the consuming conv picks it up in its forward, and in backward its dgrad epilogue
    accumulates sum(g) and sum(g (z - mean)) with g = dx * relu_mask into ``table`` — dx IS the BN's dy —
    and sets ``filled``.  The BN backward then finalizes from the table instead of re-reading dy and z
    in a reduce pass.

    ``needs_join``: the BN output has a second consumer (the residual shortcut), so its gradient is only
    complete in the dgrad of the LAST consumer of the shared gradient join (the one whose epilogue adds
    the other consumers' stashed gradients)."""

    __slots__ = ("z", "ss", "bits", "mean", "table", "needs_join", "token", "z2", "mean2", "table2", "dx", "dx_ver")

    def __init__(self, z, ss, bits, mean, table, needs_join: bool, token=None, second=None):
        self.z, self.ss, self.bits, self.mean, self.table = z, ss, bits, mean, table
        self.needs_join = needs_join
        # second BN fed by the same masked gradient (relu(bn(z) + bn2(z2))): (z2, mean2, table2)
        self.z2, self.mean2, self.table2 = second if second is not None else (None, None, None)
        # [filled] flags shared with the tables' owners (BatchNorm2d), which re-zero a table a dgrad filled
        # but no BN backward consumed (an aborted backward) before handing it out again (one per table)
        if token is None:
            token = [False]
        self.token = list(token) if isinstance(token, tuple) else [token]
        self.filled = False
        self.dx, self.dx_ver = None, -1

    def mark_filled(self, dx: torch.Tensor):
        """The dgrad that produced ``dx`` filled the table(s) from it.  ``dx`` is held so the BN backward
        can check that its incoming gradient IS this tensor, unmodified (:meth:`take_if_matches`)."""
        self.dx, self.dx_ver = dx, dx._version
        self.filled = True

    def take_if_matches(self, dy: torch.Tensor) -> bool:
        """BN backward: True when the tables hold the sums of exactly ``dy``.  If the BN output had a
        consumer besides the fused conv (an auxiliary head, a hook, a user model reusing the block),
        autograd summed its gradient into a different tensor or bumped dx's version in place: the tables
        then miss that contribution, so they are re-zeroed and False sends the caller to the reduce pass.
        Either way the flag is cleared and the hold on dx released."""
        if not self.filled:
            return False
        dx, ver = self.dx, self.dx_ver
        self.dx, self.dx_ver = None, -1
        self.filled = False
        if (dx is not None and dy.data_ptr() == dx.data_ptr() and dy.shape == dx.shape and dy._version == ver):
            return True
        self.table.zero_()
        if self.table2 is not None:
            self.table2.zero_()
        return False

    @property
    def filled(self) -> bool:
        return self.token[0][0]

    @filled.setter
    def filled(self, v: bool):
        for t in self.token:
            t[0] = bool(v)

    def usable(self, join_last: bool, has_join: bool, stride: int, addend) -> bool:
        """May the dgrad of a conv (the last contributor of its gradient join or not, stride, epilogue
        addend) fill the table?"""
        if self.z is None:
            return False
        if self.needs_join and not (has_join and join_last):
            return False
        # a strided dgrad writes the phases no tap reaches with a fill kernel: with an addend those
        # elements are nonzero and would be missing from the sums
        return stride == 1 or addend is None

    def dgrad_kwargs(self) -> dict:
        kw = dict(bst_z=self.z, bst_mean=self.mean, bst_table=self.table)
        if self.bits is not None:
            kw["bst_bits"] = self.bits
        else:
            kw["bst_ss"] = self.ss
        if self.z2 is not None:
            kw.update(bst_z2=self.z2, bst_mean2=self.mean2, bst_table2=self.table2)
        return kw
