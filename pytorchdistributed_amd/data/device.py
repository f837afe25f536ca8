"""On-device data: synthetic batch generators (HBM-resident, Philox kernel) and a side-stream
prefetcher for host datasets.

The benchmark configs use :class:`DeviceSyntheticImages` / :class:`DeviceSyntheticTokens`: each step's
batch is generated directly in HBM in the model's layout (channels-last images with channels padded
to 8 for the stem's 16-byte gathers), deterministic per (seed, rank, step), so no host RNG or PCIe copy
sits in the timed region.  Host datasets go through :class:`DevicePrefetcher`, which copies batch k+1
from pinned memory on a separate HIP stream while batch k computes.
"""
from __future__ import annotations

from typing import Iterable, Iterator, Optional

import torch

from ..ops.synth import fill_normal_, fill_randint_


class DeviceSyntheticImages:
    """Yields ``(images [B,H,W,pad_channels] bf16, labels [B] int64)`` generated on ``device``."""

    def __init__(self, batch_size: int, image_size: int = 224, num_classes: int = 1000, steps: Optional[int] = None,
                 device="cuda", dtype=torch.bfloat16, channels: int = 3, pad_channels: int = 3, seed: int = 0,
                 rank: int = 0, fixed: bool = False, nchw: bool = False):
        self.B, self.S, self.K = batch_size, image_size, num_classes
        self.steps, self.device, self.dtype = steps, torch.device(device), dtype
        self.C, self.Cp = channels, (pad_channels if self.device.type == "cuda" else channels)
        self.seed, self.rank, self.fixed, self.nchw = seed, rank, fixed, nchw
        shape = (self.B, self.C, self.S, self.S) if nchw else (self.B, self.S, self.S, self.Cp)
        self._x = torch.zeros(shape, device=self.device, dtype=dtype)
        self._y = torch.empty(self.B, device=self.device, dtype=torch.long)
        self._step = 0
        if fixed:
            self._fill(0)

    def _fill(self, step: int):
        off = (self.rank * 1_000_003 + step) * (1 << 24)
        # The padding channels (C..Cp-1) are filled too: the stem multiplies them by zero-padded weight
        # columns, so their values never reach the output and one contiguous fill is cheapest.
        fill_normal_(self._x, 0.0, 1.0, self.seed, off)
        fill_randint_(self._y, 0, self.K, self.seed + 1, off)

    def __len__(self):
        return self.steps if self.steps is not None else 0

    def next(self):
        if not self.fixed:
            self._fill(self._step)
        self._step += 1
        return self._x, self._y

    def __iter__(self) -> Iterator:
        n = 0
        while self.steps is None or n < self.steps:
            yield self.next()
            n += 1


class DeviceSyntheticTokens:
    """Yields ``(tokens [B,T], targets [B,T])`` int64 generated on ``device``."""

    def __init__(self, batch_size: int, seq_len: int, vocab: int, device="cuda", seed: int = 0, rank: int = 0,
                 fixed: bool = False):
        self.B, self.T, self.V = batch_size, seq_len, vocab
        self.device, self.seed, self.rank, self.fixed = torch.device(device), seed, rank, fixed
        self._buf = torch.empty(self.B, self.T + 1, device=self.device, dtype=torch.long)
        self._step = 0
        if fixed:
            fill_randint_(self._buf, 0, self.V, self.seed, self.rank * (1 << 32))

    def next(self):
        if not self.fixed:
            fill_randint_(self._buf, 0, self.V, self.seed, self.rank * (1 << 32) + self._step * (1 << 24))
        self._step += 1
        return self._buf[:, :-1], self._buf[:, 1:]


class DevicePrefetcher:
    """Wrap a host iterable of tensors / tuples: pin, copy to ``device`` on a side stream one batch ahead."""

    def __init__(self, loader: Iterable, device, non_blocking: bool = True):
        self.loader, self.device = loader, torch.device(device)
        self.stream = torch.cuda.Stream(self.device) if self.device.type == "cuda" else None
        self.non_blocking = non_blocking

    def _to(self, b):
        if isinstance(b, torch.Tensor):
            if self.stream is not None and not b.is_pinned():
                b = b.pin_memory()
            return b.to(self.device, non_blocking=self.non_blocking)
        if isinstance(b, (list, tuple)):
            return type(b)(self._to(x) for x in b)
        return b

    def __len__(self):
        return len(self.loader)

    def __iter__(self):
        it = iter(self.loader)
        if self.stream is None:
            for b in it:
                yield self._to(b)
            return
        nxt = None
        try:
            with torch.cuda.stream(self.stream):
                nxt = self._to(next(it))
        except StopIteration:
            return
        while nxt is not None:
            torch.cuda.current_stream(self.device).wait_stream(self.stream)
            cur = nxt
            _record(cur, torch.cuda.current_stream(self.device))
            try:
                with torch.cuda.stream(self.stream):
                    nxt = self._to(next(it))
            except StopIteration:
                nxt = None
            yield cur


def _record(b, stream):
    if isinstance(b, torch.Tensor):
        b.record_stream(stream)
    elif isinstance(b, (list, tuple)):
        for x in b:
            _record(x, stream)
