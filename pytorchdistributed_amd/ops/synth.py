"""On-device random fills — counter-based Philox, deterministic per (seed, offset)."""
from __future__ import annotations

import torch

from .._native import C


def _cpu_gen(seed, offset):
    g = torch.Generator()
    g.manual_seed((int(seed) * 1000003 + int(offset)) & 0x7FFFFFFFFFFFFFFF)
    return g


def fill_normal_(t: torch.Tensor, mean=0.0, std=1.0, seed=0, offset=0):
    if t.is_cuda:
        C().fill_random(t, seed, offset, 1, mean, std)
    else:
        t.copy_(torch.randn(t.shape, generator=_cpu_gen(seed, offset)) * std + mean)
    return t


def fill_uniform_(t: torch.Tensor, low=0.0, high=1.0, seed=0, offset=0):
    if t.is_cuda:
        C().fill_random(t, seed, offset, 0, low, high)
    else:
        t.copy_(torch.rand(t.shape, generator=_cpu_gen(seed, offset)) * (high - low) + low)
    return t


def fill_randint_(t: torch.Tensor, low: int, high: int, seed=0, offset=0):
    if t.is_cuda:
        C().fill_randint(t, seed, offset, low, high)
    else:
        t.copy_(torch.randint(low, high, t.shape, generator=_cpu_gen(seed, offset)))
    return t
