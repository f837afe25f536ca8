"""DistributedSampler with index streams identical to ``torch.utils.data.DistributedSampler``
(reference `ddp_gpus.py:76`, `ddp_gpus_torchrun.py:72`, ``set_epoch`` at
`ddp_gpus.py:47`).

Semantics: pad to ``ceil(N / W) * W`` by wrapping around (or truncate with ``drop_last``), permute
with a CPU generator seeded ``seed + epoch`` when shuffling, rank ``r`` takes ``indices[r::W]``.
"""
from __future__ import annotations

import math
from typing import Iterator, Optional

import torch
from torch.utils.data import Sampler

from .. import distributed as pdist


class DistributedSampler(Sampler):
    def __init__(self, dataset, num_replicas: Optional[int] = None, rank: Optional[int] = None,
                 shuffle: bool = True, seed: int = 0, drop_last: bool = False):
        if num_replicas is None:
            num_replicas = pdist.get_world_size()
        if rank is None:
            rank = pdist.get_rank()
        if rank >= num_replicas or rank < 0:
            raise ValueError(f"Invalid rank {rank}, rank should be in the interval [0, {num_replicas - 1}]")
        self.dataset = dataset
        self.num_replicas = num_replicas
        self.rank = rank
        self.epoch = 0
        self.drop_last = drop_last
        n = len(dataset)
        if self.drop_last and n % self.num_replicas != 0:
            self.num_samples = math.ceil((n - self.num_replicas) / self.num_replicas)
        else:
            self.num_samples = math.ceil(n / self.num_replicas)
        self.total_size = self.num_samples * self.num_replicas
        self.shuffle = shuffle
        self.seed = seed

    def __iter__(self) -> Iterator[int]:
        n = len(self.dataset)
        if self.shuffle:
            g = torch.Generator()
            g.manual_seed(self.seed + self.epoch)
            indices = torch.randperm(n, generator=g).tolist()
        else:
            indices = list(range(n))
        if not self.drop_last:
            pad = self.total_size - len(indices)
            if pad <= len(indices):
                indices += indices[:pad]
            else:
                indices += (indices * math.ceil(pad / len(indices)))[:pad]
        else:
            indices = indices[: self.total_size]
        assert len(indices) == self.total_size
        indices = indices[self.rank: self.total_size: self.num_replicas]
        assert len(indices) == self.num_samples
        return iter(indices)

    def __len__(self) -> int:
        return self.num_samples

    def set_epoch(self, epoch: int) -> None:
        self.epoch = epoch
