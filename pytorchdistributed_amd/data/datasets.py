"""The reference's synthetic datasets plus the BASELINE-config ones (CPU-resident, map-style).

* :class:`MyTrainDataset` — `ddp_gpus.py:57-66`: ``size`` tuples ``(rand(20), rand(1))``.  The reference
  leaves it unseeded (so torchrun ranks see different data); here ``seed`` defaults to 0
  so every rank builds the same data.
* :class:`SimpleDataset` — `01_multi_gpus_data_parallelism.ipynb` raw lines 52-61: ``randn(size, 10)``
  inputs and ``randint(0, 1, (size, 5))`` labels (all zero).
* :class:`SyntheticMNIST` — BASELINE config 1 (28x28 grey images, 10 classes).
* :class:`SyntheticTokens` — language-model token blocks.
* :func:`random_image_batch` — `03_model_parallel.ipynb` raw lines 374-378 ``generate_random_data``.
"""
from __future__ import annotations

import torch
from torch.utils.data import Dataset


class MyTrainDataset(Dataset):
    def __init__(self, size: int, seed: int | None = 0, in_features: int = 20, out_features: int = 1):
        g = torch.Generator()
        if seed is not None:
            g.manual_seed(seed)
        else:
            g.seed()
        self.size = size
        x = torch.rand(size, in_features, generator=g)
        y = torch.rand(size, out_features, generator=g)
        self.data = [(x[i], y[i]) for i in range(size)]

    def __len__(self):
        return self.size

    def __getitem__(self, index):
        return self.data[index]


class SimpleDataset(Dataset):
    def __init__(self, size: int = 1000, input_size: int = 10, output_size: int = 5, seed: int = 0):
        g = torch.Generator()
        g.manual_seed(seed)
        self.data = torch.randn(size, input_size, generator=g)
        self.labels = torch.randint(0, 1, (size, output_size), generator=g)

    def __len__(self):
        return len(self.data)

    def __getitem__(self, idx):
        return self.data[idx], self.labels[idx]


class SyntheticMNIST(Dataset):
    def __init__(self, size: int = 60000, seed: int = 0, num_classes: int = 10):
        g = torch.Generator()
        g.manual_seed(seed)
        self.images = torch.rand(size, 1, 28, 28, generator=g)
        self.labels = torch.randint(0, num_classes, (size,), generator=g)

    def __len__(self):
        return len(self.labels)

    def __getitem__(self, i):
        return self.images[i], self.labels[i]


class SyntheticTokens(Dataset):
    def __init__(self, num_seqs: int, seq_len: int, vocab: int, seed: int = 0):
        g = torch.Generator()
        g.manual_seed(seed)
        self.tokens = torch.randint(0, vocab, (num_seqs, seq_len + 1), generator=g)

    def __len__(self):
        return len(self.tokens)

    def __getitem__(self, i):
        t = self.tokens[i]
        return t[:-1], t[1:]


def random_image_batch(batch_size: int = 120, image_hw=(128, 128), num_classes: int = 1000, generator=None):
    """The reference's ``generate_random_data``: randn images + float one-hot labels (CPU)."""
    inputs = torch.randn(batch_size, 3, *image_hw, generator=generator)
    labels = torch.randint(0, num_classes, (batch_size,), generator=generator).view(batch_size, 1)
    one_hot = torch.zeros(batch_size, num_classes).scatter_(1, labels, 1)
    return inputs, one_hot
