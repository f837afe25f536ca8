"""Small models of the reference tutorial and the CPU plumbing config.

* :class:`TutorialMLP` — the DataParallel demo model (`01 数据并行/01_multi_gpus_data_parallelism.ipynb`
  raw lines 94-107): fc1 10->20, fc2 20->20, fc3 20->20, fc4 20->5, ReLU after fc1-fc3 (1,165 params;
  ``num_layers`` is accepted and unused, as in the reference).
* :func:`linear_20_1` — the DDP demo model ``nn.Linear(20, 1)`` (`ddp_gpus.py:77`).
* :class:`MnistMLP` — BASELINE config 1 (MNIST-shaped MLP 784-512-256-10).
"""
from __future__ import annotations

import torch.nn as tnn

from .. import nn as pnn


class TutorialMLP(tnn.Module):
    def __init__(self, input_size=10, hidden_size=20, output_size=5, num_layers=2, device=None, dtype=None):
        super().__init__()
        kw = dict(device=device, dtype=dtype)
        self.fc1 = pnn.Linear(input_size, hidden_size, relu=True, **kw)
        self.fc2 = pnn.Linear(hidden_size, hidden_size, relu=True, **kw)
        self.fc3 = pnn.Linear(hidden_size, hidden_size, relu=True, **kw)
        self.fc4 = pnn.Linear(hidden_size, output_size, **kw)

    def forward(self, x):
        return self.fc4(self.fc3(self.fc2(self.fc1(x))))


def linear_20_1(device=None, dtype=None) -> pnn.Linear:
    return pnn.Linear(20, 1, device=device, dtype=dtype)


class MnistMLP(tnn.Module):
    def __init__(self, sizes=(784, 512, 256, 10), device=None, dtype=None):
        super().__init__()
        layers = []
        for i in range(len(sizes) - 1):
            last = i == len(sizes) - 2
            layers.append(pnn.Linear(sizes[i], sizes[i + 1], relu=not last, device=device, dtype=dtype))
        self.net = tnn.Sequential(*layers)

    def forward(self, x):
        return self.net(x.reshape(x.shape[0], -1))
