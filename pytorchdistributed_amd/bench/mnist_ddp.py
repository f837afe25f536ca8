"""BASELINE config 1: MNIST-shaped MLP DDP on CPU / gloo, world_size 2 — the plumbing configuration
that runs without a GPU.  Samples/sec (whole job) over a fixed synthetic MNIST set,
DistributedSampler sharding, bucketed all-reduce (gloo, or the native host ring with
``--backend ring``), SGD with momentum.

    python -m pytorchdistributed_amd.run --standalone --nproc-per-node 2 -m pytorchdistributed_amd.bench.mnist_ddp
"""
from __future__ import annotations

import argparse
import os

import torch
from torch.utils.data import DataLoader

from .. import distributed as pdist
from ..data import DistributedSampler
from ..data.datasets import SyntheticMNIST
from ..models.mlp import MnistMLP
from ..ops import cross_entropy
from ..parallel.ddp import DistributedDataParallel
from .common import emit, timed


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=64, help="per-rank batch")
    ap.add_argument("--backend", default="gloo", choices=["gloo", "ring"])
    a = ap.parse_args(argv)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    torch.set_num_threads(max(1, (os.cpu_count() or 2) // max(1, world)))
    if world > 1:
        pdist.init_process_group(a.backend)
    torch.manual_seed(0)
    ds = SyntheticMNIST(8192)
    sampler = DistributedSampler(ds, num_replicas=world, rank=rank, shuffle=True)
    loader = DataLoader(ds, batch_size=a.batch, sampler=sampler, drop_last=True)
    model = DistributedDataParallel(MnistMLP(), bucket_cap_mb=0.5, first_bucket_mb=0.1)
    opt = torch.optim.SGD(model.parameters(), lr=0.05, momentum=0.9)
    it = iter(loader)
    state = {"epoch": 0, "loss": None}

    def step():
        nonlocal it
        try:
            x, y = next(it)
        except StopIteration:
            state["epoch"] += 1
            sampler.set_epoch(state["epoch"])
            it = iter(loader)
            x, y = next(it)
        opt.zero_grad()
        loss = cross_entropy(model(x), y)
        loss.backward()
        opt.step()
        state["loss"] = loss.item()

    secs = timed(step, a.steps, a.warmup)
    emit({"metric": "samples/sec (whole job) MNIST-MLP DDP CPU", "value": round(a.batch * world * a.steps / secs, 1),
          "unit": "samples/sec", "n_gpus": 0, "n_ranks": world, "steps": a.steps, "warmup": a.warmup,
          "ms_per_step": round(secs / a.steps * 1e3, 3), "higher_is_better": True, "scaling": "weak",
          "vs_baseline": None, "dtype": "fp32", "data": "synthetic MNIST shape (seeded), random-init weights",
          "config": {"model": "mlp-784-512-256-10", "global_batch": a.batch * world, "seq_len": None,
                     "parallelism": f"dp{world}-{a.backend}"}, "final_loss": round(state["loss"], 4)}, rank)
    if world > 1:
        pdist.destroy_process_group()


if __name__ == "__main__":
    main()
