"""Where do the hot path's stray copies come from?  Runs a few GPT-2-medium DDP steps (or the ResNet-50
bench step with ``--model resnet``) under torch.profiler with Python stacks and prints, per call site,
the count of copy / cast ops (aten::copy_, aten::to/_to_copy, aten::clone, aten::contiguous) per step.

    python tools/find_copies.py [--model gpt2|resnet] [--steps 2] [--batch 8]
"""
from __future__ import annotations

import argparse
import collections
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

COPY_OPS = {"aten::copy_", "aten::_to_copy", "aten::clone", "aten::contiguous", "aten::to", "aten::cat",
            "aten::zero_", "aten::fill_", "aten::zeros", "aten::zeros_like", "aten::new_zeros"}


def gpt2_step(batch):
    from pytorchdistributed_amd.bench.gpt2_ddp import build

    return build(batch)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="gpt2", choices=["gpt2", "resnet"])
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--batch", type=int, default=8)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    if a.model == "resnet":
        from pytorchdistributed_amd.bench.resnet_ddp import build

        _, _, step = build(a.batch, 224, dev, 0)
    else:
        from pytorchdistributed_amd.data.device import DeviceSyntheticTokens
        from pytorchdistributed_amd.models.gpt2 import GPT2, config
        from pytorchdistributed_amd.optim import AdamW
        from pytorchdistributed_amd.parallel.ddp import DistributedDataParallel

        torch.manual_seed(0)
        cfg = config("gpt2-medium")
        model = DistributedDataParallel(GPT2(cfg, device=dev, dtype=torch.bfloat16), device_ids=[0])
        opt = AdamW(model.parameters(), lr=1e-4, weight_decay=0.1)
        data = DeviceSyntheticTokens(a.batch, 1024, cfg.vocab_size, device=dev)

        def step():
            x, y = data.next()
            opt.zero_grad(set_to_none=True)
            loss = model(x, targets=y)
            loss.backward()
            opt.step()
            return loss

    for _ in range(2):
        step()
    torch.cuda.synchronize()
    acts = [torch.profiler.ProfilerActivity.CPU, torch.profiler.ProfilerActivity.CUDA]
    with torch.profiler.profile(activities=acts, with_stack=True, record_shapes=False) as prof:
        for _ in range(a.steps):
            step()
        torch.cuda.synchronize()
    sites = collections.Counter()
    for ev in prof.events():
        if ev.name not in COPY_OPS:
            continue
        stack = [f for f in (ev.stack or []) if "pytorchdistributed_amd" in f or "tools/" in f]
        site = stack[0] if stack else "(no python frame)"
        sites[(ev.name, site)] += 1
    print(f"copy / cast ops per step ({a.model}):")
    for (name, site), n in sites.most_common(40):
        print(f"{n / a.steps:8.1f}  {name:18s} {site}")
    kern = collections.Counter()
    for ev in prof.events():
        if ev.device_type == torch.autograd.DeviceType.CUDA and any(t in ev.name.lower() for t in ("copy", "fill")):
            kern[ev.name[:90]] += 1
    print("device copy kernels per step:")
    for k, n in kern.most_common(10):
        print(f"{n / a.steps:8.1f}  {k}")


if __name__ == "__main__":
    main()
