"""Reproduction of the reference's own benchmark (`03 模型并行/03_model_parallel.ipynb` raw lines 369-624;
numbers in BASELINE.md): ResNet-50, ``train(model)`` = 3 Adam steps on fresh 120 x 3x128x128 batches
with one-hot soft targets, timed with ``timeit.repeat(number=1, repeat=10)``.

Modes:
* ``parity`` — the reference's methodology: CPU data generation + pageable host->device copies inside
  the timed call, a new Adam optimizer per call; we add a final device synchronize (the reference
  stops its timer with kernels still queued) so the number is honest.
* ``clean``  — data generated on device, optimizer reused, HIP-event/synchronize bracketed.
  ``--graph`` additionally captures the step (forward, loss, backward, Adam) into one HIP graph
  (`utils/graphs.py`); every replay is a full optimizer step on a fresh device batch.
Variants: ``single`` (1 device), ``mp`` (layer split, stem..layer2 on dev0, rest on dev1), ``pp``
(micro-batch pipeline, ``--split-size``), ``sweep`` (pp over the reference's split sizes).
Precision (``--dtype``): ``fp32`` (default, the reference's precision: fp32 activations / weights /
Adam; convs on split-bf16 MFMA operands, ~1e-5 relative — the reference's A100 ran its convs in TF32,
~1e-3) or ``bf16`` (bf16 compute, fp32 master weights).
Device layout: with one visible GPU the two "devices" of mp / pp are the same GPU (``devices`` in the
output says so); the reference used two A100s.
"""
from __future__ import annotations

import argparse
import json
import timeit

import numpy as np
import torch

from ..data.datasets import random_image_batch
from ..data.device import DeviceSyntheticImages
from ..models.resnet import resnet50
from ..ops import cross_entropy
from ..optim import Adam
from ..parallel.model_parallel import ModelParallelResNet50, PipelineParallelResNet50
from ..utils.graphs import GraphedStep

REFERENCE_S = {"single": 0.248, "mp": 0.272, "pp20": 0.454,
               "sweep": {1: 4.88, 3: 1.84, 5: 1.16, 8: 0.81, 10: 0.71, 12: 0.62, 20: 0.47, 40: 0.33, 60: 0.29}}
SPLITS = [1, 3, 5, 8, 10, 12, 20, 40, 60]


def make_model(kind, devs, split=20, dtype=torch.float32):
    if kind == "single":
        return resnet50(device=devs[0], dtype=dtype), devs[0]
    base = resnet50(dtype=dtype)
    if kind == "mp":
        return ModelParallelResNet50(base, devices=devs), devs[1]
    return PipelineParallelResNet50(base, devices=devs, split_size=split), devs[1]


def run(kind, devs, mode, split=20, repeat=10, batch=120, size=128, graph=False, dtype=torch.float32):
    model, out_dev = make_model(kind, devs, split, dtype)
    in_dev = devs[0]
    dev_data = (DeviceSyntheticImages(batch, size, 1000, device=in_dev, seed=0, dtype=dtype) if mode == "clean"
                else None)
    opt_holder = {}
    if graph:
        if mode != "clean":
            raise ValueError("--graph needs --mode clean (parity re-creates the optimizer every call)")
        if kind != "single" and devs[0] != devs[1]:
            return float("nan"), float("nan")  # a HIP graph is bound to one device (see model_parallel.py)
        opt = Adam(model.parameters(), lr=1e-3)

        def step(x, y):
            opt.zero_grad(set_to_none=True)
            loss = cross_entropy(model(x), y)
            loss.backward()
            opt.step()
            return loss

        model.train()
        x0, y0 = dev_data.next()
        graphed = GraphedStep(step, (x0, y0.to(out_dev)), optimizer=opt)

        def train_graph():
            for _ in range(3):
                x, yi = dev_data.next()
                graphed(x, yi.to(out_dev))
            torch.cuda.synchronize()

        train_graph()
        times = timeit.repeat(train_graph, number=1, repeat=repeat)
        return float(np.mean(times)), float(np.std(times))

    def train():
        model.train()
        opt = Adam(model.parameters(), lr=1e-3) if mode == "parity" else opt_holder.setdefault(
            "o", Adam(model.parameters(), lr=1e-3))
        for _ in range(3):
            if mode == "parity":
                inputs, labels = random_image_batch(batch, (size, size), 1000)
                x = inputs.to(in_dev).permute(0, 2, 3, 1).to(dtype)
                y = labels.to(out_dev)
            else:
                x, yi = dev_data.next()
                y = yi.to(out_dev)
            opt.zero_grad()
            out = model(x)
            loss = cross_entropy(out, y)
            loss.backward()
            opt.step()
        torch.cuda.synchronize()

    train()  # warm-up (the reference's first timeit repeat includes it; we exclude compile/alloc effects)
    times = timeit.repeat(train, number=1, repeat=repeat)
    return float(np.mean(times)), float(np.std(times))


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="single,mp,pp")
    ap.add_argument("--mode", default="parity", choices=["parity", "clean"])
    ap.add_argument("--devices", default=None, help="comma list, e.g. 0,1 (default: 0,1 if 2 GPUs else 0,0)")
    ap.add_argument("--split-size", type=int, default=20)
    ap.add_argument("--repeat", type=int, default=10)
    ap.add_argument("--sweep", action="store_true")
    ap.add_argument("--graph", action="store_true", help="capture each step into a HIP graph (clean mode)")
    ap.add_argument("--dtype", default="fp32", choices=["fp32", "bf16"])
    a = ap.parse_args(argv)
    n = torch.cuda.device_count()
    devs = [int(d) for d in a.devices.split(",")] if a.devices else ([0, 1] if n >= 2 else [0, 0])
    devs = [torch.device("cuda", d) for d in devs]
    dtype = torch.float32 if a.dtype == "fp32" else torch.bfloat16
    results = {}
    for v in a.variants.split(","):
        m, s = run(v, devs, a.mode, a.split_size, a.repeat, graph=a.graph, dtype=dtype)
        key = "pp20" if v == "pp" and a.split_size == 20 else v
        ref = REFERENCE_S.get(key)
        results[v] = {"mean_s": round(m, 4), "std_s": round(s, 4), "img_per_s": round(360 / m, 1),
                      "reference_s_A100": ref, "speedup_vs_reference": round(ref / m, 2) if ref else None}
    if a.sweep:
        sw = {}
        for sp in SPLITS:
            m, s = run("pp", devs, a.mode, sp, a.repeat, graph=a.graph, dtype=dtype)
            ref = REFERENCE_S["sweep"][sp]
            sw[sp] = {"mean_s": round(m, 4), "std_s": round(s, 4), "reference_s_A100": ref,
                      "speedup_vs_reference": round(ref / m, 2)}
        results["sweep"] = sw
    print(json.dumps({"benchmark": "NB03 ResNet-50 train() (3 Adam steps x 120 imgs @128px)", "mode": a.mode, "graph": a.graph,
                      "devices": [str(d) for d in devs],
                      "dtype": ("fp32 (convs: split-bf16 x3 MFMA, fp32 accumulate)" if a.dtype == "fp32"
                                else "bf16 (fp32 masters)"),
                      "results": results}))


if __name__ == "__main__":
    main()
