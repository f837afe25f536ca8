"""Headline benchmark: ResNet-50 DDP images/sec on 1/2/4/8 MI355X (BASELINE.json metric / config 2).

Model: ResNet-50 v1.5 random init, bf16 parameters + fp32 masters (fused SGD, momentum 0.9, wd 5e-5);
data: synthetic ImageNet-shape batches (224x224, 1000 classes) generated on device every step;
parallelism: one process per GPU, gradients all-reduced by the bucketed DDP over RCCL, overlapped with
backward.  Weak scaling: the per-GPU batch is fixed.
"""
from __future__ import annotations

import argparse
import contextlib
import os

import torch

from ..data.device import DeviceSyntheticImages
from ..models.resnet import resnet50
from ..ops import cross_entropy
from ..optim import SGD
from ..parallel.ddp import DistributedDataParallel
from .common import comm_record, emit, group_info, setup, teardown, timed

METRIC = "images/sec (whole node) ResNet-50 DDP at 1/2/4/8 MI355X; scaling efficiency"


def build(batch: int, image: int, device, rank: int, dtype=torch.bfloat16, bucket_mb=None):
    torch.manual_seed(0)
    model = resnet50(device=device, dtype=dtype)
    model = DistributedDataParallel(model, device_ids=[device.index] if device.type == "cuda" else None,
                                    bucket_cap_mb=bucket_mb)
    opt = SGD(model.parameters(), lr=0.1, momentum=0.9, weight_decay=5e-5)
    data = DeviceSyntheticImages(batch, image, 1000, device=device, dtype=dtype, seed=1234, rank=rank)

    def step():
        x, y = data.next()
        opt.zero_grad(set_to_none=True)
        out = model(x)
        loss = cross_entropy(out, y)
        loss.backward()
        opt.step()
        return loss

    return model, opt, step


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    # per-GPU batch: 640 uses the 288 GB of an MI355X for throughput (bigger GEMM grids — the 14^2 / 7^2
    # convs' tile rounds quantise better: 640 * 196 / 256 = 490 tiles = 1.91 rounds of 256 CUs against
    # 1.53 at 512 — and less per-image launch / epilogue overhead); measured on one MI355X with the
    # current kernels (profiles/r2_resnet50_batch_sweep_v23.jsonl): 512 -> 10.94k, 576 -> 11.27k,
    # 640 -> 11.31k, 704 -> 11.07k, 768 -> 11.13k img/s (round-1 setting: --batch 256).
    ap.add_argument("--batch", type=int, default=int(os.environ.get("PDA_BENCH_BATCH", "640")),
                    help="per-GPU batch")
    ap.add_argument("--image", type=int, default=224)
    ap.add_argument("--bucket-mb", type=float, default=None)
    a = ap.parse_args(argv)
    # N=1 runs the DDP bucket all-reduces over a one-rank RCCL group (PDA_DDP_FORCE_COMM=0 turns it off)
    rank, world, local, device = setup(a.gpus, one_rank_group=True)
    if device.type == "cpu":  # plumbing-only run on a machine without a GPU
        a.batch, a.image = min(a.batch, 2), min(a.image, 64)
    # PDA_MAIN_PRIO=high: the whole step on a high-priority HIP stream (A/B knob for queue arbitration
    # against the low-priority weight-gradient side stream, ops/streams.py)
    ctx = contextlib.nullcontext()
    if device.type == "cuda" and os.environ.get("PDA_MAIN_PRIO") == "high":
        ctx = torch.cuda.stream(torch.cuda.Stream(device=device, priority=-1))
    with ctx:
        model, _, step = build(a.batch, a.image, device, rank, bucket_mb=a.bucket_mb)
        losses = []
        reset = (lambda: model.comm_stats(reset=True)) if hasattr(model, "comm_stats") else None
        secs = timed(lambda: losses.append(step()), a.steps, a.warmup, on_start=reset)
        comm = comm_record(model, a.steps)
    # (after the timed window) a benchmark that diverged would be measuring garbage
    last = float(losses[-1].item())
    if last != last or abs(last) == float("inf"):
        raise SystemExit(f"non-finite training loss {last} in the benchmark run")
    ms = secs / a.steps * 1e3
    grp = group_info(device)
    world = grp["world"]
    imgs = a.batch * world * a.steps / secs
    emit({
        "metric": METRIC, "value": round(imgs, 2), "unit": "images/sec", "n_gpus": world, "steps": a.steps,
        "warmup": a.warmup, "ms_per_step": round(ms, 3), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "rccl_world": grp["rccl_world"], "backend": grp["backend"], "dtype": "bf16" if device.type == "cuda" else "bf16-cpu-plumbing",
        "data": "synthetic (on-device Philox, ImageNet shape 224x224x3, 1000 classes), random-init weights",
        "config": {"model": "resnet50", "global_batch": a.batch * world, "per_gpu_batch": a.batch,
                   "image_size": a.image, "seq_len": None, "parallelism": f"dp{world}",
                   "optimizer": "SGD(momentum=0.9, wd=5e-5), fp32 master weights"},
        "final_loss": round(last, 4),
        "comm": comm,
        "notes": "reference publishes no number for this metric (BASELINE.json published={}); per-GPU batch "
                 f"{a.batch} (640 = throughput-optimal on 288 GB HBM by a 512-768 sweep; --batch 256 gives "
                 "the round-1 setting); NB03 parity numbers are produced by pytorchdistributed_amd.bench.nb03",
    }, rank)
    teardown()


if __name__ == "__main__":
    main()
