"""Shared benchmark plumbing: distributed setup from the torchrun / pda-run env contract and the
timed-window protocol (barrier + synchronize on both sides, MAX over ranks)."""
from __future__ import annotations

import json
import os

import torch
import torch.distributed as dist

from .. import distributed as pdist
from ..utils.timing import StepTimer


def setup(n_gpus: int):
    """Rank / world / local rank / device from the env contract; initialises the default group.

    ``PDA_DIST_BACKEND`` overrides the backend (default ``nccl`` = RCCL on a GPU, ``gloo`` on CPU).
    Rehearsal mode: with ``PDA_DIST_BACKEND=gloo`` more ranks than GPUs may share the visible GPUs
    (rank r on GPU r % count) — the whole multi-rank DDP path (hooks, buckets, collectives, timing
    protocol) runs on the native kernels of a one-GPU box; RCCL itself refuses two ranks per GPU.
    """
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if n_gpus != world and world > 1:
        raise SystemExit(f"--gpus {n_gpus} but WORLD_SIZE={world}")
    use_gpu = torch.cuda.is_available()
    backend = os.environ.get("PDA_DIST_BACKEND", "nccl" if use_gpu else "gloo")
    gpu = local
    if use_gpu:
        count = torch.cuda.device_count()
        if local >= count:
            if backend == "nccl":
                raise SystemExit(f"LOCAL_RANK {local} but only {count} GPU(s) visible (RCCL needs one GPU per "
                                 f"rank; PDA_DIST_BACKEND=gloo rehearses with shared GPUs)")
            gpu = local % count
        torch.cuda.set_device(gpu)
    # PDA_DDP_FORCE_COMM=1 at N=1: a one-rank RCCL group, so the bucket all-reduces of the multi-GPU
    # path run (and are timed) on a single GPU
    force = os.environ.get("PDA_DDP_FORCE_COMM") == "1" and use_gpu and backend == "nccl"
    if (world > 1 or force) and not dist.is_initialized():
        pdist.init_process_group(backend, rank=rank, world_size=world,
                                 device_id=gpu if use_gpu and backend == "nccl" else None)
    device = torch.device("cuda", gpu) if use_gpu else torch.device("cpu")
    return rank, world, local, device


def timed(step_fn, steps: int, warmup: int) -> float:
    """Run ``warmup`` untimed steps, then time exactly ``steps``; returns max-over-ranks seconds."""
    for _ in range(warmup):
        step_fn()
    t = StepTimer()
    t.start()
    for _ in range(steps):
        step_fn()
    secs = t.stop()
    return t.max_over_ranks(secs)


def emit(record: dict, rank: int):
    if rank == 0:
        print(json.dumps(record), flush=True)


def teardown():
    if dist.is_initialized():
        pdist.destroy_process_group()
