"""Benchmark timing.

The reference times with ``timeit`` and no device synchronisation (`03_model_parallel.ipynb` raw
lines 401-420), so queued kernels of the last step can fall outside the measurement.  Here a timed
window is bracketed by a barrier + ``torch.cuda.synchronize()`` on both sides, measured with host
wall clock and HIP events, and reduced with MAX over ranks.
"""
from __future__ import annotations

import time
from contextlib import contextmanager

import torch
import torch.distributed as dist


def sync(device=None):
    if torch.cuda.is_available():
        torch.cuda.synchronize(device)


def barrier():
    if dist.is_initialized():
        if dist.get_backend() == "nccl":
            dist.barrier(device_ids=[torch.cuda.current_device()])
        else:
            dist.barrier()


class StepTimer:
    """Wall-clock window measured between two barrier+synchronize points."""

    def __init__(self):
        self.t0 = self.t1 = None

    def start(self):
        barrier()
        sync()
        self.t0 = time.perf_counter()

    def stop(self) -> float:
        sync()
        barrier()
        self.t1 = time.perf_counter()
        return self.t1 - self.t0

    def max_over_ranks(self, seconds: float) -> float:
        if not dist.is_initialized():
            return seconds
        dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else "cpu"
        t = torch.tensor([seconds], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())


@contextmanager
def range(name: str):
    """roctx range (visible in rocprofv3 --marker-trace); no-op without a GPU."""
    if torch.cuda.is_available():
        torch.cuda.nvtx.range_push(name)
        try:
            yield
        finally:
            torch.cuda.nvtx.range_pop()
    else:
        yield
