"""pytorchdistributed_amd — an MI355X-native distributed-training framework.

Same capabilities and API surface as the JoeyOL/PytorchDistributed tutorial (DataParallel, DDP via
spawn / a torchrun-compatible launcher, DistributedSampler, layer-split model parallel and micro-
batched pipelines) plus overlapped gradient bucketing, FSDP full-shard and PPxDP, on PyTorch-ROCm
tensors + hand-written CDNA4 HIP kernels + RCCL over xGMI.  See SURVEY.md for the blueprint.
"""
import os as _os


def _ensure_hw_queues():
    """Raise HIP's hardware-queue count per process to ``PDA_HW_QUEUES`` (default 8, at most 32).

    A process's HIP streams share ``GPU_MAX_HW_QUEUES`` hardware queues round-robin (HIP default 4).
    A training step here drives the compute stream, the weight-gradient side stream (ops/streams.py),
    RCCL's streams and the IPC collective stream; with 4 queues two of them land on one queue, and a
    stream-wait packet at the head of a shared queue stalls the other stream's kernels behind it.
    Measured: ResNet-50 DDP over a one-rank RCCL group 9.30k img/s at 4 queues, 9.82k at 8 (= 16;
    profiles/r2_hw_queues.jsonl).  Only effective before the process's first HIP call.

    An exported ``GPU_MAX_HW_QUEUES`` is respected unless ``PDA_HW_QUEUES`` is also set (bench.py sets
    ``PDA_HW_QUEUES=8`` by default: its one-rank RCCL group lost 5 % at 4 queues)."""
    explicit = _os.environ.get("PDA_HW_QUEUES")
    if "GPU_MAX_HW_QUEUES" in _os.environ and not explicit:
        return  # the user chose HIP's queue count: leave it (PDA_HW_QUEUES overrides it explicitly)
    want = min(int(explicit or "8"), 32)
    have = int(_os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4)
    if want > have:
        _os.environ["GPU_MAX_HW_QUEUES"] = str(want)


_ensure_hw_queues()

from . import distributed  # noqa: E402,F401
from .distributed import (  # noqa: E402,F401
    init_process_group, destroy_process_group, get_rank, get_world_size, get_local_rank, barrier, set_device,
)
from .launch import spawn  # noqa: E402,F401

__version__ = "0.1.0"


def __getattr__(name):
    # lazy submodules keep `import pytorchdistributed_amd` light for the launcher
    import importlib

    if name in {"ops", "nn", "models", "parallel", "optim", "data", "train", "utils", "bench"}:
        return importlib.import_module(f".{name}", __name__)
    if name == "DistributedDataParallel":
        from .parallel.ddp import DistributedDataParallel
        return DistributedDataParallel
    if name == "DistributedSampler":
        from .data.sampler import DistributedSampler
        return DistributedSampler
    if name == "Trainer":
        from .train import Trainer
        return Trainer
    raise AttributeError(name)
