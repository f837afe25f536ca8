"""pytorchdistributed_amd — an MI355X-native distributed-training framework.

Same capabilities and API surface as the JoeyOL/PytorchDistributed tutorial (DataParallel, DDP via
spawn / a torchrun-compatible launcher, DistributedSampler, layer-split model parallel and micro-
batched pipelines) plus overlapped gradient bucketing, FSDP full-shard and PPxDP, on PyTorch-ROCm
tensors + hand-written CDNA4 HIP kernels + RCCL over xGMI.  See SURVEY.md for the blueprint.
"""
from . import distributed  # noqa: F401
from .distributed import (  # noqa: F401
    init_process_group, destroy_process_group, get_rank, get_world_size, get_local_rank, barrier, set_device,
)
from .launch import spawn  # noqa: F401

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
