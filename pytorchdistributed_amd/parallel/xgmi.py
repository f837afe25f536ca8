"""One-shot all-reduce over IPC-mapped peer buffers on the xGMI mesh (SURVEY §2.2 P12, §2.6 X05,
§5.8).  Kernel + communicator: `csrc/kernels/xgmi.hip`, `csrc/bindings.cpp:XgmiComm`.

Each rank owns an uncached exchange buffer; the IPC handles are swapped through the rendezvous
store once, and every call is ``copy bucket -> own buffer; one kernel reads all peers' buffers and
writes the reduced bucket`` — all 7 links of an MI355X are read concurrently, where one RCCL ring
drives one.  Opt-in (``PDA_ALLREDUCE=ipc`` for DDP buckets up to ``PDA_IPC_CAPACITY_MB``); RCCL stays
the default transport.  Single node only (peers must be IPC-reachable GPUs).

    comm = XgmiAllReduce(capacity_mb=64)        # after init_process_group
    comm(t, average=True)                       # in place, on the current HIP stream
"""
from __future__ import annotations

import os
from typing import Optional

import torch
import torch.distributed as dist

from .. import _native

_COUNTER = [0]


class XgmiAllReduce:
    def __init__(self, capacity_mb: float = 64.0, device: Optional[torch.device] = None, timeout_s: float = 10.0,
                 store=None, rank: Optional[int] = None, world: Optional[int] = None):
        self.rank = dist.get_rank() if rank is None else rank
        self.world = dist.get_world_size() if world is None else world
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device())
        self.device = device
        self.capacity = int(capacity_mb * 2 ** 20)
        self.comm = _native.C().XgmiComm(self.rank, self.world, self.capacity, device.index, timeout_s)
        store = store if store is not None else dist.distributed_c10d._get_default_store()
        tag = f"pda_xgmi/{_COUNTER[0]}"
        _COUNTER[0] += 1
        store.set(f"{tag}/{self.rank}", self.comm.handles())
        blobs = []
        for r in range(self.world):
            v = store.get(f"{tag}/{r}")
            blobs.append(bytes(v))
        self.comm.open(blobs)

    def fits(self, t: torch.Tensor) -> bool:
        return (t.is_cuda and t.device == self.device and t.is_contiguous() and t.numel() % 8 == 0
                and t.dtype in (torch.float32, torch.bfloat16) and t.numel() * t.element_size() <= self.capacity)

    def __call__(self, t: torch.Tensor, average: bool = False) -> torch.Tensor:
        self.comm.allreduce(t, average)
        return t

    def check(self):
        """Raise if a barrier of any previous call timed out (synchronises the device)."""
        e = self.comm.error()
        if e:
            raise RuntimeError(f"xgmi all-reduce: peer barrier timed out (phase {e - 1}) on rank {self.rank}")


def ipc_requested() -> bool:
    return os.environ.get("PDA_ALLREDUCE", "auto").lower() in ("ipc", "oneshot", "xgmi")


def single_node() -> bool:
    lw = os.environ.get("LOCAL_WORLD_SIZE")
    return lw is None or int(lw) == dist.get_world_size()
