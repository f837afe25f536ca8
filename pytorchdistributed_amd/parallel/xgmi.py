"""All-reduce over IPC-mapped peer buffers on the xGMI mesh.
Kernels + communicator: `csrc/kernels/xgmi.hip`, `csrc/bindings.cpp:XgmiComm`.

Each rank owns an uncached exchange buffer; the IPC handles are swapped through the rendezvous
store once, and every call is ``copy bucket -> own buffer; one kernel over the peers' buffers``:
all 7 links of an MI355X are driven concurrently, where one RCCL ring drives one.  Two algorithms:

* ``oneshot``: every rank reads all peers' whole buffers — (N-1)·S link bytes, one barrier round;
* ``twoshot``: direct reduce-scatter (rank r reduces chunk r) + direct all-gather —
  2·(N-1)/N·S link bytes, three barrier rounds;
* ``auto`` (``PDA_ALLREDUCE=ipc``): one-shot up to ``PDA_XGMI_TWOSHOT_MB`` (default 1 MB; the
  crossover is measured by ``tools/bench_allreduce.py``), two-shot above.

Opt-in for DDP buckets (``PDA_ALLREDUCE=ipc|oneshot|twoshot``); RCCL stays the default transport.
Single node only (peers must be IPC-reachable GPUs).

    comm = XgmiAllReduce(capacity_mb=64)        # after init_process_group
    comm(t, average=True, algo="auto")          # in place, on the current HIP stream
"""
from __future__ import annotations

import os
from typing import Optional

import torch
import torch.distributed as dist

from .. import _native

_COUNTER = [0]
_ALGOS = {"oneshot": 0, "twoshot": 1}


class XgmiAllReduce:
    def __init__(self, capacity_mb: float = 64.0, device: Optional[torch.device] = None, timeout_s: float = 10.0,
                 store=None, rank: Optional[int] = None, world: Optional[int] = None):
        self.rank = dist.get_rank() if rank is None else rank
        self.world = dist.get_world_size() if world is None else world
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device())
        self.device = device
        self.capacity = int(capacity_mb * 2 ** 20)
        self.twoshot_bytes = int(float(os.environ.get("PDA_XGMI_TWOSHOT_MB", "1")) * 2 ** 20)
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

    def pick(self, nbytes: int, algo: str = "auto") -> int:
        """0 = one-shot, 1 = two-shot for a message of ``nbytes`` (same answer on every rank)."""
        algo = algo.lower()
        if algo in ("auto", "ipc", "xgmi"):
            return 1 if self.world > 2 and nbytes > self.twoshot_bytes else 0
        if algo not in _ALGOS:
            raise ValueError(f"xgmi algo must be one of auto/oneshot/twoshot, got {algo!r}")
        return _ALGOS[algo]

    def __call__(self, t: torch.Tensor, average: bool = False, algo: str = "auto") -> torch.Tensor:
        self.comm.allreduce(t, average, self.pick(t.numel() * t.element_size(), algo))
        return t

    def poll(self) -> int:
        """Non-blocking: 0, or 1 + the phase of a peer barrier that timed out in a call that already
        ran.  The kernels write the error word into pinned host memory, so no device sync is needed;
        calls still in flight are covered by a later poll."""
        return self.comm.error()

    def check(self, sync: bool = True):
        """Raise if a peer barrier of any previous call timed out.  ``sync=True`` first waits for the
        device so every issued call is covered; ``sync=False`` is the cheap per-step poll.  The error is
        reset once reported; the communicator is poisoned after a timeout (peer epochs no longer line
        up), so callers should fail the step rather than retry."""
        if sync:
            torch.cuda.synchronize(self.device)
        e = self.comm.error()
        if e:
            self.comm.reset_error()
            raise RuntimeError(f"xgmi all-reduce: peer barrier timed out (phase {e - 1}) on rank {self.rank}; "
                               f"results of that call are invalid")


def ipc_requested() -> bool:
    return requested_algo() is not None


def requested_algo():
    """The IPC algorithm named by ``PDA_ALLREDUCE`` (``auto`` for ipc/xgmi), or None for RCCL."""
    v = os.environ.get("PDA_ALLREDUCE", "rccl").lower()
    if v in ("ipc", "xgmi"):
        return "auto"
    return v if v in _ALGOS else None


def single_node() -> bool:
    lw = os.environ.get("LOCAL_WORLD_SIZE")
    return lw is None or int(lw) == dist.get_world_size()
