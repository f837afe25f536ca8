"""Collectives over IPC-mapped peer buffers on the xGMI mesh.
Kernels + communicator: `csrc/kernels/xgmi.hip`, `csrc/bindings.cpp:XgmiComm`.

Each rank owns an uncached exchange buffer; the IPC handles are swapped through the rendezvous
store once, and every call is ``copy input -> own buffer; one kernel over the peers' buffers``:
all 7 links of an MI355X are driven concurrently, where one RCCL ring drives one.  All-reduce
algorithms:

* ``oneshot``: every rank reads all peers' whole buffers — (N-1)·S link bytes, one barrier round;
* ``twoshot``: direct reduce-scatter (rank r reduces chunk r) + direct all-gather —
  2·(N-1)/N·S link bytes, three barrier rounds;
* ``ring``: the reference tutorial's ring (`02 DDP基本概念/02_ddp.ipynb` raw lines 33-47) executed on
  the GPUs — N-1 reduce-scatter + N-1 all-gather neighbour steps; a correctness cross-check of the
  direct algorithms and the executable form of the concept, not a fast path (one link per step);
* ``auto`` (``PDA_ALLREDUCE=ipc``): the per-node tuning table when one is present
  (``PDA_XGMI_TUNING`` or :func:`default_table_path`, written by ``tools/bench_allreduce.py
  --write-table``: per size range the fastest of RCCL / one-shot / two-shot), otherwise one-shot up
  to ``PDA_XGMI_TWOSHOT_MB`` (default 1 MB) and two-shot above.

Plus the FSDP collectives (X18): :meth:`XgmiAllReduce.all_gather_into_tensor` (every rank pulls
each peer's shard over its own link) and :meth:`XgmiAllReduce.reduce_scatter_tensor` (rank r
reduces chunk r of every peer's buffer); ``PDA_FSDP_COMM=ipc`` routes FSDP units through them.

Zero-copy (``PDA_XGMI_ZERO_COPY``, default on): a tensor that lives as long as the collectives on it —
DDP's flat gradient buffers, FSDP's shards and unit gradient buffers — is *registered* once per layout
(:meth:`XgmiAllReduce.register`: the IPC handle of its allocation plus its offset, swapped through the
store), and the kernels then read the peers' tensors in place: no copy into the exchange buffer, no
capacity limit.  In-place all-reduce runs two-shot or ring (one-shot would overwrite its input while peers
still read it).

Opt-in for DDP buckets (``PDA_ALLREDUCE=ipc|oneshot|twoshot|ring``); RCCL stays the default transport.
Single node only (peers must be IPC-reachable GPUs).

    comm = XgmiAllReduce(capacity_mb=64)        # after init_process_group
    comm(t, average=True, algo="auto")          # in place, on the current HIP stream
"""
from __future__ import annotations

import json
import os
import socket
from typing import List, Optional

import torch
import torch.distributed as dist

from .. import _native

_COUNTER = [0]
_ALGOS = {"oneshot": 0, "twoshot": 1, "ring": 2}
RCCL = -1  # pick(): "use RCCL for this size" (tuning table entry)


def default_table_path(world: int) -> str:
    """Per-node tuning table location: ``~/.cache/pytorchdistributed_amd/xgmi_<host>_w<world>.json``."""
    return os.path.join(os.path.expanduser("~"), ".cache", "pytorchdistributed_amd",
                        f"xgmi_{socket.gethostname()}_w{world}.json")


def load_table(world: int, path: Optional[str] = None) -> Optional[List[dict]]:
    """The crossover table ``[{"max_bytes": int, "algo": "rccl"|"oneshot"|"twoshot"}, ...]`` (ascending
    ``max_bytes``; the last entry covers everything larger) for ``world`` ranks, or None."""
    path = path or os.environ.get("PDA_XGMI_TUNING") or default_table_path(world)
    if not os.path.exists(path):
        return None
    with open(path) as f:
        doc = json.load(f)
    if int(doc.get("world", -1)) != world:
        return None
    entries = sorted(doc["entries"], key=lambda e: e["max_bytes"])
    for e in entries:
        if e["algo"] not in ("rccl", "oneshot", "twoshot"):
            raise ValueError(f"xgmi tuning table {path}: bad algo {e['algo']!r}")
    return entries


def table_from_sweep(records: List[dict], world: int) -> dict:
    """Build the tuning table from ``tools/bench_allreduce.py`` records (one per size: ``size_mb`` and
    ``ms`` per transport): per size the fastest transport, adjacent sizes with the same winner merged,
    each range reaching up to the measured size (the last one open-ended)."""
    entries = []
    for rec in sorted(records, key=lambda r: r["size_mb"]):
        cands = {"rccl": rec["rccl"]["ms"], "oneshot": rec["xgmi_oneshot"]["ms"], "twoshot": rec["xgmi_twoshot"]["ms"]}
        best = min(cands, key=cands.get)
        nbytes = int(rec["size_mb"] * 2 ** 20)
        if entries and entries[-1]["algo"] == best:
            entries[-1]["max_bytes"] = nbytes
        else:
            entries.append({"max_bytes": nbytes, "algo": best})
    if entries:
        entries[-1]["max_bytes"] = 1 << 62
    return {"world": world, "entries": entries}


class XgmiAllReduce:
    def __init__(self, capacity_mb: float = 64.0, device: Optional[torch.device] = None, timeout_s: Optional[float] = None,
                 store=None, rank: Optional[int] = None, world: Optional[int] = None):
        # peer-barrier deadline inside the kernels (PDA_XGMI_TIMEOUT_S, default 60 s): long enough that a
        # peer whose first launch waits on a cold code-object load is not taken for a dead one (the
        # collective watchdog, PDA_COLLECTIVE_TIMEOUT_S, is what ends real hangs)
        if timeout_s is None:
            timeout_s = float(os.environ.get("PDA_XGMI_TIMEOUT_S", "60"))
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
        self._store, self._tag, self._nreg = store, tag, 0
        # rank 0's tuning table is THE table: every rank must pick the same algorithm per size
        if self.rank == 0:
            table = load_table(self.world)
            store.set(f"{tag}/table", json.dumps(table))
        self.table = json.loads(bytes(store.get(f"{tag}/table")).decode())
        store.set(f"{tag}/{self.rank}", self.comm.handles())
        blobs = []
        for r in range(self.world):
            v = store.get(f"{tag}/{r}")
            blobs.append(bytes(v))
        self.comm.open(blobs)

    def fits(self, t: torch.Tensor, algo: str = "auto") -> bool:
        """True if ``t`` can (and, per the tuning table, should) go through the IPC kernels."""
        if algo in ("auto", "ipc", "xgmi") and self.table is not None and \
                self.pick(t.numel() * t.element_size(), algo) == RCCL:
            return False
        return (t.is_cuda and t.device == self.device and t.is_contiguous() and t.numel() % 8 == 0
                and t.dtype in (torch.float32, torch.bfloat16) and t.numel() * t.element_size() <= self.capacity)

    def pick(self, nbytes: int, algo: str = "auto") -> int:
        """0 = one-shot, 1 = two-shot, 2 = ring, or :data:`RCCL` (tuning table says RCCL wins) for a
        message of ``nbytes`` (same answer on every rank: the table is per node)."""
        algo = algo.lower()
        if algo in ("auto", "ipc", "xgmi"):
            if self.table is not None:
                for e in self.table:
                    if nbytes <= e["max_bytes"]:
                        return RCCL if e["algo"] == "rccl" else _ALGOS[e["algo"]]
                return RCCL if self.table[-1]["algo"] == "rccl" else _ALGOS[self.table[-1]["algo"]]
            return 1 if self.world > 2 and nbytes > self.twoshot_bytes else 0
        if algo not in _ALGOS:
            raise ValueError(f"xgmi algo must be one of auto/oneshot/twoshot/ring, got {algo!r}")
        return _ALGOS[algo]

    def __call__(self, t: torch.Tensor, average: bool = False, algo: str = "auto") -> torch.Tensor:
        a = self.pick(t.numel() * t.element_size(), algo)
        if a == RCCL:  # only reachable through a tuning table; callers that route by size check first
            a = 1 if self.world > 2 else 0
        self.comm.allreduce(t, average, a)
        return t

    def all_gather_into_tensor(self, out: torch.Tensor, inp: torch.Tensor) -> torch.Tensor:
        """``out`` (world x shard, contiguous) = every rank's ``inp`` (shard) in rank order."""
        self.comm.allgather(inp, out)
        return out

    def reduce_scatter_tensor(self, out: torch.Tensor, inp: torch.Tensor, average: bool = False) -> torch.Tensor:
        """``out`` (shard) = sum (mean) over ranks of chunk ``rank`` of ``inp`` (world x shard)."""
        self.comm.reduce_scatter(inp, out, average)
        return out

    # ------------------------------------------------------------ zero-copy registrations
    def register(self, t: torch.Tensor) -> int:
        """Collective (every rank, same order, same size): register ``t`` for zero-copy collectives and
        return the registration id.  ``t`` must stay allocated and unmoved while collectives use it."""
        key = f"{self._tag}/reg{self._nreg}"
        self._nreg += 1
        self._store.set(f"{key}/{self.rank}", self.comm.reg_handle(t))
        blobs = [bytes(self._store.get(f"{key}/{r}")) for r in range(self.world)]
        return self.comm.reg_open(t, blobs)

    def all_reduce_registered(self, reg: int, t: torch.Tensor, elem_offset: int, average: bool = False,
                              algo: str = "auto") -> torch.Tensor:
        """In-place all-reduce of ``t`` = elements ``[elem_offset, elem_offset + numel)`` of registration
        ``reg``, reading every peer's slice in place (no copy-in).  ``ring`` runs the ring; everything
        else two-shot."""
        self.comm.allreduce_reg(reg, t, elem_offset, average, 2 if algo == "ring" else 1)
        return t

    def all_gather_registered(self, reg: int, out: torch.Tensor, inp: torch.Tensor) -> torch.Tensor:
        """``out`` (world x shard) = every rank's registered ``inp`` (shard), pulled in place."""
        self.comm.allgather_reg(reg, inp, out)
        return out

    def reduce_scatter_registered(self, reg: int, out: torch.Tensor, inp: torch.Tensor,
                                  average: bool = False) -> torch.Tensor:
        """``out`` (shard) = sum (mean) over ranks of chunk ``rank`` of every rank's registered ``inp``."""
        self.comm.reduce_scatter_reg(reg, inp, out, average)
        return out

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
    return v if v in _ALGOS else None  # oneshot / twoshot / ring


def zero_copy() -> bool:
    """``PDA_XGMI_ZERO_COPY`` (default on): registered tensors, no copy into the exchange buffer."""
    return os.environ.get("PDA_XGMI_ZERO_COPY", "1") != "0"


def single_node() -> bool:
    lw = os.environ.get("LOCAL_WORLD_SIZE")
    return lw is None or int(lw) == dist.get_world_size()
