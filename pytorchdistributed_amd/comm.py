"""Native RCCL communicator (reference `init_process_group(backend="nccl")` at
`02 DDP基本概念/ddp_gpus.py:20-22`, which torch serves with ProcessGroupNCCL).

:class:`Communicator` owns an ``ncclComm_t`` over a process group and a HIP stream of its own
(`csrc/comm/communicator.cpp`; default priority, ``PDA_COMM_PRIORITY=high`` for a high-priority
one).  A collective is enqueued on that stream after an event-wait on the streams that produce its
input and returns a :class:`Work`: ``wait()`` orders the current
stream after the collective without blocking the host, ``is_completed()`` polls.  The bootstrap is
the framework's own: group rank 0 calls ``ncclGetUniqueId`` and publishes the id in the rendezvous
store (the native C++ store when the framework launched the job, the launcher's otherwise), every
rank reads it and joins with ``ncclCommInitRank``.  Every communicator is registered with the native
collective watchdog's abort hook: a collective that outlives its deadline is ``ncclCommAbort``-ed.

torch.distributed (c10d) remains the control plane — rendezvous, barriers, object collectives; the
gradient / parameter traffic of DDP, FSDP and the pipeline's DP group runs here (``PDA_COMM=c10d``
switches it back to ProcessGroupNCCL).
"""
from __future__ import annotations

import os
from typing import Dict, Iterable, List, Optional, Tuple

import torch
import torch.distributed as dist

from . import _native

_DTYPE = {torch.float32: 0, torch.bfloat16: 1, torch.float16: 2, torch.float64: 3, torch.int64: 4, torch.int32: 5,
          torch.uint8: 6, torch.int8: 7}
_OPS = {"sum": 0, "avg": 1, "max": 2, "min": 3, "prod": 4}
_created: Dict[Tuple[int, ...], int] = {}
_cache: Dict[Tuple[Tuple[int, ...], int], "Communicator"] = {}
# last enqueued native operation per device: (communicator, Work) — the cross-communicator order rule
_LAST: Dict[int, tuple] = {}
_ORDER_STATS = {"order_waits": 0}


def ordered() -> bool:
    """One global order for every native communicator of a process (``PDA_COMM_ORDER``, default on).

    Each communicator owns a stream, so a rank driving two of them — PP x DP: the pipeline's P2P group
    and the stage's DP all-reduce group — could otherwise run their RCCL kernels in either order on the
    GPU.  With the rule on, an operation on communicator B is stream-ordered after the last operation
    enqueued on any other communicator A of the same device, so each rank executes its collectives in
    exactly its host enqueue order.  Ranks sharing a communicator enqueue identical sequences on it
    (same schedule), and the DP groups only join ranks of the same pipeline stage, so no two ranks can
    wait on each other's communicators in opposite orders."""
    return os.environ.get("PDA_COMM_ORDER", "1") != "0"


def enabled() -> bool:
    """Gradient collectives on the native communicator (default) or on c10d (``PDA_COMM=c10d``)."""
    return os.environ.get("PDA_COMM", "native") == "native"


def _store():
    from . import distributed as pdist

    st = pdist._STATE.get("store")
    if st is None:
        st = dist.distributed_c10d._get_default_store()
    return st


_UID_FAILED = b"pda-rccl-unique-id-failed"


class Work:
    """Completion handle of one enqueued collective; keeps its tensors alive until completion."""

    def __init__(self, w, keep: tuple = ()):
        self._w = w
        self._keep = keep

    def wait(self, stream: Optional[torch.cuda.Stream] = None):
        s = stream if stream is not None else torch.cuda.current_stream()
        self._w.wait(s.cuda_stream)
        return True

    def is_completed(self) -> bool:
        done = self._w.is_completed()
        if done:
            self._keep = ()
        return done

    def synchronize(self):
        self._w.synchronize()
        self._keep = ()

    @property
    def event(self) -> int:
        """Raw handle of the completion event (watchdog tickets retire on it)."""
        return self._w.event


class Communicator:
    """RCCL communicator over ``group`` (default: the world) on this rank's GPU."""

    def __init__(self, group=None, device: Optional[torch.device] = None, high_priority: Optional[bool] = None):
        if not dist.is_initialized():
            raise RuntimeError("Communicator needs an initialised default process group (rendezvous / store)")
        self.group = group
        self.ranks: List[int] = (dist.get_process_group_ranks(group) if group is not None
                                 else list(range(dist.get_world_size())))
        self.rank = dist.get_rank(group)
        self.size = len(self.ranks)
        self.device = device if device is not None else torch.device("cuda", torch.cuda.current_device())
        if high_priority is None:
            # one switch for every comm stream of the process (distributed.comm_high_priority)
            from .distributed import comm_high_priority

            high_priority = comm_high_priority()
        key_ranks = tuple(self.ranks)
        seq = _created.get(key_ranks, 0)
        _created[key_ranks] = seq + 1
        key = f"pda/rccl/{'-'.join(map(str, key_ranks))}/{seq}"
        store = _store()
        C = _native.C()
        if self.rank == 0:
            try:
                uid = C.rccl_unique_id()
            except Exception:
                # publish the failure, so the other ranks raise (and try_for_group falls back on
                # every rank) instead of waiting in store.get until the store times out
                store.set(key, _UID_FAILED)
                raise
            store.set(key, uid)
        else:
            uid = store.get(key)
            if bytes(uid) == _UID_FAILED:
                raise RuntimeError("rank 0 of the group could not create the RCCL unique id")
        from .utils import watchdog as _watchdog

        # ncclCommInitRank blocks (GIL released) until every rank joined: a peer that never does turns
        # into a watchdog report + abort with stacks, not a silent hang
        with _watchdog.watch(f"rccl communicator init ranks={list(key_ranks)} seq={seq}"):
            self._c = C.RcclComm(bytes(uid), self.size, self.rank, self.device.index, high_priority)
        self.stream = torch.cuda.ExternalStream(self._c.stream, device=self.device)

    # ---------------------------------------------------------------- ordering
    def _after(self, streams: Optional[Iterable[torch.cuda.Stream]]):
        for s in (streams if streams is not None else [torch.cuda.current_stream(self.device)]):
            self._c.wait_stream(s.cuda_stream)
        if ordered():
            last = _LAST.get(self.device.index)
            if last is not None and last[0] is not self and not last[0].closed and not last[1].is_completed():
                self._c.wait_event(last[1].event)
                _ORDER_STATS["order_waits"] += 1

    def _done(self, work: "Work") -> "Work":
        _LAST[self.device.index] = (self, work)
        return work

    @property
    def closed(self) -> bool:
        return self._c.closed

    def close(self):
        """ncclCommDestroy now (after draining the comm stream); later operations raise."""
        self._c.close()

    def _check(self, name: str, *ts, **kw):
        """``PDA_DEBUG=collectives``: the cross-rank fingerprint check (parallel/debug.py) covers the
        native collectives too (op, dtype, shape, reduce op / root)."""
        from .parallel import debug as _debug

        if _debug._CHECKER is not None:
            _debug._CHECKER.check("rccl." + name, ts, dict(kw, group=self.group))

    def _hold(self, *ts: torch.Tensor):
        for t in ts:
            t.record_stream(self.stream)  # the caching allocator must not recycle it under the collective

    # ---------------------------------------------------------------- collectives
    def all_reduce(self, t: torch.Tensor, op: str = "sum", streams=None) -> Work:
        """In place; ``op`` in sum / avg / max / min / prod.  ``streams``: producers of ``t`` (default:
        the current stream)."""
        assert t.is_contiguous() and t.device == self.device
        self._check("all_reduce", t, op=op)
        self._after(streams)
        self._hold(t)
        return self._done(Work(self._c.all_reduce(t.data_ptr(), t.data_ptr(), t.numel(), _DTYPE[t.dtype], _OPS[op]),
                               (t,)))

    def reduce_scatter(self, out: torch.Tensor, inp: torch.Tensor, op: str = "sum", streams=None) -> Work:
        """``out`` = op over ranks of this rank's ``out.numel()`` chunk of ``inp``."""
        assert inp.numel() == out.numel() * self.size and inp.dtype == out.dtype
        assert inp.is_contiguous() and out.is_contiguous()
        self._check("reduce_scatter", out, inp, op=op)
        self._after(streams)
        self._hold(out, inp)
        return self._done(Work(self._c.reduce_scatter(inp.data_ptr(), out.data_ptr(), out.numel(), _DTYPE[out.dtype],
                                                      _OPS[op]), (out, inp)))

    def all_gather(self, out: torch.Tensor, inp: torch.Tensor, streams=None) -> Work:
        """``out`` = concatenation over ranks of ``inp``."""
        assert out.numel() == inp.numel() * self.size and inp.dtype == out.dtype
        assert inp.is_contiguous() and out.is_contiguous()
        self._check("all_gather", out, inp)
        self._after(streams)
        self._hold(out, inp)
        return self._done(Work(self._c.all_gather(inp.data_ptr(), out.data_ptr(), inp.numel(), _DTYPE[inp.dtype]),
                               (out, inp)))

    def reduce(self, t: torch.Tensor, root: int = 0, op: str = "sum", streams=None) -> Work:
        """In place: group rank ``root``'s ``t`` becomes op over ranks (the others' ``t`` is unchanged)."""
        assert t.is_contiguous() and t.device == self.device
        self._check("reduce", t, op=op, dst=root)
        self._after(streams)
        self._hold(t)
        return self._done(Work(self._c.reduce(t.data_ptr(), t.data_ptr(), t.numel(), _DTYPE[t.dtype], _OPS[op], root),
                               (t,)))

    @property
    def cu_budget(self) -> int:
        """CUs the comm stream may dispatch to (``PDA_COMM_CUS``; 0 = unmasked)."""
        return self._c.cu_budget

    def broadcast(self, t: torch.Tensor, root: int = 0, streams=None) -> Work:
        """In place from group rank ``root``."""
        assert t.is_contiguous()
        self._check("broadcast", t, src=root)
        self._after(streams)
        self._hold(t)
        return self._done(Work(self._c.broadcast(t.data_ptr(), t.data_ptr(), t.numel(), _DTYPE[t.dtype], root), (t,)))

    def send_recv(self, sends: List[Tuple[torch.Tensor, int]], recvs: List[Tuple[torch.Tensor, int]],
                  streams=None) -> Work:
        """One fused group of point-to-point transfers (group ranks as peers)."""
        self._after(streams)
        self._c.group_start()
        try:
            for t, peer in sends:
                assert t.is_contiguous()
                self._hold(t)
                self._c.send(t.data_ptr(), t.numel(), _DTYPE[t.dtype], peer)
            for t, peer in recvs:
                assert t.is_contiguous()
                self._hold(t)
                self._c.recv(t.data_ptr(), t.numel(), _DTYPE[t.dtype], peer)
        finally:
            w = self._c.group_end()
        return self._done(Work(w, tuple(t for t, _ in sends) + tuple(t for t, _ in recvs)))

    # ---------------------------------------------------------------- failure handling
    def abort(self):
        self._c.abort()

    @property
    def aborted(self) -> bool:
        return self._c.aborted

    def async_error(self) -> str:
        return self._c.async_error()


def for_group(group=None, device: Optional[torch.device] = None) -> Communicator:
    """The process's communicator for ``group`` on ``device`` (created once; all ranks of the group
    must ask for it in the same order, like any collective)."""
    ranks = tuple(dist.get_process_group_ranks(group)) if group is not None else tuple(range(dist.get_world_size()))
    dev = device if device is not None else torch.device("cuda", torch.cuda.current_device())
    key = (ranks, dev.index)
    c = _cache.get(key)
    if c is None or c.aborted or c.closed:
        c = _cache[key] = Communicator(group, dev)
    return c


def try_for_group(group=None, device: Optional[torch.device] = None) -> Optional[Communicator]:
    """:func:`for_group`, or None on every rank when it failed on any rank (the ranks agree through one
    c10d all-reduce of a success flag, so no rank drives the native path while another uses c10d)."""
    import warnings

    comm, err = None, None
    try:
        comm = for_group(group, device)
    except Exception as e:  # noqa: BLE001 - reported below, the caller falls back to c10d
        err = e
    dev = device if device is not None else torch.device("cuda", torch.cuda.current_device())
    ok = torch.tensor([0 if err is None else 1], dtype=torch.int32, device=dev)
    dist.all_reduce(ok, group=group)
    if int(ok.item()) == 0:
        return comm
    warnings.warn(f"native RCCL communicator unavailable ({err or 'failed on another rank'}); "
                  "gradient collectives fall back to torch.distributed")
    return None


def reset():
    """Close and drop every cached communicator (destroy_process_group): ncclCommDestroy
    runs here, explicitly, while c10d's process group and the store still exist — not whenever the
    DDP / FSDP objects holding a communicator happen to be garbage-collected."""
    for c in list(_cache.values()):
        try:
            if not c.aborted:
                c.close()
        except Exception as e:  # noqa: BLE001 - teardown must reach c10d's destroy
            import warnings

            warnings.warn(f"closing a native RCCL communicator failed: {e}")
    _cache.clear()
    _LAST.clear()


def order_stats() -> dict:
    return dict(_ORDER_STATS)
