"""Process-group layer (reference `ddp_setup` in `02 DDP基本概念/ddp_gpus.py:11-23` and
`ddp_gpus_torchrun.py:11-19`).

One process per GPU.  The device collectives are RCCL (``backend="nccl"`` IS RCCL on ROCm) driven through
``torch.distributed``; the rendezvous key-value store is the framework's own C++ TCP store
(``csrc/runtime/store.cpp``) whenever the framework owns the launch (:mod:`.launch` ``spawn`` /
``pda-run``), exposed to c10d as a :class:`torch.distributed.Store` subclass.  Under ``torchrun`` the
agent already hosts a store on ``MASTER_PORT``, so the workers join it through ``env://``.

Extra transport: :func:`host_ring` returns the C++ ring communicator (the reference's ring
all-reduce, `02_ddp.ipynb` raw lines 33-47) for CPU tensors.
"""
from __future__ import annotations

import datetime
import os
import socket
from typing import Optional

import torch
import torch.distributed as dist

from . import _native

# re-exported collective API (the reference uses these names through torch.distributed)
ReduceOp = dist.ReduceOp
all_reduce = dist.all_reduce
all_gather = dist.all_gather
all_gather_into_tensor = dist.all_gather_into_tensor
reduce_scatter_tensor = dist.reduce_scatter_tensor
broadcast = dist.broadcast
send = dist.send
recv = dist.recv
isend = dist.isend
irecv = dist.irecv
batch_isend_irecv = dist.batch_isend_irecv
P2POp = dist.P2POp
all_to_all_single = dist.all_to_all_single
new_group = dist.new_group
is_initialized = dist.is_initialized

_STATE = {"server": None, "store": None, "ring": None, "backend": None}

DEFAULT_TIMEOUT = datetime.timedelta(minutes=float(os.environ.get("PDA_TIMEOUT_MIN", "30")))


class NativeStore(dist.Store):
    """c10d Store backed by the framework's C++ TCP store client."""

    def __init__(self, host: str, port: int, timeout: float = 300.0, prefix: str = ""):
        super().__init__()
        self._host, self._port, self._p = host, port, prefix
        self._c = _native.C().StoreClient(host, int(port), float(timeout))

    def _k(self, key: str) -> str:
        return self._p + key

    @staticmethod
    def _b(v) -> bytes:
        if isinstance(v, str):
            return v.encode()
        if isinstance(v, (bytes, bytearray)):
            return bytes(v)
        return bytes(v)

    def set(self, key, value):
        self._c.set(self._k(key), self._b(value))

    def get(self, key):
        return self._c.get(self._k(key))

    def add(self, key, value):
        return self._c.add(self._k(key), int(value))

    def compare_set(self, key, expected_value, desired_value):
        return self._c.compare_set(self._k(key), self._b(expected_value), self._b(desired_value))

    def delete_key(self, key):
        return self._c.delete_key(self._k(key))

    def num_keys(self):
        return self._c.num_keys()

    def check(self, keys):
        return self._c.check([self._k(k) for k in keys])

    def wait(self, keys, timeout=None):
        t = timeout.total_seconds() if isinstance(timeout, datetime.timedelta) else (timeout or 0.0)
        self._c.wait([self._k(k) for k in keys], float(t))

    def set_timeout(self, timeout):
        t = timeout.total_seconds() if isinstance(timeout, datetime.timedelta) else float(timeout)
        self._c.set_timeout(t)

    @property
    def timeout(self):
        return datetime.timedelta(seconds=self._c.timeout)


def start_store_server(host: str = "0.0.0.0", port: int = 0):
    """Host the native store in this process (used by the launcher / rank 0). Returns the server."""
    return _native.C().StoreServer(host, int(port))


def free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _env_int(name: str, default: Optional[int] = None) -> Optional[int]:
    v = os.environ.get(name)
    return int(v) if v not in (None, "") else default


def comm_high_priority() -> bool:
    """``PDA_COMM_PRIORITY``: ``high`` (or 1 / true) puts every communication stream of this process —
    the native RCCL communicators' (comm.py) and torch's process group's — at high priority; ``normal``
    (default, or 0 / false) leaves them at the default priority, which measured 0.6 % faster on the
    one-rank headline step (profiles/r3_comm_priority_ab.jsonl)."""
    v = os.environ.get("PDA_COMM_PRIORITY", "normal").strip().lower()
    if v in ("high", "1", "true", "yes", "on"):
        return True
    if v in ("normal", "0", "false", "no", "off", "low", ""):
        return False
    raise ValueError(f"PDA_COMM_PRIORITY={v!r}: expected high | normal")


def init_process_group(
    backend: str = "nccl",
    init_method: Optional[str] = None,
    rank: Optional[int] = None,
    world_size: Optional[int] = None,
    timeout: datetime.timedelta = DEFAULT_TIMEOUT,
    store: Optional[dist.Store] = None,
    device_id: Optional[int] = None,
):
    """Initialise the default process group.

    ``backend``: ``"nccl"``/``"rccl"`` (RCCL over xGMI), ``"gloo"`` (CPU), or ``"ring"`` (gloo for
    control plus the native host ring transport for CPU all-reduce).
    Rank / world size default to ``RANK`` / ``WORLD_SIZE`` (torchrun / pda-run env contract).
    """
    if backend == "rccl":
        backend = "nccl"
    want_ring = backend == "ring"
    if want_ring:
        backend = "gloo"
    rank = rank if rank is not None else _env_int("RANK", 0)
    world_size = world_size if world_size is not None else _env_int("WORLD_SIZE", 1)
    os.environ.setdefault("RANK", str(rank))
    os.environ.setdefault("WORLD_SIZE", str(world_size))
    under_torchrun = os.environ.get("TORCHELASTIC_USE_AGENT_STORE") == "True"

    if store is None and init_method is None and not under_torchrun:
        host = os.environ.get("MASTER_ADDR", "127.0.0.1")
        port = _env_int("MASTER_PORT", 29500)
        if rank == 0 and os.environ.get("PDA_STORE_HOSTED") != "1":
            _STATE["server"] = start_store_server("0.0.0.0", port)
        # a relaunched worker group (pda-run --max-restarts) must not read the previous attempt's keys
        store = NativeStore(host, port, timeout.total_seconds(),
                            prefix=f"pda/attempt{os.environ.get('PDA_RESTART_COUNT', '0')}/")
    _STATE["store"] = store
    kwargs = dict(backend=backend, timeout=timeout, rank=rank, world_size=world_size)
    if store is not None:
        kwargs["store"] = store
    elif init_method is not None:
        kwargs["init_method"] = init_method
    if device_id is not None and backend == "nccl":
        kwargs["device_id"] = torch.device("cuda", device_id)
    if backend == "nccl" and comm_high_priority():
        # PDA_COMM_PRIORITY=high: RCCL's internal streams at high priority as well,
        # the same switch as the native communicators' (comm.py)
        opts = dist.ProcessGroupNCCL.Options()
        opts.is_high_priority_stream = True
        kwargs["pg_options"] = opts
    dist.init_process_group(**kwargs)
    _STATE["backend"] = "ring" if want_ring else backend
    if want_ring:
        host_ring()
    from .parallel import debug as _debug

    _debug.maybe_enable()  # PDA_DEBUG=collectives: cross-rank fingerprint check before every collective
    return dist.group.WORLD


def host_ring():
    """Lazily build the native ring over the default group's store (CPU tensors)."""
    if _STATE["ring"] is not None:
        return _STATE["ring"]
    store = _STATE["store"]
    if store is None:
        raise RuntimeError("host ring needs the framework-owned store (launch with spawn / pda-run)")
    r, w = get_rank(), get_world_size()
    ring = _native.C().HostRing(r, w)
    host = os.environ.get("PDA_RING_HOST", "127.0.0.1")
    addr = ring.listen(host)
    store.set(f"pda/ring/{r}", addr)
    right = (r + 1) % w
    rhost, rport = store.get(f"pda/ring/{right}").decode().rsplit(":", 1)
    ring.connect(rhost, int(rport), 60.0)
    _STATE["ring"] = ring
    return ring


def ring_all_reduce(t: torch.Tensor, average: bool = False) -> torch.Tensor:
    """In-place sum (or mean) of a contiguous CPU fp32/fp64 tensor over the native ring."""
    assert t.device.type == "cpu" and t.is_contiguous()
    ring = host_ring()
    if t.dtype == torch.float32:
        ring.allreduce_f32(t.data_ptr(), t.numel())
    elif t.dtype == torch.float64:
        ring.allreduce_f64(t.data_ptr(), t.numel())
    else:
        raise TypeError("ring all-reduce supports float32/float64")
    if average:
        t.div_(ring.world)
    return t


def backend() -> Optional[str]:
    return _STATE["backend"]


def get_rank(group=None) -> int:
    return dist.get_rank(group) if dist.is_initialized() else 0


def get_world_size(group=None) -> int:
    return dist.get_world_size(group) if dist.is_initialized() else 1


def get_local_rank() -> int:
    return _env_int("LOCAL_RANK", 0)


def get_local_world_size() -> int:
    return _env_int("LOCAL_WORLD_SIZE", 1)


def barrier(group=None):
    if not dist.is_initialized():
        return
    if _STATE["backend"] == "nccl" and torch.cuda.is_available():
        dist.barrier(group=group, device_ids=[torch.cuda.current_device()])
    else:
        dist.barrier(group=group)


def set_device(local_rank: int):
    """`torch.cuda.set_device` equivalent (reference `PY1:23`, `PY2:19`)."""
    if torch.cuda.is_available():
        torch.cuda.set_device(local_rank)


def destroy_process_group():
    from . import comm as _comm

    _comm.reset()  # native RCCL communicators first (ncclCommDestroy), then c10d's
    if dist.is_initialized():
        dist.destroy_process_group()
    _STATE["ring"] = None
    _STATE["store"] = None
    srv = _STATE.pop("server", None)
    _STATE["server"] = None
    if srv is not None:
        srv.stop()
    _STATE["backend"] = None
