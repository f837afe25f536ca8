"""Synchronous parameter-server training (the PS-worker concept of
`/root/reference/02 DDP基本概念/02_ddp.ipynb:28-31`, which the reference describes but never runs).

Every rank computes gradients on its shard of the batch; the gradients meet on the server rank as ONE
reduce per dtype (a persistent flat buffer), the server alone runs the optimizer, and the updated
parameters go back as ONE broadcast per dtype.  Workers therefore hold no optimizer state (the server's
Adam moments live on one GPU only — with 288 GB of HBM a single server rank holds the whole state of a
model that DDP would replicate N times).

Transport: on GPUs the reduce and the broadcast run on the framework's own RCCL communicator
(``comm.py``, ``ncclReduce`` / ``ncclBroadcast`` on its comm stream, stream-ordered after the backward and
before the optimizer, each under a watchdog ticket that retires on the GPU's completion event), like
every other strategy's collectives; c10d serves CPU tensors (gloo) and ``PDA_COMM=c10d``.

Traffic: reduce-to-root + broadcast moves 2x the gradient bytes through the server's links, the same as
a ring all-reduce moves per rank; over xGMI's point-to-point links RCCL runs both as trees/rings, so the
server is not a single-link bottleneck.  DDP (parallel/ddp.py) overlaps its all-reduce with backward and
is the faster choice when every rank can hold the optimizer state; this mode trades that overlap for
optimizer-state memory.

Semantics kept from single-process training: a parameter that no rank produced a gradient for keeps
``grad = None`` on the server (its optimizer leaves it untouched — no momentum / weight decay step); a
"has grad" flag per parameter rides at the end of the reduced buffer.  Frozen parameters are synced from
the server once at construction, with the rest of the module state.

    ps = ParameterServer(model, lambda params: SGD(params, lr=0.1), server=0)
    loss = F.cross_entropy(ps(x), y); loss.backward(); ps.step(); ps.zero_grad()
"""
from collections import OrderedDict
from typing import Callable, Iterable, List, Optional

import torch
import torch.distributed as dist

from .. import comm as _comm
from ..utils import watchdog as _watchdog


def _unflat_into(flat: torch.Tensor, ts: List[torch.Tensor]):
    o = 0
    for t in ts:
        n = t.numel()
        t.copy_(flat[o:o + n].view_as(t))
        o += n


class ParameterServer(torch.nn.Module):
    """Wrap ``module``; ``optimizer_factory(params)`` is called on the server rank only.

    ``step()`` (after ``backward``): reduce the averaged gradients to ``server``, step the server's
    optimizer, broadcast the parameters.  At construction the server's parameters (trainable and frozen)
    and buffers are broadcast so every rank starts from the same state (as DDP does)."""

    def __init__(self, module: torch.nn.Module, optimizer_factory: Callable[[Iterable], object],
                 server: int = 0, group: Optional[dist.ProcessGroup] = None, broadcast_buffers: bool = True):
        super().__init__()
        self.module = module
        self.group = group
        self.server = server
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.broadcast_buffers = broadcast_buffers
        self._params = [p for p in module.parameters() if p.requires_grad]
        self._by_dtype = OrderedDict()
        for p in self._params:
            self._by_dtype.setdefault((p.dtype, p.device), []).append(p)
        # persistent flat gradient buffers: [grads of the group..., one has-grad flag per parameter]
        self._gbuf = {k: torch.empty(sum(p.numel() for p in ps) + len(ps), dtype=k[0], device=k[1])
                      for k, ps in self._by_dtype.items()}
        self.optimizer = optimizer_factory(self._params) if self.is_server else None
        self.steps = 0
        self.comm_bytes = 0
        self._ncomm = None
        cuda = [k for k in self._by_dtype if k[1].type == "cuda"]
        if cuda and _comm.enabled():
            self._ncomm = _comm.try_for_group(group, cuda[0][1])
        self._sync_state()

    @property
    def is_server(self) -> bool:
        return self.rank == self.server

    @property
    def native(self) -> bool:
        """True when the collectives run on the framework's RCCL communicator."""
        return self._ncomm is not None

    def _global_src(self) -> int:
        return dist.get_global_rank(self.group, self.server) if self.group is not None else self.server

    def _use_native(self, t: torch.Tensor) -> bool:
        return self._ncomm is not None and t.is_cuda and t.device == self._ncomm.device

    def _enqueue(self, what: str, t: torch.Tensor, fn):
        """Run one collective on the native comm stream under a watchdog ticket; the current stream waits
        for its result (no host blocking)."""
        work = fn()
        _watchdog.track(f"param-server {what} ({t.numel() * t.element_size() / 2**20:.1f} MB, {t.dtype})",
                        self._ncomm.stream)
        work.wait()

    @torch.no_grad()
    def _broadcast(self, ts: List[torch.Tensor]):
        if not ts:
            return
        flat = torch.cat([t.reshape(-1) for t in ts])
        if self._use_native(flat):
            self._enqueue("broadcast", flat, lambda: self._ncomm.broadcast(flat, self.server))
        else:
            dist.broadcast(flat, self._global_src(), group=self.group)
        self.comm_bytes += flat.numel() * flat.element_size()
        if not self.is_server:
            _unflat_into(flat, ts)

    @torch.no_grad()
    def _sync_state(self):
        groups = OrderedDict()
        for p in self.module.parameters():  # trainable AND frozen: every rank starts from the server's model
            groups.setdefault((p.dtype, p.device), []).append(p.data)
        for ps in groups.values():
            self._broadcast(ps)
        self._broadcast_buffers()

    @torch.no_grad()
    def _broadcast_buffers(self):
        if not self.broadcast_buffers:
            return
        bufs = OrderedDict()
        for b in self.module.buffers():
            bufs.setdefault((b.dtype, b.device), []).append(b)
        for bs in bufs.values():
            self._broadcast(bs)

    def forward(self, *args, **kwargs):
        return self.module(*args, **kwargs)

    @torch.no_grad()
    def _reduce(self, key, ps: List[torch.nn.Parameter]):
        flat = self._gbuf[key]
        n = flat.numel() - len(ps)
        o = 0
        for p in ps:
            k = p.numel()
            if p.grad is not None:
                flat[o:o + k].copy_(p.grad.reshape(-1))
            else:
                flat[o:o + k].zero_()
            o += k
        flat[n:].copy_(torch.tensor([p.grad is not None for p in ps], dtype=flat.dtype), non_blocking=True)
        if self._use_native(flat):
            self._enqueue("reduce", flat, lambda: self._ncomm.reduce(flat, self.server, op="avg"))
        else:
            dist.reduce(flat, self._global_src(), op=dist.ReduceOp.SUM, group=self.group)
            if self.is_server:
                flat[:n].div_(self.world)
        self.comm_bytes += flat.numel() * flat.element_size()
        if not self.is_server:
            return
        has = (flat[n:] != 0).tolist()  # the only host sync: which parameters any rank produced a gradient for
        o = 0
        for p, h in zip(ps, has):
            k = p.numel()
            if not h:
                p.grad = None  # no rank touched it: the server's optimizer skips it, as single-process training does
            elif p.grad is None:
                p.grad = flat[o:o + k].view_as(p).clone()
            else:
                p.grad.copy_(flat[o:o + k].view_as(p))
            o += k

    @torch.no_grad()
    def step(self):
        """Reduce gradients to the server, update there, broadcast the new parameters."""
        for key, ps in self._by_dtype.items():
            self._reduce(key, ps)
        if self.is_server:
            self.optimizer.step()
        for ps in self._by_dtype.values():
            self._broadcast([p.data for p in ps])
        self._broadcast_buffers()  # running statistics (BN) follow the server's copy, as in DDP
        self.steps += 1

    def zero_grad(self, set_to_none: bool = True):
        for p in self._params:
            if set_to_none:
                p.grad = None
            elif p.grad is not None:
                p.grad.zero_()
