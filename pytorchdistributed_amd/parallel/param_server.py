"""Synchronous parameter-server training (the PS-worker concept of
`/root/reference/02 DDP基本概念/02_ddp.ipynb:28-31`, which the reference describes but never runs).

Every rank computes gradients on its shard of the batch; the gradients meet on the server rank as ONE
sum-reduce per dtype (coalesced flat buffer), the server alone runs the optimizer, and the updated
parameters go back as ONE broadcast per dtype.  Workers therefore hold no optimizer state (the server's
Adam moments live on one GPU only — with 288 GB of HBM a single server rank holds the whole state of a
model that DDP would replicate N times).

Traffic: reduce-to-root + broadcast moves 2x the gradient bytes through the server's links, the same as
a ring all-reduce moves per rank; over xGMI's point-to-point links RCCL runs both as trees/rings, so the
server is not a single-link bottleneck.  DDP (parallel/ddp.py) overlaps its all-reduce with backward and
is the faster choice when every rank can hold the optimizer state; this mode trades that overlap for
optimizer-state memory.

    ps = ParameterServer(model, lambda params: SGD(params, lr=0.1), server=0)
    loss = F.cross_entropy(ps(x), y); loss.backward(); ps.step(); ps.zero_grad()
"""
from collections import OrderedDict
from typing import Callable, Iterable, List, Optional

import torch
import torch.distributed as dist


def _flat(ts: List[torch.Tensor]) -> torch.Tensor:
    return torch.cat([t.reshape(-1) for t in ts]) if len(ts) > 1 else ts[0].reshape(-1).clone()


def _unflat_into(flat: torch.Tensor, ts: List[torch.Tensor]):
    o = 0
    for t in ts:
        n = t.numel()
        t.copy_(flat[o:o + n].view_as(t))
        o += n


class ParameterServer(torch.nn.Module):
    """Wrap ``module``; ``optimizer_factory(params)`` is called on the server rank only.

    ``step()`` (after ``backward``): reduce the averaged gradients to ``server``, step the server's
    optimizer, broadcast the parameters.  At construction the server's parameters and buffers are
    broadcast so every rank starts from the same state (as DDP does)."""

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
        self.optimizer = optimizer_factory(self._params) if self.is_server else None
        self.steps = 0
        self.comm_bytes = 0
        self._sync_state()

    @property
    def is_server(self) -> bool:
        return self.rank == self.server

    def _global_src(self) -> int:
        return dist.get_global_rank(self.group, self.server) if self.group is not None else self.server

    @torch.no_grad()
    def _broadcast(self, ts: List[torch.Tensor]):
        if not ts:
            return
        flat = _flat(ts)
        dist.broadcast(flat, self._global_src(), group=self.group)
        self.comm_bytes += flat.numel() * flat.element_size()
        if not self.is_server:
            _unflat_into(flat, ts)

    @torch.no_grad()
    def _sync_state(self):
        for ps in self._by_dtype.values():
            self._broadcast([p.data for p in ps])
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
    def step(self):
        """Reduce gradients to the server, update there, broadcast the new parameters."""
        for ps in self._by_dtype.values():
            grads = [p.grad if p.grad is not None else torch.zeros_like(p) for p in ps]
            flat = _flat(grads)
            dist.reduce(flat, self._global_src(), op=dist.ReduceOp.SUM, group=self.group)
            self.comm_bytes += flat.numel() * flat.element_size()
            if self.is_server:
                flat.div_(self.world)
                for p, g in zip(ps, grads):
                    if p.grad is None:
                        p.grad = g
                _unflat_into(flat, [p.grad for p in ps])
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
