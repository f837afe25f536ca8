"""FullyShardedDataParallel, full-shard (ZeRO-3) (BASELINE config 4
"Llama-3 8B FSDP full-shard on 8xMI355X").

Per *unit* (every submodule whose type is in ``unit_types`` — e.g. each transformer block — plus a
root unit holding the remaining parameters):

* the unit's parameters are flattened (16-byte aligned, padded to a multiple of the world size) and
  each rank keeps ONE shard in the compute dtype, which is the ``nn.Parameter`` the optimizer sees:
  the fused AdamW keeps the fp32 master of the shard and writes the bf16 shard in the same launch, so
  the shard is all-gathered as is (no per-step cast kernel);
* the module's parameters become persistent leaf tensors whose storage is a view of the unit's
  gathered flat buffer; before the unit's forward the shard is all-gathered (RCCL over xGMI) into
  that buffer (at world 1 the buffer IS the shard: nothing is copied);
* every leaf's gradient lands in its slot of ONE flat gradient buffer per unit — the native
  conv/linear/norm/embedding backward kernels write it there directly (``flat.grad_target``), any
  other op's gradient is copied in by the leaf's post-accumulate hook — so there is no autograd
  ``cat`` of the unit's gradients and no fp32 round trip;
* after forward the gathered storage is released (``reshard_after_forward``) and re-gathered in place
  when the unit's backward starts (hook on the unit output), so saved views see the right bytes;
* when the unit's last leaf gradient arrived the flat gradient is reduce-scattered (average) straight
  into the shard's grad; the next unit's all-gather is prefetched while the current unit computes
  (forward order recorded on the first iteration, reversed for backward).

Collectives run on the native RCCL communicator's stream (comm.py): the all-gathers (prefetch
included) and the reduce-scatters queue there in issue order; a unit's reduce-scatter never makes the
compute stream wait — the shard gradients are collected once, in the final backward callback.

Memory per rank for Llama-3 8B: 8.03e9 x (2 B shard + 4 B master + 8 B Adam) / 8 ~= 14 GB, plus the
gradient buffers of the units whose backward / reduce-scatter is in flight (allocated at the unit's
backward, released once its reduce-scatter is queued) and the gathered units in flight: a small
fraction of the 288 GB HBM.
Checkpoints: :meth:`full_state_dict` (consolidated, original names), :meth:`save_sharded` /
:meth:`load_sharded` (``shard_{rank:05d}.pt`` with the rank's optimizer state — fp32 master, Adam
moments, step — + ``meta.json``: an exact resume), :func:`consolidate` (model only) and
:func:`consolidate_snapshot` (the stock ``{"MODEL_STATE", "OPTIMIZER_STATE"}`` file).
"""
from __future__ import annotations

import contextlib
import json
import os
from typing import Dict, List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist
import torch.nn as tnn

from .. import distributed as pdist
from ..ops import streams as _streams
from ..utils import watchdog as _watchdog

ALIGN = 8


def _round(n, a):
    return (n + a - 1) // a * a


class _StreamWork:
    """Work handle of a side-stream collective: wait() orders the current stream after it."""

    def __init__(self, event):
        self.event = event

    def wait(self):
        torch.cuda.current_stream().wait_event(self.event)

    def is_completed(self):
        return self.event.query()


def _join_side_streams(units) -> None:
    """A backward that raised never ran its final callback, so its side-stream weight gradients were
    never joined: order the compute stream after them before anything reuses the buffers."""
    devs = {leaf.device for u in units for leaf in u.leaves if leaf.is_cuda}
    for d in devs:
        _streams.join(d)


class _Slot:
    """One slot of the FSDP gradient ring: the buffer and the reduce-scatter that last read it."""

    def __init__(self, buf: torch.Tensor):
        self.buf, self.work = buf, None


class _Unit:
    def __init__(self, fsdp: "FullyShardedDataParallel", module: tnn.Module, params: List[Tuple[tnn.Module, str]],
                 index: int):
        self.fsdp, self.module, self.index = fsdp, module, index
        self.entries = []  # (owner module, attr name, shape, offset, numel)
        off = 0
        first = getattr(params[0][0], params[0][1])
        deferred = first.is_meta
        self.device = fsdp.init_device if deferred else first.device
        for owner, name in params:
            p = getattr(owner, name)
            self.entries.append((owner, name, tuple(p.shape), off, p.numel()))
            off += _round(p.numel(), ALIGN)
        W = fsdp.world
        self.numel = _round(max(off, 1), W * ALIGN)
        self.shard_numel = self.numel // W
        r = fsdp.rank
        if deferred:
            # deferred construction: materialise THIS unit only, as views of one compute-dtype buffer, let
            # the model initialise it (identical on every rank: per-unit seeded streams), keep this rank's
            # shard and drop the rest — a rank never holds more than one full unit plus its shards
            full = torch.zeros(self.numel, dtype=fsdp.param_dtype, device=self.device)
            for (owner, name, shape, o, n) in self.entries:
                rg = owner._parameters[name].requires_grad
                owner._parameters[name] = tnn.Parameter(full[o: o + n].view(shape), requires_grad=rg)
            fsdp.param_init_fn(module, index)
            fsdp._note_init(full.numel() * full.element_size())
        else:
            full = torch.zeros(self.numel, dtype=torch.float32, device=self.device)
            for (owner, name, shape, o, n) in self.entries:
                full[o: o + n].copy_(getattr(owner, name).detach().reshape(-1).float())
        self.shard = tnn.Parameter(full[r * self.shard_numel: (r + 1) * self.shard_numel].to(fsdp.shard_dtype,
                                                                                              copy=True))
        del full
        fsdp._shard_bytes += self.shard.numel() * self.shard.element_size()
        for (owner, name, *_rest) in self.entries:
            del owner._parameters[name]
        # world 1 with a compute-dtype shard: the shard itself is the gathered buffer (no copy, never freed)
        self.alias = not fsdp.comm_on and fsdp.shard_dtype == fsdp.param_dtype
        self.flat = self.shard.detach() if self.alias else torch.empty(self.numel, dtype=fsdp.param_dtype,
                                                                       device=self.device)
        # flat gradient buffer (every slot is fully rewritten each backward; the alignment padding is
        # zeroed whenever the storage is (re)allocated).  Transient above world 1: allocated when the
        # unit's backward starts, released as soon as its reduce-scatter is queued (the comm stream
        # keeps it alive until the collective has read it), so a rank holds the gradient of the units
        # in flight, not of the whole model (the root unit's, whose leaves get gradients at both ends
        # of backward, stays resident)
        self.grad_buffer = torch.zeros(self.numel, dtype=fsdp.param_dtype, device=self.device)
        covered = torch.zeros(self.numel, dtype=torch.bool)
        for (_owner, _name, _shape, o, n) in self.entries:
            covered[o: o + n] = True
        self.pad_index = (~covered).nonzero().flatten().to(self.device)
        self.transient_grad = False  # set by the FSDP wrapper for non-root units at world > 1
        self.arrived = 0
        # persistent leaf tensors (plain tensors, not registered Parameters: the optimizer sees only the
        # shard) viewing the gathered buffer; `_pda_flat` routes native backward kernels to the grad slot
        self.leaves: List[torch.Tensor] = []
        for (owner, name, shape, o, n) in self.entries:
            # (`.data =` gives the leaf the view's storage but its OWN version counter: re-filling the
            # gathered buffer in place is not an update of the parameter as far as saved tensors go)
            leaf = torch.empty(0, dtype=fsdp.param_dtype, device=self.device).requires_grad_(True)
            leaf.data = self.flat[o: o + n].view(shape)
            leaf._pda_flat = (self, o)
            leaf.register_post_accumulate_grad_hook(self._make_leaf_hook(o, n, shape))
            setattr(owner, name, leaf)
            self.leaves.append(leaf)
        self.gathered = self.alias
        if not self.alias:
            self.flat.untyped_storage().resize_(0)
        self.pending_ag = None
        self.ag_reg = self.rs_reg = None  # zero-copy IPC registrations (PDA_FSDP_COMM=ipc)
        self.ring = False  # gathered buffer is a slot of the FSDP ring (FullyShardedDataParallel._enable_ring)
        self.grad_slot = None  # gradient-ring slot (native RCCL path)
        # compute-dtype copy of an fp32 shard, made by the forward gather and reused by the backward
        # re-gather of the same step.  Invalidated at every forward entry: fused optimizers update the
        # shard through raw pointers, which does not bump its autograd version counter.
        self._cast = None

    def _make_leaf_hook(self, o: int, n: int, shape):
        def hook(t: torch.Tensor):
            slot = self.grad_buffer[o: o + n]
            g = t.grad
            if g is not None and g.data_ptr() != slot.data_ptr():
                slot.view(shape).copy_(g)
            t.grad = None  # the slot holds it; a None .grad lets the next backward write in place again
            t._pda_claimed = False
            t._pda_seen = True
            self.arrived += 1
            if self.arrived == len(self.leaves):
                self.fsdp._grad_ready(self)
        return hook

    def flush_missing(self):
        """Backward ended with some leaves unused: zero their slots and reduce-scatter anyway (every
        rank runs the same graph, so the collectives still match)."""
        if 0 < self.arrived < len(self.leaves):
            # leaves whose hook did not fire still hold an earlier step's slot contents
            fired = set()
            for leaf, (_o, _n, _s, o, n) in zip(self.leaves, self.entries):
                if getattr(leaf, "_pda_seen", False):
                    fired.add(o)
            for (_o, _n, _s, o, n) in self.entries:
                if o not in fired:
                    self.grad_buffer[o: o + n].zero_()
            self.arrived = len(self.leaves)
            self.fsdp._grad_ready(self)

    def alloc_grad(self):
        """(Re)allocate a released gradient buffer (zero padding) before the unit's backward writes it.
        Ring mode: the unit's slot of the gradient ring; the compute stream first waits for the
        reduce-scatter of the slot's previous user (long done with 3 slots)."""
        if self.grad_slot is not None:
            slot = self.grad_slot
            if slot.work is not None:
                slot.work.wait()
                slot.work = None
            if self.pad_index.numel():
                self.grad_buffer.index_fill_(0, self.pad_index, 0)
            return
        st = self.grad_buffer.untyped_storage()
        if st.size() == 0:
            st.resize_(self.numel * self.grad_buffer.element_size())
            if self.pad_index.numel():
                self.grad_buffer.index_fill_(0, self.pad_index, 0)

    def release_grad(self):
        if self.grad_slot is not None:
            return  # the ring slot stays; its next user waits for this unit's reduce-scatter
        if self.transient_grad:
            self.grad_buffer.untyped_storage().resize_(0)

    def _send_buffer(self) -> torch.Tensor:
        if self.shard.dtype == self.fsdp.param_dtype:
            return self.shard.detach()
        if self._cast is None:  # fp32 shards (shard_dtype=float32): one cast per step, reused by backward
            self._cast = self.shard.detach().to(self.fsdp.param_dtype)
        return self._cast

    # ------------------------------------------------------------ gather / reshard
    def start_gather(self):
        if self.gathered or self.pending_ag is not None:
            return
        if self.flat.untyped_storage().size() == 0:
            self.flat.untyped_storage().resize_(self.numel * self.flat.element_size())
        with torch.no_grad():
            send = self._send_buffer()
            self.fsdp._count(self.flat)
            if not self.fsdp.comm_on:
                self.flat.copy_(send)
                self.gathered = True
            elif self.fsdp.xgmi is not None:
                flat = self.flat
                reg = self.ag_reg
                if reg is not None:  # zero-copy: the peers' shards are read in place
                    fn = lambda: self.fsdp.xgmi.all_gather_registered(reg, flat, send)  # noqa: E731
                else:
                    fn = lambda: self.fsdp.xgmi.all_gather_into_tensor(flat, send)  # noqa: E731
                self.pending_ag = self.fsdp._ipc(fn, [torch.cuda.current_stream(self.device)], [send, flat],
                                                 ("ag", self.index))
                self.fsdp._track("xgmi all_gather", self, self.fsdp._ipc_stream)
            elif self.fsdp.ncomm is not None:
                self.pending_ag = self.fsdp.ncomm.all_gather(self.flat, send)
                self.fsdp._track("all_gather", self, self.fsdp.ncomm.stream)
            else:
                self.pending_ag = dist.all_gather_into_tensor(self.flat, send, group=self.fsdp.group,
                                                              async_op=True)

    def finish_gather(self):
        if self.pending_ag is not None:
            with self.fsdp._exposed(), self.fsdp._watch_c10d(f"all_gather unit {self.index}"):
                self.pending_ag.wait()
            self.pending_ag = None
            self.gathered = True
        elif not self.gathered:
            self.start_gather()
            self.finish_gather()

    def reshard(self):
        if self.alias:
            return
        if self.ring:  # the slot belongs to the ring: nothing is freed, the next gather overwrites it
            self.gathered = False
            return
        if self.gathered:
            self.flat.untyped_storage().resize_(0)
        self.gathered = False


class FullyShardedDataParallel(tnn.Module):
    def __init__(self, module: tnn.Module, process_group=None, unit_types: Sequence[type] = (),
                 param_dtype: Optional[torch.dtype] = None, reshard_after_forward: bool = True,
                 prefetch: bool = True, shard_dtype: Optional[torch.dtype] = None, param_init_fn=None,
                 device: Optional[torch.device] = None):
        """``param_dtype``: compute dtype of the gathered parameters (default: the module's).
        ``shard_dtype``: dtype of the sharded ``nn.Parameter`` the optimizer updates (default: the
        compute dtype — the fused optimizers then keep fp32 masters themselves and write the shard in
        the same launch; ``torch.float32`` keeps fp32 shards and casts them once per step).

        Deferred initialisation (a ``module`` built on the meta device): each unit is materialised on
        ``device`` (default: the current GPU, else the CPU) one at a time, initialised by
        ``param_init_fn(unit_module, unit_index)`` (default: ``module.init_unit``) — which must give every
        rank the same values (e.g. a generator seeded per unit) — and reduced to this rank's shard before
        the next unit exists: peak construction memory is the shards plus ONE full unit, not the model."""
        super().__init__()
        self.module = module
        self.param_init_fn = param_init_fn if param_init_fn is not None else getattr(module, "init_unit", None)
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else \
                torch.device("cpu")
        self.init_device = torch.device(device)
        self.deferred = any(p.is_meta for p in module.parameters())
        if self.deferred and self.param_init_fn is None:
            raise ValueError("a meta-device module needs param_init_fn (or an init_unit(module, index) method)")
        self._shard_bytes = 0
        self.ring_enabled = False
        self.init_peak_bytes = 0  # deferred construction: max bytes held at once (one unit + the shards so far)
        self.group = process_group
        self.world = pdist.get_world_size(process_group)
        self.rank = pdist.get_rank(process_group)
        self.param_dtype = param_dtype or next(module.parameters()).dtype
        self.shard_dtype = shard_dtype or self.param_dtype
        self.reshard_after_forward = reshard_after_forward
        self.prefetch = prefetch
        self.nccl = dist.is_initialized() and dist.get_backend(process_group) == "nccl"
        # PDA_FSDP_FORCE_COMM=1: run the unit all-gathers / reduce-scatters even at world size 1 (a
        # one-rank RCCL group on a one-GPU box executes every ncclAllGather / ncclReduceScatter, stream
        # wait and transient buffer of the multi-GPU path instead of aliasing the shard)
        self.comm_on = self.world > 1 or (os.environ.get("PDA_FSDP_FORCE_COMM") == "1" and dist.is_initialized())
        # communication accounting (comm_stats): bytes / calls, and with PDA_TRACK_COMM=1 (or
        # PDA_METRICS_DIR) the compute-stream time spent waiting on the collectives (exposed comm)
        self.track_comm = bool(os.environ.get("PDA_METRICS_DIR")) or os.environ.get("PDA_TRACK_COMM") == "1"
        self._stats = {"comm_bytes": 0, "comm_calls": 0}
        # PDA_FSDP_IPC_LOG=1: record (kind, unit) of every IPC collective in issue order (debugging the
        # cross-rank op order; unbounded, so off by default)
        self._ipc_log: Optional[List] = [] if os.environ.get("PDA_FSDP_IPC_LOG") == "1" else None
        self._exposed_events: List = []
        self._deferred_release: List = []
        # ---- build units: typed submodules first (outermost match), root takes the rest
        unit_mods, seen = [], set()
        for m in module.modules():
            if unit_types and isinstance(m, tuple(unit_types)) and not any(m is u or _is_child(u, m) for u in unit_mods):
                unit_mods.append(m)
        claimed = set()
        self.units: List[_Unit] = []
        self.names: List[List[str]] = []
        full_names = {id(p): n for n, p in module.named_parameters()}
        for m in unit_mods:
            params = [(owner, name) for owner in m.modules() for name, p in list(owner._parameters.items())
                      if p is not None and id(p) not in claimed]
            for owner, name in params:
                claimed.add(id(getattr(owner, name)))
            if params:
                self.names.append([full_names[id(getattr(o, n))] for o, n in params])
                self.units.append(_Unit(self, m, params, len(self.units)))
        rest = [(owner, name) for owner in module.modules() for name, p in list(owner._parameters.items())
                if p is not None and id(p) not in claimed]
        self.root_unit = None
        if rest:
            self.names.append([full_names[id(getattr(o, n))] for o, n in rest])
            self.root_unit = _Unit(self, module, rest, len(self.units))
            self.units.append(self.root_unit)
        self.shards = tnn.ParameterList([u.shard for u in self.units])
        if self.deferred:
            for mod in module.modules():  # meta buffers (none in the shipped models): zero-filled on the device
                for bn, b in list(mod._buffers.items()):
                    if b is not None and b.is_meta:
                        mod._buffers[bn] = torch.zeros(b.shape, dtype=b.dtype, device=self.init_device)
        # ---- hooks on unit modules
        self._fwd_order: List[_Unit] = []
        self._order_frozen = False
        for u in self.units:
            if u is not self.root_unit:
                u.module.register_forward_pre_hook(self._make_pre_fwd(u))
                u.module.register_forward_hook(self._make_post_fwd(u))
        self._pending_rs: List[tuple] = []  # (unit, work, out) reduce-scatters queued this backward
        self._callback_queued = False
        self._callback_task = -1
        # ---- native RCCL communicator for the unit all-gathers / reduce-scatters (comm.py; ordered on
        # one high-priority comm stream, so a unit's reduce-scatter never makes the compute stream wait:
        # the shard gradients are collected in the final callback).  PDA_COMM=c10d: ProcessGroupNCCL.
        self.ncomm = None
        if self.nccl and all(u.device.type == "cuda" for u in self.units) and self.comm_on:
            from .. import comm as _comm

            if _comm.enabled():
                self.ncomm = _comm.try_for_group(process_group, self.units[0].device)
        for u in self.units:
            u.transient_grad = self.comm_on and u is not self.root_unit
            u.release_grad()
        # ---- optional direct xGMI collectives (PDA_FSDP_COMM=ipc, one node): the unit all-gathers pull
        # every peer's shard over its own link and the gradient reduce-scatters reduce chunk `rank` of
        # every peer's buffer (csrc/kernels/xgmi.hip), on one ordered side stream; RCCL by default
        self.xgmi = None
        if os.environ.get("PDA_FSDP_COMM", "rccl").lower() in ("ipc", "xgmi") and self.world > 1 and \
                process_group is None and all(u.device.type == "cuda" for u in self.units):
            from . import xgmi as _xgmi

            if _xgmi.single_node():
                cap = max(u.numel for u in self.units) * torch.tensor([], dtype=self.param_dtype).element_size()
                self.xgmi = _xgmi.XgmiAllReduce(capacity_mb=cap / 2 ** 20 + 1, device=self.units[0].device)
                self._ipc_stream = torch.cuda.Stream(self.units[0].device)
                if _xgmi.zero_copy():
                    # zero-copy: the shards (all-gather sources) and persistent unit gradient buffers
                    # (reduce-scatter sources) are registered once; peers read them in place
                    for u in self.units:
                        u.transient_grad = False
                        u.alloc_grad()
                        u.ag_reg = (self.xgmi.register(u.shard.detach())
                                    if u.shard.dtype == self.param_dtype and u.shard_numel % 8 == 0 else None)
                        u.rs_reg = self.xgmi.register(u.grad_buffer) if u.numel % (8 * self.world) == 0 else None

    def _note_init(self, unit_bytes: int):
        self.init_peak_bytes = max(self.init_peak_bytes, self._shard_bytes + unit_bytes)

    # ------------------------------------------------------------ communication accounting
    def _count(self, t: torch.Tensor):
        if self.comm_on:
            self._stats["comm_bytes"] += t.numel() * t.element_size()
            self._stats["comm_calls"] += 1

    @contextlib.contextmanager
    def _exposed(self):
        """Brackets a compute-stream wait on a collective: with tracking on, the events' elapsed time
        is how long the compute stream sat behind the communication (SURVEY §5.1 overlap ratio)."""
        if not (self.track_comm and self.comm_on and torch.cuda.is_available() and self.units
                and self.units[0].device.type == "cuda"):
            yield
            return
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        yield
        b.record()
        self._exposed_events.append((a, b))

    def comm_stats(self, reset: bool = True) -> dict:
        """Bytes / calls of the unit all-gathers + reduce-scatters since the last reset and, when
        tracking is on, ``exposed_comm_ms``: compute-stream time spent waiting on them."""
        out = dict(self._stats)
        if self._exposed_events:
            self._exposed_events[-1][1].synchronize()
            out["exposed_comm_ms"] = round(sum(a.elapsed_time(b) for a, b in self._exposed_events), 3)
        if reset:
            self._stats = {"comm_bytes": 0, "comm_calls": 0}
            self._exposed_events = []
        return out

    def _release_completed(self):
        """c10d path: release the transient gradient storage of units whose reduce-scatter finished."""
        keep = []
        for u, work in self._deferred_release:
            if work is None or work.is_completed():
                u.release_grad()
            else:
                keep.append((u, work))
        self._deferred_release = keep

    def _watch_c10d(self, what: str):
        """Deadline for a c10d wait (gloo blocks the host there); native / IPC collectives already carry a
        ticket from their enqueue (:meth:`_track`)."""
        if not self.comm_on or self.ncomm is not None or self.xgmi is not None:
            return contextlib.nullcontext()
        return _watchdog.watch(f"fsdp c10d {what}")

    def _track(self, what: str, u: "_Unit", stream):
        """Watchdog ticket for a unit collective just enqueued on ``stream``: it retires on
        an event the native thread records behind the collective, so a peer that never joins the
        all-gather / reduce-scatter ends in a report + ncclCommAbort + stack dump, not a silent hang in the
        next synchronize."""
        nbytes = (u.numel if "gather" in what else u.shard_numel) * u.flat.element_size()
        _watchdog.track(f"fsdp {what} unit {u.index} ({nbytes / 2**20:.1f} MB)", stream)
        self._stats["tickets"] = self._stats.get("tickets", 0) + 1

    def _ipc(self, fn, producers, tensors, tag=None):
        """Run ``fn`` on the IPC stream after ``producers``; returns a work handle (wait = stream wait)."""
        if tag is not None and self._ipc_log is not None:
            self._ipc_log.append(tag)
        s = self._ipc_stream
        for p in producers:
            s.wait_stream(p)
        for t in tensors:
            t.record_stream(s)
        with torch.cuda.stream(s):
            fn()
            done = torch.cuda.Event()
            done.record(s)
        return _StreamWork(done)

    # ------------------------------------------------------------ forward hooks
    def _next_in_order(self, u: _Unit, backward: bool) -> Optional[_Unit]:
        if not self._order_frozen:
            return None
        order = self._fwd_order[::-1] if backward else self._fwd_order
        try:
            i = order.index(u)
        except ValueError:
            return None
        return order[i + 1] if i + 1 < len(order) else None

    def _make_pre_fwd(self, u: _Unit):
        def hook(mod, args):
            if not self._order_frozen:
                self._fwd_order.append(u)
            u.finish_gather()
            if self.prefetch:
                nxt = self._next_in_order(u, backward=False)
                if nxt is not None:
                    nxt.start_gather()
        return hook

    def _make_post_fwd(self, u: _Unit):
        def hook(mod, args, out):
            if self.reshard_after_forward and torch.is_grad_enabled():
                u.reshard()
            elif not torch.is_grad_enabled():
                u.reshard()
            if torch.is_grad_enabled():
                for t in _tensors(out):
                    if t.requires_grad:
                        t.register_hook(lambda g, u=u: self._pre_backward(u, g))
            return out
        return hook

    def _queue_final(self):
        """One final callback per backward pass, keyed on the autograd graph task (a backward that
        raised never ran its callback: the next pass must queue its own and start clean)."""
        task = torch._C._current_graph_task_id()
        if self._callback_queued and self._callback_task == task:
            return
        if self._callback_queued:  # aborted pass: drop its partial arrivals / pending reduce-scatters
            for _, work, _ in self._pending_rs:  # (their outputs are discarded, but let them finish first)
                if work is not None:
                    work.wait()
            self._pending_rs = []
            deferred, self._deferred_release = self._deferred_release, []
            for du, _work in deferred:
                du.release_grad()
            _join_side_streams(self.units)
            for u in self.units:
                u.arrived = 0
                for leaf in u.leaves:
                    leaf._pda_seen = False
        self._callback_queued = True
        self._callback_task = task
        torch.autograd.Variable._execution_engine.queue_callback(self._post_backward_final)

    def _pre_backward(self, u: _Unit, g):
        u.alloc_grad()
        if not u.gathered:
            u.start_gather()
            u.finish_gather()
        if self.prefetch:
            nxt = self._next_in_order(u, backward=True)
            if nxt is not None and nxt is not self.root_unit:
                nxt.start_gather()
        self._queue_final()
        return g

    # ------------------------------------------------------------ gradient reduce-scatter
    def _grad_ready(self, u: _Unit):
        grad_full = u.grad_buffer
        if not self.comm_on:
            # the shard's gradient IS the flat gradient buffer (no copy); the slots were just rewritten,
            # so a gradient still held from an earlier backward cannot be accumulated into
            if u.shard.grad is not None and u.shard.grad.data_ptr() == grad_full.data_ptr():
                raise RuntimeError("FSDP at world size 1 does not accumulate gradients across backward "
                                   "passes: call zero_grad(set_to_none=True) between steps")
            self._pending_rs.append((u, None, grad_full))
            self._queue_final()
            return
        out = torch.empty(u.shard_numel, dtype=grad_full.dtype, device=grad_full.device)
        # weight gradients of this unit may still be running on the side stream (ops/streams.py): the
        # collective is ordered after both streams
        producers = _streams.producer_streams(grad_full.device) if grad_full.is_cuda else []
        if self.xgmi is not None:
            if u.rs_reg is not None:  # zero-copy: every peer's gradient buffer read in place
                fn = lambda: self.xgmi.reduce_scatter_registered(u.rs_reg, out, grad_full, average=True)  # noqa: E731
            else:
                fn = lambda: self.xgmi.reduce_scatter_tensor(out, grad_full, average=True)  # noqa: E731
            work = self._ipc(fn, producers, [out, grad_full], ("rs", u.index))
            self._track("xgmi reduce_scatter", u, self._ipc_stream)
        elif self.ncomm is not None:
            work = self.ncomm.reduce_scatter(out, grad_full, "avg", streams=producers)
            self._track("reduce_scatter", u, self.ncomm.stream)
        else:
            ctx = contextlib.nullcontext()
            if len(producers) > 1:
                if self.nccl:  # RCCL waits on the current stream: make it the side stream, after main
                    producers[1].wait_stream(producers[0])
                    ctx = torch.cuda.stream(producers[1])
                    out.record_stream(producers[1])
                    grad_full.record_stream(producers[1])
                else:
                    producers[0].wait_stream(producers[1])
            with ctx:
                if self.nccl:
                    work = dist.reduce_scatter_tensor(out, grad_full, op=dist.ReduceOp.AVG, group=self.group,
                                                      async_op=True)
                else:
                    work = dist.reduce_scatter_tensor(out, grad_full, group=self.group, async_op=True)
        self._count(grad_full)
        self._pending_rs.append((u, work, out))
        if u.grad_slot is not None:
            u.grad_slot.work = work  # the slot's next user waits for this reduce-scatter
        if self.xgmi is not None or self.ncomm is not None:
            u.release_grad()  # record_stream on the collective's stream holds the storage until it is read
        else:
            # c10d: with TORCH_NCCL_AVOID_RECORD_STREAMS=1 (and on gloo) nothing ties the storage to the
            # in-flight collective, so a unit's storage is released once ITS collective has completed
            # (polled here at every later unit, the rest in _finish_rs) — never the whole unsharded
            # gradient held to the end of backward
            self._release_completed()
            self._deferred_release.append((u, work))
        if u is not self.root_unit:
            u.reshard()
        self._queue_final()

    def _finish_rs(self):
        """Collect every queued reduce-scatter into its shard's gradient (the compute stream waits on
        the collectives here, once, at the end of backward)."""
        pending, self._pending_rs = self._pending_rs, []
        with self._exposed(), self._watch_c10d(f"reduce_scatter x{len(pending)}"):
            for _u, work, _out in pending:
                if work is not None:
                    work.wait()
        deferred, self._deferred_release = self._deferred_release, []
        for u, _work in deferred:
            u.release_grad()
        for u, work, out in pending:
            if not self.nccl and self.xgmi is None and self.world > 1:
                out.div_(self.world)
            g = out if out.dtype == u.shard.dtype else out.to(u.shard.dtype)
            if u.shard.grad is None:
                u.shard.grad = g
            else:
                u.shard.grad.add_(g)

    def _post_backward_final(self):
        self._callback_queued = False
        for u in self.units:
            u.flush_missing()
        self._finish_rs()
        if self.xgmi is not None and self.xgmi.poll():
            # a peer barrier of an IPC gather / reduce-scatter timed out: that call's output is garbage
            # (the kernels give up instead of hanging) — fail the step rather than train on it
            self.xgmi.check(sync=False)
        for u in self.units:
            u.reshard()
            u.arrived = 0
            for leaf in u.leaves:
                leaf._pda_seen = False
        if not self._order_frozen:
            self._order_frozen = True
            self._enable_ring()

    def _enable_ring(self):
        """Preallocated rings for the transient unit buffers, once the first iteration has
        recorded the forward order: the gathered parameters of the unit at forward position p live in
        slot p % 2 of a 2-slot ring (the unit computing + the one prefetched), and its flat gradient in
        slot p % 3 of a 3-slot ring (native RCCL path) — instead of a caching-allocator block per gather /
        backward, which, with record_stream holding every block until the collective has run, fragmented
        the pool (286 GiB reserved for a 190 GiB peak, one allocator retry in the timed steps at world 1).

        Why fixed slots are safe: a unit's leaves (and every tensor autograd saved from them) view its
        slot, and are only read while that unit computes — forward, or its backward after the re-gather
        into the same slot.  Between two uses the slot carries other units, but a gather into slot s is
        enqueued on the comm stream after every kernel already queued on the compute stream, i.e. after
        the previous user of s (position p - 2) has finished; the prefetched unit (p +- 1) is always in the
        other slot.  ``PDA_FSDP_RING=0`` keeps the allocator path."""
        if os.environ.get("PDA_FSDP_RING", "1") == "0" or not self.comm_on or not self.reshard_after_forward \
                or self.xgmi is not None:
            return
        order = [u for u in self._fwd_order if u is not self.root_unit]
        units = [u for u in self.units if u is not self.root_unit]
        if len(order) < 3 or len(order) != len(units) or len({id(u) for u in order}) != len(order) or \
                any(u.alias for u in order):
            return
        dev = order[0].device
        n = max(u.numel for u in order)
        self._flat_slots = [torch.empty(n, dtype=self.param_dtype, device=dev) for _ in range(2)]
        grad_ring = self.ncomm is not None
        if grad_ring:
            self._grad_slots = [_Slot(torch.zeros(n, dtype=self.param_dtype, device=dev)) for _ in range(3)]
        for pos, u in enumerate(order):
            u.flat = self._flat_slots[pos % 2][: u.numel]
            for leaf, (_o, _n, shape, o, k) in zip(u.leaves, u.entries):
                leaf.data = u.flat[o: o + k].view(shape)
            u.ring = True
            u.gathered = False
            if grad_ring:
                u.grad_buffer.untyped_storage().resize_(0)
                slot = self._grad_slots[pos % 3]
                u.grad_buffer = slot.buf[: u.numel]
                u.grad_slot = slot
        self.ring_enabled = True

    # ------------------------------------------------------------ module API
    def forward(self, *args, **kwargs):
        for u in self.units:
            u._cast = None
        if self.root_unit is not None:
            self.root_unit.finish_gather()
        if self._order_frozen and self.prefetch and self._fwd_order:
            self._fwd_order[0].start_gather()
        out = self.module(*args, **kwargs)
        if not self._order_frozen and not torch.is_grad_enabled():
            self._order_frozen = True
        return out

    # ------------------------------------------------------------ state dicts
    @torch.no_grad()
    def full_state_dict(self) -> Dict[str, torch.Tensor]:
        """All-gather every unit; returns {original name: fp32 tensor} (on every rank)."""
        out = {}
        for u, names in zip(self.units, self.names):
            full = torch.empty(u.numel, dtype=u.shard.dtype, device=u.device)
            if self.world == 1:
                full.copy_(u.shard)
            else:
                dist.all_gather_into_tensor(full, u.shard.detach(), group=self.group)
            full = full.float()
            for (owner, name, shape, o, n), full_name in zip(u.entries, names):
                out[full_name] = full[o: o + n].view(shape).clone().cpu()
        return out

    def sharded_state_dict(self, optimizer=None) -> Dict[str, object]:
        """This rank's shards and, with ``optimizer``, its state for them (fp32 master, Adam moments,
        step) and the param-group hyperparameters: everything a bit-exact resume needs."""
        sd: Dict[str, object] = {f"unit{u.index}": u.shard.detach().cpu() for u in self.units}
        if optimizer is not None:
            ost = {}
            for u in self.units:
                st = optimizer.state.get(u.shard, {})
                ost[f"unit{u.index}"] = {k: (v.detach().cpu().clone() if torch.is_tensor(v) else torch.tensor(v))
                                         for k, v in st.items()}
            sd["optim"] = ost
            sd["param_groups"] = [{k: v for k, v in g.items() if k != "params"} for g in optimizer.param_groups]
        return sd

    def save_sharded(self, directory: str, optimizer=None):
        """``shard_{rank:05d}.pt`` per rank (+ optimizer state) and ``meta.json`` (layout of units and of
        the optimizer state) from rank 0."""
        os.makedirs(directory, exist_ok=True)
        sd = self.sharded_state_dict(optimizer)
        tmp = os.path.join(directory, f"shard_{self.rank:05d}.pt.tmp")
        torch.save(sd, tmp)
        os.replace(tmp, os.path.join(directory, f"shard_{self.rank:05d}.pt"))
        if self.rank == 0:
            meta = {"world_size": self.world, "units": [
                {"numel": u.numel, "shard_numel": u.shard_numel,
                 "params": [{"name": nm, "shape": list(e[2]), "offset": e[3], "numel": e[4]}
                            for e, nm in zip(u.entries, names)]} for u, names in zip(self.units, self.names)]}
            if optimizer is not None:
                # which param group each unit's shard belongs to (consolidate_snapshot maps every
                # parameter of the unit to that group)
                for um, u in zip(meta["units"], self.units):
                    um["param_group"] = next((gi for gi, g in enumerate(optimizer.param_groups)
                                              if any(q is u.shard for q in g["params"])), 0)
                st0 = sd["optim"]["unit0"]
                meta["optimizer"] = {
                    "type": type(optimizer).__name__,
                    "state": {k: {"dtype": str(v.dtype).replace("torch.", ""), "per_element": v.dim() > 0}
                              for k, v in st0.items()},
                    "param_groups": [{k: v for k, v in g.items() if isinstance(v, (int, float, bool, str, list, tuple))}
                                     for g in sd["param_groups"]]}
            with open(os.path.join(directory, "meta.json"), "w") as f:
                json.dump(meta, f, indent=1)

    @torch.no_grad()
    def load_sharded(self, directory: str, optimizer=None):
        sd = torch.load(os.path.join(directory, f"shard_{self.rank:05d}.pt"), map_location="cpu", weights_only=True)
        for u in self.units:
            u.shard.copy_(sd[f"unit{u.index}"])
            u._cast = None
        if optimizer is not None and "optim" in sd:
            for u in self.units:
                st = optimizer.state[u.shard]
                for k, v in sd["optim"][f"unit{u.index}"].items():
                    if k == "step" and v.dim() == 0:
                        st[k] = int(v.item()) if v.dtype in (torch.int64, torch.int32) else float(v.item())
                    else:
                        st[k] = v.to(u.shard.device)
            for g, saved in zip(optimizer.param_groups, sd.get("param_groups", [])):
                g.update(saved)


def consolidate(directory: str) -> Dict[str, torch.Tensor]:
    """Offline: merge ``shard_*.pt`` + ``meta.json`` into one {name: tensor} state dict (CPU)."""
    meta = json.load(open(os.path.join(directory, "meta.json")))
    W = meta["world_size"]
    shards = [torch.load(os.path.join(directory, f"shard_{r:05d}.pt"), map_location="cpu", weights_only=True)
              for r in range(W)]
    out = {}
    for i, u in enumerate(meta["units"]):
        full = torch.cat([s[f"unit{i}"] for s in shards])
        for p in u["params"]:
            out[p["name"]] = full[p["offset"]: p["offset"] + p["numel"]].view(p["shape"]).clone()
    return out


def consolidate_snapshot(directory: str, path: Optional[str] = None) -> Dict[str, object]:
    """Offline: merge a sharded checkpoint saved WITH its optimizer into the framework's single-file
    snapshot layout ``{"MODEL_STATE", "OPTIMIZER_STATE", "EPOCHS_RUN"}`` (utils/checkpoint.py), the
    optimizer state in torch's format (parameter index = order of ``MODEL_STATE``; per-element state
    such as ``exp_avg`` / ``master_param`` un-sharded to each parameter's shape).  Written to ``path``
    when given."""
    meta = json.load(open(os.path.join(directory, "meta.json")))
    W = meta["world_size"]
    shards = [torch.load(os.path.join(directory, f"shard_{r:05d}.pt"), map_location="cpu", weights_only=True)
              for r in range(W)]
    model, ostate, pi = {}, {}, 0
    saved_groups = shards[0].get("param_groups", [{}]) or [{}]
    group_params: List[List[int]] = [[] for _ in saved_groups]
    if len(saved_groups) > 1 and any("param_group" not in u for u in meta["units"]):
        raise ValueError("checkpoint has several optimizer param groups but meta.json does not record "
                         "which group each unit belongs to (saved by an older version)")
    for i, u in enumerate(meta["units"]):
        gi = int(u.get("param_group", 0))
        full = torch.cat([s_[f"unit{i}"] for s_ in shards])
        opt_full = {}
        if "optim" in shards[0]:
            for k, v in shards[0]["optim"][f"unit{i}"].items():
                opt_full[k] = torch.cat([s_["optim"][f"unit{i}"][k] for s_ in shards]) if v.dim() > 0 else v
        for p in u["params"]:
            sl = slice(p["offset"], p["offset"] + p["numel"])
            model[p["name"]] = full[sl].view(p["shape"]).clone()
            if opt_full:
                ostate[pi] = {k: (v[sl].view(p["shape"]).clone() if v.dim() > 0 else v) for k, v in opt_full.items()}
            group_params[gi].append(pi)
            pi += 1
    snap: Dict[str, object] = {"MODEL_STATE": model, "EPOCHS_RUN": 0}
    if ostate:
        groups = []
        for g, params in zip(saved_groups, group_params):
            g = dict(g)
            g["params"] = params
            groups.append(g)
        snap["OPTIMIZER_STATE"] = {"state": ostate, "param_groups": groups}
    if path is not None:
        torch.save(snap, path)
    return snap


def _is_child(parent: tnn.Module, m: tnn.Module) -> bool:
    return any(c is m for c in parent.modules())


def _tensors(out):
    if isinstance(out, torch.Tensor):
        yield out
    elif isinstance(out, (list, tuple)):
        for o in out:
            yield from _tensors(o)
    elif isinstance(out, dict):
        for o in out.values():
            yield from _tensors(o)


FSDP = FullyShardedDataParallel
