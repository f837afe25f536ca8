"""Multi-process pipeline parallelism (reference concept docs
`03 模型并行/03_model_parallel.ipynb` raw lines 637-705: GPipe re-computation, 1F1B, PipeDream flush,
interleaving; reference code: the single-process micro-batch loop at raw lines 538-561).

One process per stage, activations / gradients moved with RCCL point-to-point (``send``/``recv`` over
xGMI).  Schedules:

* ``gpipe`` — all forwards, then all backwards (fill-drain);
* ``1f1b``  — PipeDream-flush: ``S - s - 1`` warm-up forwards, then one-forward-one-backward, then the
  cool-down backwards; peak activation memory is bounded by the stage depth instead of the number of
  micro-batches;
* ``interleaved`` — virtual-pipeline 1F1B: each rank holds ``v`` model chunks (virtual stages
  ``c * S + s``), which divides the fill/drain bubble by ``v``; executed from a tick plan computed
  identically on every rank (:func:`plan_interleaved`) with one batched P2P group per tick.

In the 1F1B steady state a stage's "send activation to s+1" and "receive gradient from s+1" are issued
as ONE batched P2P group (likewise "send gradient to s-1" + "receive next activation from s-1"), so two
neighbours never wait on each other's opposite-direction transfer (the classic blocking-P2P deadlock).
``recompute=True`` keeps only each micro-batch's stage input and re-runs the stage forward in backward
(GPipe re-materialisation, raw lines 637-643).  :func:`pp_dp_groups` builds the PP x DP process groups
(e.g. 4 stages x 2 replicas: PP {0-3},{4-7}; DP {0,4},{1,5},{2,6},{3,7}).  The DP gradient average
runs through the stage's :class:`~.ddp.DistributedDataParallel` over the DP group (``dp_module``):
bucketed, launched during the last micro-batch's backward (interleaved: each chunk's last), overlapped
with it and with the drain (there is no blocking post-flush gradient all-reduce).
"""
from __future__ import annotations

import contextlib
import json
import os
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist
import torch.nn as tnn
from torch.utils.checkpoint import checkpoint

from .. import distributed as pdist
from ..utils import watchdog as _watchdog

_nullctx = contextlib.nullcontext
# PDA_PP_SYNC_P2P=1: every native P2P group is waited on by the compute stream right after it is enqueued
# (round-4 behaviour, for A/B traces: tools/overlap_report.py)
_SYNC_P2P = os.environ.get("PDA_PP_SYNC_P2P") == "1"


# ------------------------------------------------------------------ schedules (pure functions)
def schedule_gpipe(num_stages: int, num_micro: int, stage: int) -> List[Tuple[str, int]]:
    return [("F", i) for i in range(num_micro)] + [("B", i) for i in range(num_micro)]


def schedule_1f1b(num_stages: int, num_micro: int, stage: int) -> List[Tuple[str, int]]:
    warm = min(num_stages - stage - 1, num_micro)
    out = [("F", i) for i in range(warm)]
    steady = num_micro - warm
    for i in range(steady):
        out.append(("F", warm + i))
        out.append(("B", i))
    out += [("B", i) for i in range(steady, num_micro)]
    return out


SCHEDULES = {"gpipe": schedule_gpipe, "1f1b": schedule_1f1b}


def schedule_interleaved(num_stages: int, num_micro: int, stage: int, chunks: int) -> List[Tuple[str, int, int]]:
    """Interleaved 1F1B (virtual pipeline, `NB03` raw lines 699-705): rank ``stage`` holds ``chunks``
    model chunks; chunk ``c`` is virtual stage ``c * num_stages + stage``.  Units are
    ``(kind, chunk, micro_batch)``.  Micro-batches advance in groups of ``num_stages`` through the
    chunks (forward chunk 0 -> v-1, backward v-1 -> 0); each rank runs
    ``2 (S - s - 1) + (v - 1) S`` warm-up forwards, then one-forward-one-backward, then the cool-down
    backwards.  The bubble shrinks by ``v`` versus 1F1B at the cost of ``v`` times more P2P."""
    S, M, v = num_stages, num_micro, chunks
    if M % S:
        raise ValueError(f"interleaved schedule needs num_microbatches ({M}) divisible by stages ({S})")
    total = M * v

    def unit(k, backward):
        c = (k // S) % v
        mb = (k // (S * v)) * S + k % S
        return ("B" if backward else "F", v - 1 - c if backward else c, mb)

    warm = min(2 * (S - stage - 1) + (v - 1) * S, total)
    out = [unit(k, False) for k in range(warm)]
    for j in range(total - warm):
        out.append(unit(warm + j, False))
        out.append(unit(j, True))
    out += [unit(k, True) for k in range(total - warm, total)]
    return out


def plan_interleaved(num_stages: int, num_micro: int, chunks: int):
    """Deterministic tick plan shared by every rank: per tick, the unit each rank runs (or None) and
    the transfers delivered at the end of that tick, as ``(src_rank, dst_rank, kind, vstage, mb)``
    (``kind`` "F": output of virtual stage ``vstage`` to ``vstage + 1``; "B": input gradient of
    ``vstage`` to ``vstage - 1``).  Each tick's transfers are exchanged as ONE batched P2P group on
    both ends, so opposite-direction and wrap-around (last rank -> rank 0) traffic cannot deadlock.
    Raises if the unit lists cannot complete."""
    S, v = num_stages, chunks
    G = S * v
    units = [schedule_interleaved(S, num_micro, s, v) for s in range(S)]
    pos = [0] * S
    avail = [set() for _ in range(S)]  # ("F"|"B", chunk, mb) inputs that arrived at each rank
    fdone = [set() for _ in range(S)]
    ticks = []
    while any(pos[s] < len(units[s]) for s in range(S)):
        run: List[Optional[Tuple[str, int, int]]] = [None] * S
        xfers = []
        for s in range(S):
            if pos[s] >= len(units[s]):
                continue
            kind, c, mb = units[s][pos[s]]
            g = c * S + s
            if kind == "F":
                ready = g == 0 or ("F", c, mb) in avail[s]
            else:
                ready = (c, mb) in fdone[s] and (g == G - 1 or ("B", c, mb) in avail[s])
            if not ready:
                continue
            run[s] = (kind, c, mb)
            pos[s] += 1
            if kind == "F":
                fdone[s].add((c, mb))
                if g + 1 < G:
                    xfers.append((s, (g + 1) % S, "F", g, mb))
            elif g > 0:
                xfers.append((s, (g - 1) % S, "B", g, mb))
        if all(r is None for r in run):
            raise RuntimeError("interleaved schedule cannot make progress")
        for src, dst, kind, g, mb in xfers:
            tgt = g + 1 if kind == "F" else g - 1
            avail[dst].add((kind, tgt // S, mb))
        ticks.append((run, xfers))
    return ticks


def check_schedule(fn, num_stages: int, num_micro: int) -> bool:
    """Simulate every stage's action list with unbounded send buffers; True iff it completes."""
    acts = [list(fn(num_stages, num_micro, s)) for s in range(num_stages)]
    done_f = [set() for _ in range(num_stages)]
    done_b = [set() for _ in range(num_stages)]
    pos = [0] * num_stages
    progress = True
    while progress:
        progress = False
        for s in range(num_stages):
            if pos[s] >= len(acts[s]):
                continue
            kind, mb = acts[s][pos[s]]
            if kind == "F":
                ok = s == 0 or mb in done_f[s - 1]
            else:
                ok = mb in done_f[s] and (s == num_stages - 1 or mb in done_b[s + 1])
            if ok:
                (done_f if kind == "F" else done_b)[s].add(mb)
                pos[s] += 1
                progress = True
    return all(p == len(a) for p, a in zip(pos, acts))


# ------------------------------------------------------------------ process groups
def pp_dp_groups(pp: int, dp: int):
    """Returns (pp_group, dp_group, stage, dp_rank, pp_ranks) for this rank; rank = dp_rank * pp + stage."""
    rank, world = pdist.get_rank(), pdist.get_world_size()
    assert world == pp * dp, f"world {world} != pp {pp} x dp {dp}"
    pp_group = dp_group = None
    my_pp_ranks = None
    for d in range(dp):
        ranks = [d * pp + s for s in range(pp)]
        g = dist.new_group(ranks)
        if rank in ranks:
            pp_group, my_pp_ranks = g, ranks
    for s in range(pp):
        ranks = [d * pp + s for d in range(dp)]
        g = dist.new_group(ranks)
        if rank in ranks:
            dp_group = g
    return pp_group, dp_group, rank % pp, rank // pp, my_pp_ranks


# ------------------------------------------------------------------ the pipeline engine
class _P2PWork:
    """Completion of a P2P group that received buffers: ``wait()`` orders the current stream after it
    (native: a stream-event wait; c10d: the works' own wait)."""

    def __init__(self, native=None, c10d=None, desc: str = "pp p2p"):
        self.native, self.c10d, self.desc = native, c10d, desc

    def wait(self):
        if self.native is not None:
            self.native.wait()  # the native group's watchdog ticket was armed at enqueue
        if self.c10d:
            # c10d (gloo: the wait blocks the host) under a deadline of its own
            with _watchdog.watch(f"{self.desc} (c10d wait)"):
                for w in self.c10d:
                    w.wait()
        self.native, self.c10d = None, None


class Pipeline:
    """Drive one pipeline stage.

    ``stage_module``: this rank's stage; ``ranks``: global ranks of the pipeline in stage order;
    ``loss_fn(output, target)`` is applied on the last stage per micro-batch.
    """

    def __init__(self, stage_module, ranks: Sequence[int], num_microbatches: int,
                 schedule: str = "1f1b", loss_fn: Optional[Callable] = None, recompute: bool = False,
                 group=None, device=None, dp_module=None):
        """``dp_module``: the stage wrapped in :class:`~.ddp.DistributedDataParallel` over its DP group
        (PP x DP).  Micro-batches 0..M-2 run backward under ``no_sync`` (local accumulation); the last
        micro-batch's backward launches the gradient buckets as they become ready, so the DP all-reduce
        overlaps that backward and the pipeline drain (reference DDP semantics, `ddp_gpus.py:35,41`)."""
        # schedule="interleaved": ``stage_module`` is the list of this rank's model chunks (chunk c =
        # virtual stage c * len(ranks) + stage)
        self.chunks = list(stage_module) if isinstance(stage_module, (list, tuple, tnn.ModuleList)) else None
        if (schedule == "interleaved") != (self.chunks is not None):
            raise ValueError("schedule='interleaved' takes a list of model chunks (and only it does)")
        self.module = tnn.ModuleList(self.chunks) if self.chunks is not None else stage_module
        self.ranks = list(ranks)
        self.S = len(self.ranks)
        self.rank = pdist.get_rank()
        self.stage = self.ranks.index(self.rank)
        self.M = num_microbatches
        self.schedule_name = schedule
        self.loss_fn = loss_fn
        self.recompute = recompute
        self.group = group
        self.device = device or next(self.module.parameters()).device
        self.prev = self.ranks[self.stage - 1] if self.stage > 0 else None
        self.next = self.ranks[self.stage + 1] if self.stage < self.S - 1 else None
        self._fwd_meta = None  # (shape, dtype) received from prev
        self._bwd_meta = None  # (shape, dtype) of our output (grad received from next)
        self.dp_module = dp_module
        if dp_module is not None and schedule == "interleaved":
            # the chunks' DP reduction: each chunk's parameters are marked ready in the backward of its
            # LAST micro-batch, i.e. over v separate backward passes; the DDP wrapper keeps its bucket
            # state across them and finalizes once every bucket has been launched
            dp_module.set_multi_pass(True)
        # activations / gradients between stages on the native RCCL communicator of the PP group
        # (comm.py: one fused send/recv group per tick / transfer pair, ordered on its own stream; the
        # consumer stream waits on an event, no host blocking); c10d batch_isend_irecv on gloo /
        # PDA_COMM=c10d.  PDA_PP_FORCE_COMM=1 at one stage: the interleaved schedule's chunk-to-chunk
        # hand-offs go through RCCL send/recv to this same rank (a one-GPU box runs the P2P path).
        self._ncomm = None
        self._send_works: List = []
        self._tickets = 0  # watchdog tickets armed for native P2P groups (tests / stats)
        force = os.environ.get("PDA_PP_FORCE_COMM") == "1"
        if (self.device.type == "cuda" and dist.is_initialized() and dist.get_backend(group) == "nccl"
                and (self.S > 1 or force)):
            from .. import comm as _comm

            if _comm.enabled():
                self._ncomm = _comm.try_for_group(group, self.device)

    @property
    def is_first(self):
        return self.stage == 0

    @property
    def is_last(self):
        return self.stage == self.S - 1

    # ---------------- shape handshake (once) and p2p helpers
    # Transfers never make the compute stream wait for a SEND: a send is enqueued on the P2P stream after
    # the producing kernels, its tensor is held for the allocator by record_stream on that stream
    # (comm.py _hold), and the next micro-batch's forward runs while it is in flight (the reference's
    # point, "B can run concurrently with A", NB03 raw lines 551-556).  The compute stream waits only
    # before it CONSUMES a received buffer (:class:`_P2PWork`).  Every native P2P group is armed on the
    # collective watchdog and retires on the GPU's own completion.
    def _peer(self, r: int) -> int:
        return dist.get_group_rank(self.group, r) if self.group is not None else r

    def _native_group(self, sends, recvs, what: str):
        w = self._ncomm.send_recv([(t.contiguous(), self._peer(r)) for t, r in sends],
                                  [(t, self._peer(r)) for t, r in recvs])
        nbytes = sum(t.numel() * t.element_size() for t, _ in list(sends) + list(recvs))
        _watchdog.track(f"pp {what} stage {self.stage} ({len(sends)} send / {len(recvs)} recv, "
                        f"{nbytes / 2**20:.2f} MB)", self._ncomm.stream)
        self._tickets += 1
        return w

    def _send_meta(self, t: torch.Tensor, dst: int):
        meta = self._meta_tensor(t)
        if self._ncomm is not None:
            self._native_group([(meta, dst)], [], "shape send")
        else:
            dist.send(meta, dst, group=self.group)

    def _recv_meta(self, src: int):
        meta = torch.zeros(10, dtype=torch.long, device=self.device)
        if self._ncomm is not None:
            self._native_group([], [(meta, src)], "shape recv").synchronize()  # host needs the shape
        else:
            with _watchdog.watch(f"pp shape recv stage {self.stage} from {src}"):
                dist.recv(meta, src, group=self.group)
        nd = int(meta[0])
        dtype = [torch.float32, torch.bfloat16, torch.float16][int(meta[1])]
        return tuple(int(v) for v in meta[2: 2 + nd]), dtype

    def _p2p_group(self, sends: List[Tuple[torch.Tensor, int]], recvs: List[Tuple[torch.Tensor, int]],
                   what: str = "p2p") -> Optional["_P2PWork"]:
        """One fused group of transfers (global ranks as peers): native RCCL send/recv on the P2P stream,
        or c10d batch_isend_irecv.  Returns the work to wait on before consuming the received buffers
        (None when there are none); send-only groups are never waited on by the compute stream (c10d
        send works are kept and retired by :meth:`_drain_sends` at the end of the step)."""
        if not sends and not recvs:
            return None
        if self._ncomm is not None:
            w = self._native_group(sends, recvs, what)
            if _SYNC_P2P:  # A/B knob: the round-4 behaviour (the compute stream waits on every group at once)
                w.wait()
                return None
            return _P2PWork(native=w) if recvs else None
        ops = [dist.P2POp(dist.isend, t.contiguous(), r, group=self.group) for t, r in sends]
        ops += [dist.P2POp(dist.irecv, t, r, group=self.group) for t, r in recvs]
        works = dist.batch_isend_irecv(ops)
        if not recvs:
            self._send_works.extend(works)
            return None
        return _P2PWork(c10d=works, desc=f"pp {what} stage {self.stage}")

    def _p2p(self, send: Optional[Tuple[torch.Tensor, int]] = None, recv: Optional[Tuple[torch.Tensor, int]] = None):
        """Blocking-for-the-consumer transfer pair: the current stream waits for the receive (if any)."""
        w = self._p2p_group([send] if send is not None else [], [recv] if recv is not None else [],
                            "send+recv" if send is not None and recv is not None else ("recv" if recv is not None else "send"))
        if w is not None:
            w.wait()

    def _drain_sends(self):
        if self._send_works:
            with _watchdog.watch(f"pp sends stage {self.stage} (c10d wait, {len(self._send_works)} ops)"):
                for w in self._send_works:
                    w.wait()
        self._send_works = []

    def _empty(self, meta):
        shape, dtype = meta
        return torch.empty(shape, dtype=dtype, device=self.device)

    # ---------------- compute
    def _forward(self, x: torch.Tensor):
        if self.recompute and torch.is_grad_enabled():
            return checkpoint(self.module, x, use_reentrant=False)
        return self.module(x)

    def _step_interleaved(self, inputs, targets):
        S, M, v = self.S, self.M, len(self.chunks)
        G = S * v
        first = self.is_first  # rank 0 holds virtual stage 0 (chunk 0)
        last = self.is_last    # rank S-1 holds virtual stage G-1 (chunk v-1)
        in_mb = list(inputs.chunk(M)) if (first and inputs is not None) else [None] * M
        tg_mb = list(targets.chunk(M)) if (last and targets is not None) else [None] * M
        if not hasattr(self, "_plan") or self._plan_key != (S, M, v):
            self._plan, self._plan_key = plan_interleaved(S, M, v), (S, M, v)
            self._vmeta = {}  # virtual stage g -> (shape, dtype) of its output (known to g and g+1)
        acts_in, acts_out, inbox = {}, {}, {}
        losses = []

        def take(key):
            # a received buffer is waited on only here, when it is consumed: the hand-off of tick t
            # overlaps whatever this rank runs before it needs the data
            buf, work = inbox.pop(key)
            if work is not None:
                work.wait()
            return buf

        def fwd(c, x):
            m = self.chunks[c]
            if self.recompute and torch.is_grad_enabled():
                return checkpoint(m, x, use_reentrant=False)
            return m(x)

        for run, xfers in self._plan:
            out_t = {}
            if run[self.stage] is not None:
                kind, c, mb = run[self.stage]
                g = c * S + self.stage
                if kind == "F":
                    x = in_mb[mb].to(self.device) if g == 0 else take(("F", c, mb))
                    if g > 0:
                        x.requires_grad_()
                    acts_in[(c, mb)] = x
                    y = fwd(c, x)
                    if g == G - 1:
                        loss = self.loss_fn(y, tg_mb[mb].to(self.device)) / M if self.loss_fn else y.float().mean() / M
                        losses.append(loss.detach())
                        acts_out[(c, mb)] = loss
                    else:
                        acts_out[(c, mb)] = y
                        self._vmeta[g] = (tuple(y.shape), y.dtype)
                        out_t[("F", g, mb)] = y.detach()
                else:
                    out = acts_out.pop((c, mb))
                    # DP: a chunk's gradients are complete after the backward of its last micro-batch
                    ctx = (self.dp_module.no_sync() if (self.dp_module is not None and mb != M - 1)
                           else _nullctx())
                    with ctx:
                        if g == G - 1:
                            out.backward()
                        else:
                            torch.autograd.backward(out, take(("B", c, mb)))
                    x = acts_in.pop((c, mb))
                    if g > 0:
                        out_t[("B", g, mb)] = x.grad
            # this tick's transfers: first-time forward shapes, then one batched group of tensors
            mine = [t for t in xfers if self.stage in (t[0], t[1])]
            meta_ops, meta_in, ops, local = [], [], [], []
            for src, dst, kind, g, mb in mine:
                tgt = g + 1 if kind == "F" else g - 1
                key = (kind, tgt // S, mb)
                if src == dst:  # S == 1: hand over within the rank (through RCCL under PDA_PP_FORCE_COMM)
                    t = out_t[(kind, g, mb)]
                    w = None
                    if self._ncomm is not None:
                        buf = torch.empty_like(t)
                        w = self._p2p_group([(t, self.rank)], [(buf, self.rank)], "loopback")
                        t = buf
                    local.append((key, t, w))
                    continue
                if src == self.stage:
                    t = out_t[(kind, g, mb)].contiguous()
                    if kind == "F" and ("sent", g) not in self._vmeta:
                        self._vmeta[("sent", g)] = True
                        meta_ops.append((self._meta_tensor(t), self.ranks[dst]))
                    ops.append((t, self.ranks[dst]))
                else:
                    if kind == "F" and g not in self._vmeta:
                        mt = torch.zeros(10, dtype=torch.long, device=self.device)
                        meta_ops.append((None, -1))  # marks that this tick has a shape exchange
                        meta_in.append((g, mt, self.ranks[src]))
                    # shape of what arrives: virtual stage g's output (F) or input (B, = output of tgt)
                    ops.append((key, src, g if kind == "F" else tgt))
            if meta_ops:
                if self._ncomm is not None:  # first-use shapes on the same native communicator
                    w = self._native_group([(t, r) for t, r in meta_ops if t is not None and r >= 0],
                                           [(mt, r) for _g, mt, r in meta_in], "shapes")
                    if meta_in:
                        w.synchronize()  # the host allocates the receive buffers from them
                else:
                    ops_ = [dist.P2POp(dist.isend, t, r, group=self.group) for t, r in meta_ops if t is not None]
                    ops_ += [dist.P2POp(dist.irecv, mt, r, group=self.group) for _g, mt, r in meta_in]
                    with _watchdog.watch(f"pp shapes stage {self.stage} (c10d wait)"):
                        for r in dist.batch_isend_irecv(ops_):
                            r.wait()
                for g, mt, _r in meta_in:
                    nd = int(mt[0])
                    self._vmeta[g] = (tuple(int(q) for q in mt[2: 2 + nd]),
                                      [torch.float32, torch.bfloat16, torch.float16][int(mt[1])])
            sends, recvs, recvd = [], [], []
            for op in ops:
                if len(op) == 3 and isinstance(op[0], tuple):
                    key, src, mg = op
                    buf = self._empty(self._vmeta[mg])
                    recvs.append((buf, self.ranks[src]))
                    recvd.append((key, buf))
                else:
                    sends.append(op)
            w = self._p2p_group(sends, recvs, "tick")
            for key, buf in recvd:
                inbox[key] = (buf, w)
            for key, buf, lw in local:
                inbox[key] = (buf, lw)
        self._drain_sends()
        if self.dp_module is not None:
            self.dp_module.finish_multi_pass()
        if last:
            return torch.stack(losses).sum()
        return None

    def _meta_tensor(self, t: torch.Tensor) -> torch.Tensor:
        meta = torch.zeros(10, dtype=torch.long, device=self.device)
        meta[0] = t.dim()
        meta[1] = {torch.float32: 0, torch.bfloat16: 1, torch.float16: 2}[t.dtype]
        meta[2: 2 + t.dim()] = torch.tensor(t.shape, dtype=torch.long)
        return meta

    def step(self, inputs: Optional[torch.Tensor] = None, targets: Optional[torch.Tensor] = None):
        """Run one optimisation step's forward+backward over ``num_microbatches``; returns the mean loss
        on the last stage (None elsewhere).  Gradients accumulate into the stage parameters."""
        if self.schedule_name == "interleaved":
            return self._step_interleaved(inputs, targets)
        M = self.M
        in_mb = list(inputs.chunk(M)) if (self.is_first and inputs is not None) else [None] * M
        tg_mb = list(targets.chunk(M)) if (self.is_last and targets is not None) else [None] * M
        acts_in: List[Optional[torch.Tensor]] = [None] * M
        acts_out: List[Optional[torch.Tensor]] = [None] * M
        losses = []

        # first-step handshakes so receivers can allocate buffers
        def ensure_fwd_meta():
            if self._fwd_meta is None and not self.is_first:
                self._fwd_meta = self._recv_meta(self.prev)

        def recv_forward(i):
            if self.is_first:
                x = in_mb[i].to(self.device)
                return x
            ensure_fwd_meta()
            buf = self._empty(self._fwd_meta)
            self._p2p(recv=(buf, self.prev))
            return buf.requires_grad_()

        def run_forward(i, x):
            if not self.is_first:
                x.requires_grad_()
            acts_in[i] = x
            y = self._forward(x)
            if self.is_last:
                loss = self.loss_fn(y, tg_mb[i].to(self.device)) / M if self.loss_fn else y.float().mean() / M
                losses.append(loss.detach())
                acts_out[i] = loss
                return None
            acts_out[i] = y
            if self._bwd_meta is None:
                self._bwd_meta = (tuple(y.shape), y.dtype)
                self._send_meta(y, self.next)
            return y

        def run_backward(i, dy):
            out = acts_out[i]
            # DP gradient sync only in the last micro-batch's backward (both schedules run it last)
            ctx = self.dp_module.no_sync() if (self.dp_module is not None and i != M - 1) else _nullctx()
            with ctx:
                if self.is_last:
                    out.backward()
                else:
                    torch.autograd.backward(out, dy)
            dx = acts_in[i].grad if not self.is_first else None
            acts_in[i] = acts_out[i] = None
            return dx

        sched = self.schedule_name
        if sched == "gpipe":
            for i in range(M):
                y = run_forward(i, recv_forward(i))
                if y is not None:
                    self._p2p(send=(y.detach(), self.next))
            for i in range(M):
                dy = None
                if not self.is_last:
                    dy = self._empty(self._bwd_meta)
                    self._p2p(recv=(dy, self.next))
                dx = run_backward(i, dy)
                if not self.is_first:
                    self._p2p(send=(dx, self.prev))
        elif sched == "1f1b":
            warm = min(self.S - self.stage - 1, M)
            steady = M - warm
            for i in range(warm):
                y = run_forward(i, recv_forward(i))
                if y is not None:
                    self._p2p(send=(y.detach(), self.next))
            x = recv_forward(warm) if steady > 0 else None
            for j in range(steady):
                fi = warm + j
                y = run_forward(fi, x)
                dy = None
                if not self.is_last:
                    dy = self._empty(self._bwd_meta)
                    self._p2p(send=(y.detach(), self.next), recv=(dy, self.next))  # send fwd + recv bwd
                dx = run_backward(j, dy)
                if j == steady - 1:
                    if not self.is_first:
                        self._p2p(send=(dx, self.prev))
                else:
                    if self.is_first:
                        x = recv_forward(fi + 1)
                    else:
                        ensure_fwd_meta()
                        x = self._empty(self._fwd_meta)
                        self._p2p(send=(dx, self.prev), recv=(x, self.prev))  # send bwd + recv fwd
            for i in range(steady, M):
                dy = None
                if not self.is_last:
                    dy = self._empty(self._bwd_meta)
                    self._p2p(recv=(dy, self.next))
                dx = run_backward(i, dy)
                if not self.is_first:
                    self._p2p(send=(dx, self.prev))
        else:
            raise ValueError(f"unknown schedule {sched!r}")
        self._drain_sends()
        if self.is_last:
            return torch.stack(losses).sum()
        return None


# ------------------------------------------------------------------ checkpoints (PP layout)
def _atomic_save(obj, path: str):
    tmp = path + ".tmp"
    torch.save(obj, tmp)
    os.replace(tmp, path)


def save_pipeline_checkpoint(directory: str, pipe: "Pipeline", optimizer=None, step: int = 0,
                             partition: Optional[List[Tuple[int, int]]] = None, dp_rank: int = 0,
                             extra: Optional[dict] = None):
    """Per-stage files + the stage-partition map.

    ``stage_{s:03d}.pt`` = ``{"MODEL_STATE", "OPTIMIZER_STATE", "STEP", "STAGE"}`` of pipeline stage s
    (written by the stage's DP replica 0 only — replicas are identical after the DP gradient sync);
    ``pipeline.json`` (stage 0) = stages, schedule, micro-batches, model chunks per rank and the
    [start, end) layer range of every (virtual) stage, which :func:`consolidate_pipeline` uses to
    renumber stage-local layers into one full-model state dict.  Collective over nothing: each stage
    writes its own file; call a barrier afterwards if other ranks read it right away.
    """
    if dp_rank != 0:
        return
    os.makedirs(directory, exist_ok=True)
    snap = {"MODEL_STATE": pipe.module.state_dict(), "STEP": int(step), "STAGE": pipe.stage}
    if optimizer is not None:
        snap["OPTIMIZER_STATE"] = optimizer.state_dict()
    if extra:
        snap.update(extra)
    _atomic_save(snap, os.path.join(directory, f"stage_{pipe.stage:03d}.pt"))
    if pipe.stage == 0:
        meta = {"num_stages": pipe.S, "schedule": pipe.schedule_name, "num_microbatches": pipe.M,
                "chunks": len(pipe.chunks) if pipe.chunks is not None else 1,
                "partition": [list(r) for r in partition] if partition is not None else None}
        tmp = os.path.join(directory, "pipeline.json.tmp")
        with open(tmp, "w") as f:
            json.dump(meta, f, indent=1)
        os.replace(tmp, os.path.join(directory, "pipeline.json"))


def load_pipeline_checkpoint(directory: str, pipe: "Pipeline", optimizer=None, map_location="cpu") -> int:
    """Restore this rank's stage (every DP replica of the stage reads the same file); returns the step."""
    meta = json.load(open(os.path.join(directory, "pipeline.json")))
    chunks = len(pipe.chunks) if pipe.chunks is not None else 1
    if meta["num_stages"] != pipe.S or meta["chunks"] != chunks:
        raise ValueError(f"checkpoint has {meta['num_stages']} stages x {meta['chunks']} chunks, "
                         f"pipeline has {pipe.S} x {chunks}")
    snap = torch.load(os.path.join(directory, f"stage_{pipe.stage:03d}.pt"), map_location=map_location,
                      weights_only=True)
    pipe.module.load_state_dict(snap["MODEL_STATE"])
    if optimizer is not None and "OPTIMIZER_STATE" in snap:
        optimizer.load_state_dict(snap["OPTIMIZER_STATE"])
        sync = getattr(optimizer, "sync_from_state", None)
        if sync is not None:
            sync()
    return int(snap.get("STEP", 0))


def consolidate_pipeline(directory: str, layer_prefix: str = "h") -> Dict[str, torch.Tensor]:
    """Offline: merge ``stage_*.pt`` into one full-model state dict.  Keys ``{layer_prefix}.{i}.*`` of
    (virtual) stage v are renumbered to ``{layer_prefix}.{start_v + i}.*`` using the partition map; for
    interleaved checkpoints the chunk index prefix (``c.``) selects virtual stage ``c * stages + s``.
    Other keys (embeddings, final norm, head) pass through unchanged."""
    meta = json.load(open(os.path.join(directory, "pipeline.json")))
    S, V, part = meta["num_stages"], meta["chunks"], meta["partition"]
    out: Dict[str, torch.Tensor] = {}
    for s in range(S):
        sd = torch.load(os.path.join(directory, f"stage_{s:03d}.pt"), map_location="cpu",
                        weights_only=True)["MODEL_STATE"]
        for k, v in sd.items():
            c, key = 0, k
            if V > 1:
                c_str, key = k.split(".", 1)
                c = int(c_str)
            vs = c * S + s
            head, _, rest = key.partition(".")
            if part is not None and head == layer_prefix and rest:
                idx, _, tail = rest.partition(".")
                key = f"{layer_prefix}.{part[vs][0] + int(idx)}.{tail}" if tail else f"{layer_prefix}.{part[vs][0] + int(idx)}"
            if key in out:
                raise ValueError(f"duplicate key {key!r} while consolidating stage {s}")
            out[key] = v
    return out


def partition_layers(num_layers: int, num_stages: int) -> List[Tuple[int, int]]:
    """Contiguous [start, end) layer ranges, balanced (earlier stages get the remainder)."""
    base, rem = divmod(num_layers, num_stages)
    out, s = [], 0
    for i in range(num_stages):
        n = base + (1 if i < rem else 0)
        out.append((s, s + n))
        s += n
    return out
