"""Single-process multi-device DataParallel (reference
``nn.DataParallel(model)`` at `01 数据并行/01_multi_gpus_data_parallelism.ipynb` raw lines 117-121,
forward at 139-145: replicate -> scatter -> parallel_apply -> gather).

MI355X version:
* the module is explicitly moved to ``device_ids[0]`` (the reference never moves it);
* the master's parameters (and buffers) live as views of ONE flat buffer per dtype on ``device_ids[0]``
  (re-homed once at construction), and every other device keeps a persistent flat replica of it: a
  forward refreshes each replica with ONE peer copy per dtype over xGMI (``copy_`` into the existing
  buffer: no per-forward concatenation, no per-forward allocation) and the replica's module runs on
  views of it through a functional call — torch's ``Broadcast`` / ``broadcast_coalesced`` idea without
  the flatten.  Backward: each replica's flat gradient comes back to ``device_ids[0]`` as one copy and
  autograd sums them with the master's own gradient before one split into per-parameter views (the
  reference's PS-style "reduce grads to master");
* the per-device forwards run in one Python thread per device, each on its own device/stream;
* outputs are gathered (concatenated) on ``output_device``.
``device_ids`` may also list CPU devices (used by the CPU tests to exercise the same code path).
"""
from __future__ import annotations

import threading
from typing import List, Optional, Sequence

import torch
import torch.nn as tnn
from torch.func import functional_call


def _as_devices(ids) -> List[torch.device]:
    out = []
    for d in ids:
        if isinstance(d, torch.device):
            out.append(d)
        elif isinstance(d, int):
            out.append(torch.device("cuda", d))
        else:
            out.append(torch.device(d))
    return out


def scatter(x, devices: Sequence[torch.device], dim: int = 0):
    if isinstance(x, torch.Tensor):
        chunks = x.chunk(len(devices), dim)
        return [c.to(d, non_blocking=True) for c, d in zip(chunks, devices)]
    if isinstance(x, (list, tuple)):
        per = [scatter(v, devices, dim) for v in x]
        return [type(x)(p[i] for p in per) for i in range(len(per[0]) if per else len(devices))]
    return [x for _ in devices]


def gather(outs, device: torch.device, dim: int = 0):
    first = outs[0]
    if isinstance(first, torch.Tensor):
        return torch.cat([o.to(device, non_blocking=True) for o in outs], dim)
    if isinstance(first, (list, tuple)):
        return type(first)(gather([o[i] for o in outs], device, dim) for i in range(len(first)))
    if isinstance(first, dict):
        return {k: gather([o[k] for o in outs], device, dim) for k in first}
    return first


class _FlatOf(torch.autograd.Function):
    """The master's flat parameter buffer as one differentiable tensor of its parameters (which are views
    of it): forward returns the buffer itself (no copy); backward splits the summed flat gradient into
    per-parameter views."""

    @staticmethod
    def forward(ctx, flat, *params):
        ctx.shapes = [(off, p.shape) for off, p in zip(_offsets(params), params)]
        return flat.view(-1)

    @staticmethod
    def backward(ctx, g):
        return (None,) + tuple(g[off: off + sh.numel()].view(sh) for off, sh in ctx.shapes)


def _offsets(ts):
    out, o = [], 0
    for t in ts:
        out.append(o)
        o += t.numel()
    return out


class _CopyInto(torch.autograd.Function):
    """``buf.copy_(src)`` (one peer copy into a persistent replica buffer); backward: the gradient goes back
    to ``src``'s device as one copy."""

    @staticmethod
    def forward(ctx, src, buf):
        buf.copy_(src, non_blocking=True)
        ctx.src_device = src.device
        return buf.view_as(buf)

    @staticmethod
    def backward(ctx, g):
        return g.to(ctx.src_device, non_blocking=True), None


class DataParallel(tnn.Module):
    def __init__(self, module: tnn.Module, device_ids: Optional[Sequence] = None, output_device=None, dim: int = 0):
        super().__init__()
        if device_ids is None:
            n = torch.cuda.device_count()
            device_ids = list(range(n)) if n > 0 else ["cpu"]
        self.devices = _as_devices(device_ids)
        self.device_ids = list(device_ids)
        self.output_device = _as_devices([output_device])[0] if output_device is not None else self.devices[0]
        self.dim = dim
        self.module = module.to(self.devices[0])
        self._groups: List[tuple] = []   # (flat, [(name, param)], is_param)
        self._replicas: dict = {}        # (group index, device index) -> persistent replica buffer
        self.replica_copies = 0          # peer copies issued by forwards (one per dtype group and device)
        if len(self.devices) > 1:
            self._flatten()

    # tests set this to copy even to the master's own device (the CPU tier has one device type)
    _force_copy = False

    @torch.no_grad()
    def _flatten(self):
        """Re-home the master's parameters and buffers as views of one flat buffer per (dtype, kind)."""
        self._groups, self._replicas = [], {}
        groups = {}
        for n, p in self.module.named_parameters():
            groups.setdefault((p.dtype, True), []).append((n, p))
        owners = {}
        for mod_name, mod in self.module.named_modules():
            for bn, b in mod._buffers.items():
                if b is not None:
                    owners.setdefault((b.dtype, False), []).append((f"{mod_name}.{bn}" if mod_name else bn, mod, bn, b))
        for (dt, _), items in groups.items():
            flat = torch.empty(sum(p.numel() for _, p in items), dtype=dt, device=self.devices[0])
            o = 0
            for _, p in items:
                flat[o: o + p.numel()].copy_(p.detach().reshape(-1))
                p.data = flat[o: o + p.numel()].view_as(p)
                o += p.numel()
            self._groups.append((flat, items, True))
        for (dt, _), items in owners.items():
            flat = torch.empty(sum(b.numel() for *_, b in items), dtype=dt, device=self.devices[0])
            o = 0
            named = []
            for name, mod, bn, b in items:
                view = flat[o: o + b.numel()].view_as(b)
                view.copy_(b)
                mod._buffers[bn] = view
                named.append((name, view))
                o += b.numel()
            self._groups.append((flat, named, False))

    def _stale(self) -> bool:
        """A parameter / buffer replaced since the flattening (not a view of its group's buffer any more)."""
        for flat, items, _ in self._groups:
            lo = flat.data_ptr()
            hi = lo + flat.numel() * flat.element_size()
            for _, t in items:
                if not (lo <= t.data_ptr() < hi):
                    return True
        named = dict(self.module.named_parameters())
        return any(is_p and any(named.get(n) is not t for n, t in items) for _, items, is_p in self._groups)

    def _replica_states(self, devs: Sequence[torch.device]) -> List[dict]:
        """Parameter / buffer dicts for functional_call on every device: the master's tensors on
        ``devs[0]``; elsewhere views of the device's persistent flat replica, refreshed by one copy per
        group (parameters through autograd, so gradients flow back to the master; buffers without)."""
        if not self._groups or self._stale():
            self._flatten()
        states = [dict() for _ in devs]
        for _, items, _ in self._groups:
            for n, t in items:
                states[0][n] = t
        targets = [i for i in range(1, len(devs)) if self._force_copy or devs[i] != devs[0]]
        for i in range(1, len(devs)):
            if i not in targets:
                states[i] = dict(states[0])
        if not targets:
            return states
        grad = torch.is_grad_enabled()
        for gi, (flat, items, is_param) in enumerate(self._groups):
            src = _FlatOf.apply(flat, *[t for _, t in items]) if (is_param and grad) else flat
            sizes = [t.numel() for _, t in items]
            for i in targets:
                key = (gi, i)
                buf = self._replicas.get(key)
                if buf is None or buf.device != devs[i] or buf.numel() != flat.numel():
                    buf = self._replicas[key] = torch.empty(flat.numel(), dtype=flat.dtype, device=devs[i])
                if is_param and grad:
                    rep = _CopyInto.apply(src, buf)
                else:
                    with torch.no_grad():
                        buf.copy_(src, non_blocking=True)
                    rep = buf
                self.replica_copies += 1
                for (n, t), piece in zip(items, rep.split(sizes)):
                    states[i][n] = piece.view_as(t)
        return states

    def forward(self, *inputs, **kwargs):
        if len(self.devices) == 1:
            ins = [i.to(self.devices[0]) if isinstance(i, torch.Tensor) else i for i in inputs]
            return self.module(*ins, **kwargs)
        n = min(len(self.devices), inputs[0].shape[self.dim] if isinstance(inputs[0], torch.Tensor) else len(self.devices))
        devs = self.devices[:n]
        scattered = scatter(list(inputs), devs, self.dim)
        states = self._replica_states(devs)
        results: List = [None] * n
        errors: List = [None] * n
        grad_enabled = torch.is_grad_enabled()

        def work(i):
            try:
                torch.set_grad_enabled(grad_enabled)
                dev = devs[i]
                if dev.type == "cuda":
                    with torch.cuda.device(dev), torch.cuda.stream(torch.cuda.current_stream(dev)):
                        results[i] = functional_call(self.module, states[i], tuple(scattered[i]), kwargs)
                else:
                    results[i] = functional_call(self.module, states[i], tuple(scattered[i]), kwargs)
            except BaseException as e:  # noqa: BLE001
                errors[i] = e

        threads = [threading.Thread(target=work, args=(i,)) for i in range(1, n)]
        for t in threads:
            t.start()
        work(0)
        for t in threads:
            t.join()
        for e in errors:
            if e is not None:
                raise e
        return gather(results, self.output_device, self.dim)
