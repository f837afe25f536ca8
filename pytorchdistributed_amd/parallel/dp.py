"""Single-process multi-device DataParallel (reference
``nn.DataParallel(model)`` at `01 数据并行/01_multi_gpus_data_parallelism.ipynb` raw lines 117-121,
forward at 139-145: replicate -> scatter -> parallel_apply -> gather).

MI355X version:
* the module is explicitly moved to ``device_ids[0]`` (the reference never moves it);
* replication is a functional call with coalesced per-device parameter copies: the parameters of one
  dtype are concatenated once on ``device_ids[0]`` and each other device receives ONE peer copy over
  xGMI (buffers likewise, without autograd), which it views as its replica's tensors — not one copy per
  tensor (torch's ``Broadcast`` / ``broadcast_coalesced`` idea); autograd's copy- and cat-backward
  reduce-add every replica's gradient into the master parameters on ``device_ids[0]`` (the
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

    # tests set this to copy even to the master's own device (the CPU tier has one device type)
    _force_copy = False

    def _replica_states(self, devs: Sequence[torch.device]) -> List[dict]:
        """Parameter / buffer dicts for functional_call on every device: the master's tensors on
        ``devs[0]``; elsewhere views of one coalesced copy per dtype (parameters through autograd, so
        gradients flow back to the master; buffers without)."""
        states = [dict() for _ in devs]
        named = [(n, p, True) for n, p in self.module.named_parameters()] + \
                [(n, b, False) for n, b in self.module.named_buffers()]
        for n, t, _ in named:
            states[0][n] = t
        targets = [i for i in range(1, len(devs)) if self._force_copy or devs[i] != devs[0]]
        for i in range(1, len(devs)):
            if i not in targets:
                states[i] = dict(states[0])
        if not targets:
            return states
        groups = {}
        for n, t, is_param in named:
            groups.setdefault((t.dtype, t.device, is_param), []).append((n, t))
        for (_dt, _dev, is_param), items in groups.items():
            with torch.set_grad_enabled(is_param and torch.is_grad_enabled()):
                flat = torch.cat([t.reshape(-1) for _, t in items]) if len(items) > 1 else items[0][1].reshape(-1)
                sizes = [t.numel() for _, t in items]
                for i in targets:
                    rep = flat.to(devs[i], non_blocking=True) if devs[i] != flat.device else flat.clone()
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
