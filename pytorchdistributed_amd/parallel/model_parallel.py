"""Single-process layer-split model parallelism and micro-batched pipelining over several devices
(reference `03 模型并行/03_model_parallel.ipynb`: ``ModelParallelResNet50``
raw lines 325-349, ``PipelineParallelResNet50`` raw lines 538-561, ``device_map="auto"`` raw line 86).

* :class:`ModelParallel` / :func:`split_model` — stages on devices, activations moved at boundaries.
* :class:`ModelParallelResNet50` — the reference's exact split: stem+layer1+layer2 on device 0,
  layer3+layer4+avgpool+fc on device 1.
* :class:`PipelineParallelResNet50` — the reference's ``split_size`` micro-batch pipeline, but with
  explicit concurrency instead of "the CPU happens to run ahead": every stage runs on its own device
  stream, each boundary copy is ordered by events, and each micro-batch's logits are written into its
  slice of one preallocated output tensor as soon as that micro-batch finishes (an autograd-recorded
  slice write on the stage's stream; no ``torch.cat`` of the outputs at the end).
* :func:`auto_place` — budget-driven placement of a sequential model's children across devices
  (GPU > CPU), the analogue of HF ``device_map="auto"``.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence

import torch
import torch.nn as tnn

from ..models.resnet import ResNet, _Head


def _dev(d) -> torch.device:
    if isinstance(d, torch.device):
        return d
    return torch.device("cuda", d) if isinstance(d, int) else torch.device(d)


class ModelParallel(tnn.Module):
    """Run ``stages[i]`` on ``devices[i]``; the input goes to ``devices[0]``."""

    def __init__(self, stages: Sequence[tnn.Module], devices: Sequence):
        super().__init__()
        assert len(stages) == len(devices)
        self.devices = [_dev(d) for d in devices]
        self.stages = tnn.ModuleList([s.to(d) for s, d in zip(stages, self.devices)])

    def forward(self, x):
        for s, d in zip(self.stages, self.devices):
            x = s(x.to(d, non_blocking=True))
        return x


def split_model(model: tnn.Module, boundaries: Sequence[int], devices: Sequence) -> ModelParallel:
    """Split ``model``'s ordered stage list (``model.stage_modules()`` or its children) at ``boundaries``."""
    parts = list(model.stage_modules()) if hasattr(model, "stage_modules") else list(model.children())
    cuts = [0] + list(boundaries) + [len(parts)]
    stages = [tnn.Sequential(*parts[cuts[i]:cuts[i + 1]]) for i in range(len(cuts) - 1)]
    return ModelParallel(stages, devices)


class ModelParallelResNet50(tnn.Module):
    """Reference split (`NB03:325-349`): seq1 = stem, layer1, layer2 on dev0; seq2 = layer3, layer4,
    avgpool (+fc) on dev1."""

    def __init__(self, model: Optional[ResNet] = None, devices: Sequence = (0, 1), num_classes: int = 1000,
                 dtype=None):
        super().__init__()
        model = model if model is not None else ResNet(num_classes=num_classes, dtype=dtype)
        self.dev0, self.dev1 = _dev(devices[0]), _dev(devices[1])
        self.seq1 = tnn.Sequential(model.stem, model.layer1, model.layer2).to(self.dev0)
        self.seq2 = tnn.Sequential(model.layer3, model.layer4).to(self.dev1)
        self.head = _Head(model.fc).to(self.dev1)

    def forward(self, x):
        x = self.seq2(self.seq1(x.to(self.dev0)).to(self.dev1))
        return self.head(x)


class PipelineParallelResNet50(ModelParallelResNet50):
    """Micro-batched pipeline of the reference (`NB03:538-561`, default ``split_size=20``)."""

    def __init__(self, *args, split_size: int = 20, **kwargs):
        super().__init__(*args, **kwargs)
        self.split_size = split_size
        self._streams = {}

    def _stream(self, stage, dev):
        """One stream per stage (also when both stages share a device, so their micro-batches overlap)."""
        if dev.type != "cuda":
            return None
        if stage not in self._streams:
            self._streams[stage] = torch.cuda.Stream(dev)
        return self._streams[stage]

    def forward(self, x):
        splits = x.split(self.split_size, dim=0)
        s0, s1 = self._stream(0, self.dev0), self._stream(1, self.dev1)
        capturing = s0 is not None and torch.cuda.is_current_stream_capturing()
        if capturing and self.dev0 != self.dev1:
            raise RuntimeError("HIP-graph capture of a two-device pipeline is not supported (a graph is bound "
                               "to one device); capture each stage on its own device instead")
        if s0 is None or s1 is None or capturing:
            # CPU devices: sequential reference semantics.  Under HIP-graph capture the micro-batches are
            # issued on the capturing stream only: backward through side-stream forwards breaks
            # hipStreamEndCapture on this ROCm stack (tools/graph_stream_repro.py, mode C), and the
            # replayed graph has no launch gaps to hide anyway.
            out = None
            lo = 0
            for s in splits:
                o = self.head(self.seq2(self.seq1(s.to(self.dev0)).to(self.dev1)))
                out = self._out(out, x.shape[0], o)
                out[lo: lo + o.shape[0]] = o
                lo += o.shape[0]
            return out
        # stage-0 work of micro-batch i overlaps stage-1 work of micro-batch i-1: the two devices
        # run independent streams, joined only by the activation hand-off event of each split.
        cur0, cur1 = torch.cuda.current_stream(self.dev0), torch.cuda.current_stream(self.dev1)
        s0.wait_stream(cur0)
        s1.wait_stream(cur1)
        handoff = []
        with torch.cuda.stream(s0):
            for sp in splits:
                a = self.seq1(sp.to(self.dev0, non_blocking=True))
                ev = torch.cuda.Event()
                ev.record(s0)
                handoff.append((a, ev))
        out = None
        lo = 0
        with torch.cuda.stream(s1):
            for a, ev in handoff:
                s1.wait_event(ev)
                a.record_stream(s1)  # produced on s0, read on s1: keep the allocator from recycling it early
                a1 = a.to(self.dev1, non_blocking=True)
                o = self.head(self.seq2(a1))
                if out is None:  # allocated on the stream that consumes it after the join below
                    with torch.cuda.stream(cur1):
                        out = self._out(None, x.shape[0], o)
                    out.record_stream(s1)
                # this micro-batch's logits go straight into their slice of the output (autograd records
                # the slice write; its backward hands each micro-batch a view of its gradient rows)
                out[lo: lo + o.shape[0]] = o
                lo += o.shape[0]
        cur0.wait_stream(s0)
        cur1.wait_stream(s1)
        return out

    @staticmethod
    def _out(out, rows, o):
        """The preallocated [rows, classes] output (no ``torch.cat`` of micro-batch outputs)."""
        if out is None:
            out = torch.empty((rows,) + tuple(o.shape[1:]), device=o.device, dtype=o.dtype)
        return out


def auto_place(model: tnn.Module, max_memory: Optional[Dict] = None, devices: Optional[Sequence] = None,
               no_split: Sequence[type] = ()) -> ModelParallel:
    """Greedy placement of ``model``'s children in order: fill each GPU up to its budget (bytes of
    parameters+buffers), then CPU.  ``max_memory`` maps device -> bytes; by default every visible GPU
    offers 90 % of its free memory (288 GB MI355X: large models fit without offload)."""
    if devices is None:
        devices = list(range(torch.cuda.device_count())) + ["cpu"]
    devs = [_dev(d) for d in devices]
    if max_memory is None:
        max_memory = {}
        for d in devs:
            if d.type == "cuda":
                free, _ = torch.cuda.mem_get_info(d)
                max_memory[d] = int(free * 0.9)
            else:
                max_memory[d] = 1 << 62
    budget = {_dev(k): v for k, v in max_memory.items()}
    children = list(model.stage_modules()) if hasattr(model, "stage_modules") else list(model.children())
    placement: List[List[tnn.Module]] = [[] for _ in devs]
    di, used = 0, 0
    for ch in children:
        size = sum(p.numel() * p.element_size() for p in ch.parameters()) + sum(
            b.numel() * b.element_size() for b in ch.buffers())
        while di < len(devs) - 1 and used + size > budget.get(devs[di], 0):
            di, used = di + 1, 0
        placement[di].append(ch)
        used += size
    stages, sdevs = [], []
    for d, mods in zip(devs, placement):
        if mods:
            stages.append(tnn.Sequential(*mods))
            sdevs.append(d)
    mp = ModelParallel(stages, sdevs)
    mp.device_map = {f"stage{i}": str(d) for i, d in enumerate(sdevs)}
    return mp
