"""HIP-graph capture of a whole training step (forward, loss, backward, optimizer update).

The reference leans on eager PyTorch; its small-micro-batch pipeline sweep (`NB03` raw lines
586-624, split sizes 1..60) is dominated by per-launch host overhead.  Instead of a tracing compiler
we capture the step once into a HIP graph and replay it: one ``hipGraphLaunch`` per step, no Python,
no per-kernel launch cost.  Everything in the step must already be device-resident and shape-static:
the fused optimizers keep their step counter on the device (``optim/fused.py:_device_step``) and
learning rate / gradient scale can be device tensors, so a replay is a real optimizer step.

    step = GraphedStep(lambda x, y: train_step(model, opt, x, y), (x0, y0), optimizer=opt)
    for x, y in batches:
        loss = step(x, y)       # copies into the static inputs, replays the graph

Inputs are copied into static buffers captured by the graph; the returned tensors are the graph's
static outputs (overwritten by the next replay — clone what you keep).
"""
from __future__ import annotations

from typing import Callable, Optional, Sequence

import torch


class GraphedStep:
    def __init__(self, fn: Callable, sample_inputs: Sequence[torch.Tensor], warmup: int = 2,
                 optimizer: Optional[torch.optim.Optimizer] = None, pool=None):
        if not torch.cuda.is_available():
            raise RuntimeError("GraphedStep needs a GPU")
        self.fn = fn
        self.optimizer = optimizer
        self.static_inputs = [t.detach().clone() for t in sample_inputs]
        self.replays = 0
        # warm up on a side stream: lazy allocations, autotuned plans and cached kernel attributes
        # happen here, outside the capture (PyTorch's documented whole-network capture recipe)
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(max(1, warmup)):
                fn(*self.static_inputs)
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph, pool=pool):
            self.static_outputs = fn(*self.static_inputs)
        # capture recorded the kernels without running them
        if optimizer is not None and hasattr(optimizer, "advance_steps"):
            optimizer.advance_steps(-1)

    def __call__(self, *inputs: torch.Tensor):
        for dst, src in zip(self.static_inputs, inputs):
            if src is not None and src.data_ptr() != dst.data_ptr():
                dst.copy_(src, non_blocking=True)
        self.graph.replay()
        self.replays += 1
        if self.optimizer is not None and hasattr(self.optimizer, "advance_steps"):
            self.optimizer.advance_steps(1)
        return self.static_outputs

    def pool(self):
        return self.graph.pool()
