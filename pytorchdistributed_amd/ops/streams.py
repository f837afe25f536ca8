"""Side-stream weight gradients (MI355X: overlap compute-bound wgrad GEMMs with the memory-bound
BatchNorm backward and the next layer's data gradient).

In a conv/linear backward the data gradient (dx) is on the critical path — the next layer's
backward needs it — while the weight gradient (dw) only feeds the gradient all-reduce and the
optimizer.  With ``PDA_WGRAD_STREAM=1`` (default on a GPU) the dw GEMM of each layer is launched on
a per-device side stream, ordered after the producing kernels by an event, so it runs concurrently
with the main stream's dgrad, BatchNorm backward reductions and applies of the layers below it:
the BN kernels stream HBM at 4-5 TB/s with the MFMA pipes idle, the wide wgrad tiles are MFMA-bound,
and the GPU's dispatcher fills CUs from both queues (also the CUs a wgrad launch's last, partial
round of tiles leaves idle: ResNet-50's M = 256*49*k rows quantise to 0.77 of 256 CUs).

Stream safety:
* every tensor read on the side stream is ``record_stream``-ed, so the caching allocator does not
  hand its memory to a main-stream allocation while the side kernel still reads it;
* the first side launch of a backward pass queues an autograd final callback that makes the main
  stream wait for the side stream, so anything after ``backward()`` (optimizer, grad clipping,
  checkpointing, HIP-graph capture end) sees finished gradients;
* :func:`producer_streams` lets a gradient all-reduce (DDP buckets) wait for the side stream as
  well as the main stream before it reads a bucket.
"""
from __future__ import annotations

import contextlib
import os
from typing import Dict, List

import torch

_streams: Dict[int, torch.cuda.Stream] = {}
_join_pending: Dict[int, bool] = {}
_join_task: Dict[int, int] = {}  # autograd graph task whose final callback joins the device's side stream
_enabled_override = None


def enabled() -> bool:
    if _enabled_override is not None:
        return _enabled_override
    return os.environ.get("PDA_WGRAD_STREAM", "1") == "1"


def set_enabled(flag) -> None:
    """Force side-stream weight gradients on/off (None: back to ``PDA_WGRAD_STREAM``)."""
    global _enabled_override
    _enabled_override = flag


def side_priority() -> str:
    """Queue priority of the side stream: ``normal`` (default) or ``low`` (``PDA_WGRAD_PRIO``).

    A wgrad GEMM wave holds a whole SIMD's register file, so a critical-path kernel launched while
    wgrad tiles are resident waits for a CU to drain; at equal priority the dispatcher often refills
    that CU from the side queue first (BN-backward finalize: 9 us alone, ~105 us beside the wgrads).
    Measured on ResNet-50 bs 640 (profiles/r2_stream_priority_ab.jsonl): low / normal side queue x
    high / normal main stream all within 0.5 % — HIP queue priority does not reorder CU dispatch
    here, so the default stays the plain pool stream."""
    return os.environ.get("PDA_WGRAD_PRIO", "normal")


def side_cus() -> int:
    """``PDA_WGRAD_CU_MASK=n``: the side stream's hardware queue dispatches to n CUs only (spread over the 8
    XCDs), so weight-gradient tiles can never occupy more than n CUs beside the critical-path kernels of
    the compute stream (0 = unmasked, the default)."""
    return int(os.environ.get("PDA_WGRAD_CU_MASK", "0"))


def side_stream(device: torch.device) -> torch.cuda.Stream:
    idx = device.index if device.index is not None else torch.cuda.current_device()
    s = _streams.get(idx)
    if s is None:
        if side_cus() > 0:
            from .._native import C

            s = torch.cuda.ExternalStream(C().stream_create_cumask(idx, side_cus()), device=torch.device("cuda", idx))
        elif side_priority() == "low":
            from .._native import C

            lo, _hi = C().stream_priority_range(idx)
            s = torch.cuda.ExternalStream(C().stream_create(idx, lo), device=torch.device("cuda", idx))
        else:
            s = torch.cuda.Stream(device=idx)
        _streams[idx] = s
    return s


def _join(idx: int) -> None:
    _join_pending[idx] = False
    _join_task.pop(idx, None)
    s = _streams.get(idx)
    if s is not None:
        torch.cuda.current_stream(idx).wait_stream(s)


def join(device: torch.device) -> None:
    """Make the current stream wait for the device's side stream now (also what the autograd final
    callback does).  Needed only after a backward that raised: its queued callbacks never ran."""
    idx = device.index if device.index is not None else torch.cuda.current_device()
    _join(idx)


def wait_side(device: torch.device) -> None:
    """Order the current stream after the side stream's queued work (without ending the pass's
    side-stream use): a gradient the current stream is about to combine with a side-stream output."""
    idx = device.index if device.index is not None else torch.cuda.current_device()
    s = _streams.get(idx)
    if s is not None and _join_pending.get(idx, False):
        torch.cuda.current_stream(idx).wait_stream(s)


def side_ok(param: torch.Tensor) -> bool:
    """May ``param``'s weight gradient be written on the side stream?

    Not for a parameter used more than once in a graph (tied weights, marked by
    :func:`..parallel.flat.grad_target`): autograd sums its gradients on the compute stream.  Not
    under ``create_graph=True`` (grad mode on inside backward): AccumulateGrad then clones the
    gradient on the compute stream instead of adopting the flat-buffer slot."""
    return enabled() and not getattr(param, "_pda_shared", False) and not torch.is_grad_enabled()


def active(device: torch.device) -> bool:
    """True while a backward pass has side-stream work on ``device`` not yet joined."""
    idx = device.index if device.index is not None else torch.cuda.current_device()
    return _join_pending.get(idx, False)


@contextlib.contextmanager
def wgrad_stream(device: torch.device, *tensors: torch.Tensor):
    """Run the body on the device's side stream, after everything queued so far on the current
    stream; ``tensors`` (inputs the body reads) are protected from reuse until the side stream is
    done with them.  Must be entered inside an autograd backward pass (it queues the join)."""
    idx = device.index if device.index is not None else torch.cuda.current_device()
    main = torch.cuda.current_stream(idx)
    s = side_stream(device)
    s.wait_stream(main)
    for t in tensors:
        if t is not None:
            t.record_stream(s)
    # one join per backward pass: keyed on the autograd graph task, so a backward that raised (its
    # callbacks never run) cannot leave a stale "join pending" that stops the next pass from queueing
    task = torch._C._current_graph_task_id()
    if not _join_pending.get(idx, False) or _join_task.get(idx) != task:
        _join_pending[idx] = True
        _join_task[idx] = task
        torch.autograd.Variable._execution_engine.queue_callback(lambda: _join(idx))
    with torch.cuda.stream(s):
        yield s


def producer_streams(device: torch.device) -> List[torch.cuda.Stream]:
    """Streams whose queued work may still be writing gradients on ``device``: the current stream
    and, during a backward pass with side-stream weight gradients, the side stream."""
    idx = device.index if device.index is not None else torch.cuda.current_device()
    out = [torch.cuda.current_stream(idx)]
    if _join_pending.get(idx, False) and idx in _streams:
        out.append(_streams[idx])
    return out
