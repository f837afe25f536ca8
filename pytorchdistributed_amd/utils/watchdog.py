"""Collective watchdog front end.  The native thread lives in ``_C.Watchdog``
(`csrc/runtime/watchdog.cpp`); this module owns the per-process instance and the ``watch`` helper
used by DDP (bucket all-reduces), FSDP (parameter all-gathers / gradient reduce-scatters, ``track``) and
the pipeline (native P2P groups, ``track``; c10d P2P waits, ``watch``).  Tickets of GPU collectives
retire on an event the native thread records behind the collective on its stream.

Config: ``PDA_WATCHDOG`` (default on), ``PDA_COLLECTIVE_TIMEOUT_S`` (default 600 s),
``PDA_WATCHDOG_ACTION`` = abort | exit | report.
"""
from __future__ import annotations

import faulthandler
import os
import sys
from contextlib import contextmanager
from typing import Optional

from .. import _native

_WD = None


def get_watchdog(rank: Optional[int] = None):
    """The process's watchdog, or None when disabled (``PDA_WATCHDOG=0``)."""
    global _WD
    if _WD is not None:
        return _WD
    from ..config import get_config

    cfg = get_config()
    if not cfg.watchdog:
        return None
    if rank is None:
        rank = int(os.environ.get("RANK", "0"))
    action = os.environ.get("PDA_WATCHDOG_ACTION", "abort")
    if action == "abort" and not faulthandler.is_enabled():
        faulthandler.enable(file=sys.stderr, all_threads=True)  # Python stacks of every thread on SIGABRT
    _WD = _native.C().Watchdog(cfg.collective_timeout_s, rank, action)
    return _WD


def reset_watchdog():
    global _WD
    if _WD is not None:
        _WD.stop()
    _WD = None


def arm(desc: str, timeout: float = -1.0) -> int:
    wd = get_watchdog()
    return wd.arm(desc, timeout) if wd is not None else 0


def attach(ticket: int, stream) -> bool:
    """Tie an armed ticket to the completion of everything queued so far on ``stream`` (a
    ``torch.cuda.Stream`` or a raw handle — the stream the collective was just enqueued on): the native
    thread records an event of its own there and disarms the ticket once that event has completed, so a
    ticket never outlives its collective even when the owner's sweep does not run (a DDP stage driven by
    a pipeline schedule, an FSDP unit whose work is waited on by a stream only) or the process idles after
    its last step.  The ticket owns the event: nothing the caller frees can leave the watchdog querying a
    dead handle.  Returns False when the watchdog is off or has no GPU event support."""
    if not ticket or _WD is None or stream is None:
        return False
    handle = stream if isinstance(stream, int) else getattr(stream, "cuda_stream", 0)
    return bool(_WD.attach_stream(ticket, int(handle)))


def track(desc: str, stream, timeout: float = -1.0) -> int:
    """Arm a ticket for a collective just enqueued on ``stream`` and let it retire on the GPU's own
    completion (:func:`attach`).  Returns the ticket (0 when the watchdog is off)."""
    t = arm(desc, timeout)
    if t and not attach(t, stream):
        disarm(t)  # no event support: nothing would ever retire it
        return 0
    return t


def armed() -> int:
    """Tickets currently armed in this process (0 when the watchdog is off)."""
    return _WD.armed if _WD is not None else 0


def disarm(ticket: int):
    if ticket and _WD is not None:
        _WD.disarm(ticket)


@contextmanager
def watch(desc: str, timeout: float = -1.0):
    """Deadline for a blocking section (a collective wait, a P2P receive...)."""
    t = arm(desc, timeout)
    try:
        yield
    finally:
        disarm(t)
