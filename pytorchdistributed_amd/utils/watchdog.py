"""Collective watchdog front end.  The native thread lives in ``_C.Watchdog``
(`csrc/runtime/watchdog.cpp`); this module owns the per-process instance and the ``watch`` helper
used by DDP (bucket all-reduces), FSDP (all-gather / reduce-scatter) and the pipeline (P2P waits).

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


def attach(ticket: int, work) -> None:
    """Tie an armed ticket to ``work``'s completion event, when it has one (native RCCL works, event
    works): the native thread then disarms the ticket by itself once the collective completed, so
    a ticket never outlives its collective even when the owner's sweep does not run (a DDP stage
    driven by a pipeline schedule) or the process idles after its last step.  The caller keeps
    ``work`` alive until it calls :func:`disarm`."""
    if not ticket or _WD is None:
        return
    ev = getattr(work, "event", None)
    if ev is None:
        return
    handle = ev if isinstance(ev, int) else getattr(ev, "cuda_event", 0)
    if handle:
        _WD.attach_event(ticket, int(handle))


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
