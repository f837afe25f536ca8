"""Fault injection for failure-handling tests (test tier T5).

``PDA_FAULT="rank:step:kind[,rank:step:kind...]"`` with kind in {crash, hang, slow, exit}; the Trainer
calls :func:`maybe_inject` once per step.  ``PDA_FAULT_ONCE=1`` (default) only fires on the first launch
(``PDA_RESTART_COUNT`` == 0) so a ``--max-restarts`` relaunch can be tested for recovery.
"""
from __future__ import annotations

import os
import sys
import time


def _specs():
    raw = os.environ.get("PDA_FAULT", "")
    out = []
    for item in filter(None, raw.split(",")):
        r, s, k = item.split(":")
        out.append((int(r), int(s), k))
    return out


def maybe_inject(rank: int, step: int):
    specs = _specs()
    if not specs:
        return
    if os.environ.get("PDA_FAULT_ONCE", "1") == "1" and int(os.environ.get("PDA_RESTART_COUNT", "0")) > 0:
        return
    for r, s, kind in specs:
        if r == rank and s == step:
            sys.stderr.write(f"[fault] rank {rank} step {step}: injecting {kind}\n")
            sys.stderr.flush()
            if kind == "crash":
                raise RuntimeError(f"injected crash on rank {rank} at step {step}")
            if kind == "exit":
                os._exit(17)
            if kind == "hang":
                while True:
                    time.sleep(1)
            if kind == "slow":
                time.sleep(float(os.environ.get("PDA_FAULT_SLOW_S", "2")))
