"""Per-rank logging.

The reference prints from every rank with no synchronisation, so lines from different ranks glue
together (`02_ddp.ipynb` output).  Here every line is written with one ``write`` call and
flushed, and :func:`epoch_line` keeps the reference's exact format (`ddp_gpus.py:46`).
"""
from __future__ import annotations

import json
import os
import sys
import time


def epoch_line(gpu_id, epoch: int, batch_size: int, steps: int) -> str:
    return f"[GPU: {gpu_id}] Epoch: {epoch} | Batchsize: {batch_size} | Steps: {steps}"


def log(msg: str, rank0_only: bool = False, stream=None):
    rank = int(os.environ.get("RANK", "0"))
    if rank0_only and rank != 0:
        return
    stream = stream or sys.stdout
    stream.write(msg + "\n")
    stream.flush()


class MetricsWriter:
    """JSONL metrics per rank (step time, throughput, loss, ...)."""

    def __init__(self, path: str | None):
        self.path = path
        self._f = open(path, "a", buffering=1) if path else None

    def write(self, **kv):
        if self._f is None:
            return
        kv.setdefault("time", time.time())
        kv.setdefault("rank", int(os.environ.get("RANK", "0")))
        self._f.write(json.dumps(kv) + "\n")

    def close(self):
        if self._f:
            self._f.close()
            self._f = None
