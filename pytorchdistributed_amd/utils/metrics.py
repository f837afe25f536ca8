"""Per-rank metrics JSONL: step time, throughput, loss, communication volume and
bandwidth, exposed-communication (overlap) ratio and peak HBM.  The reference logs nothing but the
epoch line (`ddp_gpus.py:46`); the exact reference line is kept in :mod:`.log`.

    m = MetricsLogger("runs/metrics", rank)       # or PDA_METRICS_DIR=runs/metrics
    m.log(step=i, step_ms=..., items_per_s=..., loss=loss.item(), **ddp.comm_stats(reset=True))
    m.close()

One ``rank{r}.jsonl`` per rank, one JSON object per line; :func:`read_metrics` loads them back and
:func:`summarize` aggregates the job (max step time over ranks, summed throughput).
"""
from __future__ import annotations

import glob
import json
import os
import time
from typing import Dict, List, Optional

import torch


def bus_bandwidth_gbs(op: str, nbytes: int, seconds: float, world: int) -> float:
    """NCCL-tests convention: algorithm bandwidth x the collective's bus factor."""
    if seconds <= 0 or world <= 1:
        return 0.0
    alg = nbytes / seconds / 1e9
    factor = {"all_reduce": 2 * (world - 1) / world, "all_gather": (world - 1) / world,
              "reduce_scatter": (world - 1) / world, "broadcast": 1.0, "all_to_all": (world - 1) / world}.get(op, 1.0)
    return alg * factor


class MetricsLogger:
    def __init__(self, directory: Optional[str] = None, rank: Optional[int] = None, flush_every: int = 1):
        directory = directory or os.environ.get("PDA_METRICS_DIR", "")
        self.enabled = bool(directory)
        self.rank = int(os.environ.get("RANK", "0")) if rank is None else rank
        self.flush_every = max(1, flush_every)
        self._n = 0
        self._fh = None
        if self.enabled:
            os.makedirs(directory, exist_ok=True)
            self.path = os.path.join(directory, f"rank{self.rank}.jsonl")
            self._fh = open(self.path, "a", buffering=1)

    def log(self, **fields):
        if not self.enabled:
            return
        rec = {"time": time.time(), "rank": self.rank}
        if torch.cuda.is_available() and torch.cuda.is_initialized():
            rec["peak_hbm_gb"] = round(torch.cuda.max_memory_allocated() / 2 ** 30, 3)
        for k, v in fields.items():
            if isinstance(v, torch.Tensor):
                v = v.item() if v.numel() == 1 else v.tolist()
            rec[k] = v
        self._fh.write(json.dumps(rec) + "\n")
        self._n += 1
        if self._n % self.flush_every == 0:
            self._fh.flush()

    def close(self):
        if self._fh is not None:
            self._fh.close()
            self._fh = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


def read_metrics(directory: str) -> Dict[int, List[dict]]:
    out: Dict[int, List[dict]] = {}
    for p in sorted(glob.glob(os.path.join(directory, "rank*.jsonl"))):
        r = int(os.path.basename(p)[4:-6])
        with open(p) as fh:
            out[r] = [json.loads(line) for line in fh if line.strip()]
    return out


def summarize(directory: str, key_time: str = "step_ms", key_tput: str = "items_per_s") -> dict:
    """Job-level view: per step, MAX step time over ranks and SUM of per-rank throughput."""
    data = read_metrics(directory)
    if not data:
        return {}
    steps: Dict[int, List[dict]] = {}
    for recs in data.values():
        for rec in recs:
            if "step" in rec:
                steps.setdefault(rec["step"], []).append(rec)
    rows = []
    for s in sorted(steps):
        recs = steps[s]
        row = {"step": s, "ranks": len(recs)}
        if all(key_time in r for r in recs):
            row[key_time] = max(r[key_time] for r in recs)
        if all(key_tput in r for r in recs):
            row[key_tput] = sum(r[key_tput] for r in recs)
        if all("exposed_comm_ms" in r for r in recs):
            row["exposed_comm_ms"] = max(r["exposed_comm_ms"] for r in recs)
        rows.append(row)
    return {"ranks": sorted(data), "steps": rows}
