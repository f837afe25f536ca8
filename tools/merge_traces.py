"""Merge the per-rank rocprofv3 kernel traces written by ``pda-run --profile-dir D`` (``D/rank<r>/…
*kernel_trace.csv``) into ONE Chrome/Perfetto trace (``pid`` = rank, ``tid`` = HIP queue), and report
per rank the kernel time, the RCCL kernel time and how much of it was NOT overlapped by compute
kernels (the overlap ratio of bucketed all-reduce vs backward, measured from the trace).

    python tools/merge_traces.py D [merged.json]      # open merged.json in ui.perfetto.dev
"""
from __future__ import annotations

import csv
import glob
import json
import os
import re
import sys
from typing import Dict, List, Tuple

_COMM = re.compile(r"nccl|rccl|allreduce|all_reduce|reduce_scatter|allgather|xgmi_", re.I)


def _union(iv: List[Tuple[int, int]]) -> List[Tuple[int, int]]:
    out: List[Tuple[int, int]] = []
    for a, b in sorted(iv):
        if out and a <= out[-1][1]:
            out[-1] = (out[-1][0], max(out[-1][1], b))
        else:
            out.append((a, b))
    return out


def _covered(a: int, b: int, merged: List[Tuple[int, int]]) -> int:
    tot = 0
    for x, y in merged:
        if y <= a:
            continue
        if x >= b:
            break
        tot += min(b, y) - max(a, x)
    return tot


def load_rank(path: str):
    rows = list(csv.DictReader(open(path)))
    return [(r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
             int(r.get("Queue_Id") or r.get("Stream_Id") or 0)) for r in rows]


def merge(directory: str, out: str | None = None) -> Dict[int, dict]:
    files = {}
    for d in glob.glob(os.path.join(directory, "rank*")):
        m = re.search(r"rank(\d+)$", d)
        hits = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
        if m and hits:
            files[int(m.group(1))] = hits[0]
    if not files:
        raise SystemExit(f"no rank*/…kernel_trace.csv under {directory}")
    data = {r: load_rank(p) for r, p in sorted(files.items())}
    t0 = min(k[1] for ks in data.values() for k in ks)
    events, report = [], {}
    for r, ks in data.items():
        comp = _union([(s, e) for n, s, e, _ in ks if not _COMM.search(n)])
        comm = [(s, e) for n, s, e, _ in ks if _COMM.search(n)]
        comm_ns = sum(e - s for s, e in comm)
        exposed = sum((e - s) - _covered(s, e, comp) for s, e in comm)
        report[r] = {"kernels": len(ks), "kernel_ms": round(sum(e - s for _, s, e, _ in ks) / 1e6, 3),
                     "comm_ms": round(comm_ns / 1e6, 3), "comm_exposed_ms": round(exposed / 1e6, 3),
                     "overlap_ratio": round(1 - exposed / comm_ns, 3) if comm_ns else None}
        for n, s, e, q in ks:
            events.append({"name": n[:160], "ph": "X", "pid": r, "tid": q, "ts": (s - t0) / 1e3,
                           "dur": (e - s) / 1e3, "cat": "comm" if _COMM.search(n) else "compute"})
        events.append({"name": "process_name", "ph": "M", "pid": r, "args": {"name": f"rank {r}"}})
    if out:
        with open(out, "w") as f:
            json.dump({"traceEvents": events, "displayTimeUnit": "ms"}, f)
    return report


if __name__ == "__main__":
    rep = merge(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None)
    for r, v in rep.items():
        print(json.dumps({"rank": r, **v}))
