"""Per-step GPU occupancy from a rocprofv3 kernel trace: is the step bound by kernels or by gaps?

    python tools/busy_timeline.py <kernel_trace.csv> <step_marker_substring> [skip_steps] [out.md]

Steps are delimited by launches of the marker kernel (e.g. ``sgd`` for the fused optimizer, one
launch per step).  For each step it reports the wall span, the union of all kernel intervals (time
at least one kernel runs), the busy time per HIP stream / queue, and the idle gaps of the busiest
stream — a step whose union is close to its span is kernel-bound (only less kernel work helps); a
large gap total says launches, host syncs or dependency stalls are exposed.
"""
import csv
import sys
from collections import defaultdict


def _col(row, *names):
    for n in names:
        if n in row:
            return row[n]
    raise KeyError(names)


def load(path):
    out = []
    for r in csv.DictReader(open(path)):
        name = _col(r, "Kernel_Name", "KernelName", "Name")
        t0 = int(_col(r, "Start_Timestamp", "StartNs", "Start"))
        t1 = int(_col(r, "End_Timestamp", "EndNs", "End"))
        q = r.get("Stream_Id") or r.get("Queue_Id") or "0"
        out.append((t0, t1, name, q))
    out.sort()
    return out


def union(iv):
    tot, cur0, cur1 = 0, None, None
    for a, b in sorted(iv):
        if cur1 is None or a > cur1:
            if cur1 is not None:
                tot += cur1 - cur0
            cur0, cur1 = a, b
        else:
            cur1 = max(cur1, b)
    if cur1 is not None:
        tot += cur1 - cur0
    return tot


def gaps(iv):
    """Idle intervals (ns) between consecutive kernels of one stream."""
    out, end = [], None
    for a, b in sorted(iv):
        if end is not None and a > end:
            out.append(a - end)
        end = b if end is None else max(end, b)
    return out


def main():
    path, marker = sys.argv[1], sys.argv[2]
    skip = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    rows = load(path)
    marks = [t0 for t0, _, n, _ in rows if marker in n]
    if len(marks) < skip + 2:
        raise SystemExit(f"only {len(marks)} marker launches of {marker!r}")
    lines = ["| step | span ms | union busy ms | busy % | per-stream busy ms | main-stream gaps ms (count) |",
             "|---:|---:|---:|---:|---|---|"]
    for i in range(skip, len(marks) - 1):
        lo, hi = marks[i], marks[i + 1]
        ks = [(max(a, lo), min(b, hi), n, q) for a, b, n, q in rows if b > lo and a < hi]
        u = union([(a, b) for a, b, _, _ in ks])
        per = defaultdict(list)
        for a, b, _, q in ks:
            per[q].append((a, b))
        busy = {q: union(v) for q, v in per.items()}
        main_q = max(busy, key=busy.get)
        g = gaps(per[main_q])
        per_s = ", ".join(f"{q}: {v / 1e6:.2f}" for q, v in sorted(busy.items(), key=lambda kv: -kv[1]))
        lines.append(f"| {i} | {(hi - lo) / 1e6:.2f} | {u / 1e6:.2f} | {100 * u / (hi - lo):.1f} | {per_s} | "
                     f"{sum(g) / 1e6:.2f} ({len(g)}) |")
    text = "\n".join(lines)
    print(text)
    if len(sys.argv) > 4:
        open(sys.argv[4], "w").write(text + "\n")


if __name__ == "__main__":
    main()
