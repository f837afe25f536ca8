"""Per-step kernel table from a rocprofv3 kernel trace (``*_kernel_trace.csv``): the dispatches between two
consecutive launches of the optimizer kernel (one steady-state training step), so init-time fills and
copies are not averaged into the step as they are by ``--stats`` divided by the step count.

    python tools/step_kernels.py TRACE.csv [--marker sgd_kernel] [--step -2] [--top 40] [--out FILE.md]
"""
import argparse
import collections
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--marker", default="sgd_kernel", help="kernel name substring that ends a step")
    ap.add_argument("--step", type=int, default=-2, help="which step (index into the marker list)")
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--out", default="")
    ap.add_argument("--title", default="")
    ap.add_argument("--stream", default="", help="only the dispatches of this Stream_Id / Queue_Id ('list': "
                                                  "print each stream's kernel time in the step)")
    a = ap.parse_args()
    rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
    marks = [i for i, r in enumerate(rows) if a.marker in r["Kernel_Name"]]
    if len(marks) < 2:
        raise SystemExit(f"fewer than two '{a.marker}' dispatches in the trace")
    lo, hi = marks[a.step - 1], marks[a.step]
    step = rows[lo + 1: hi + 1]

    def sid(r):
        return r.get("Stream_Id") or r.get("Queue_Id") or "0"

    if a.stream == "list":
        per = collections.defaultdict(float)
        cnt = collections.Counter()
        for r in step:
            per[sid(r)] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
            cnt[sid(r)] += 1
        for k, v in sorted(per.items(), key=lambda kv: -kv[1]):
            print(f"stream {k}: {v:.3f} ms of kernels in {cnt[k]} dispatches")
        return
    if a.stream:
        step = [r for r in step if sid(r) == a.stream]
    t = collections.defaultdict(float)
    n = collections.Counter()
    for r in step:
        k = r["Kernel_Name"]
        t[k] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        n[k] += 1
    wall = (int(step[-1]["End_Timestamp"]) - int(step[0]["Start_Timestamp"])) / 1e6
    total = sum(t.values())
    lines = [f"# {a.title or a.trace}: one steady-state step (dispatches after one '{a.marker}' up to the next)",
             f"# {len(step)} dispatches, kernel time {total:.3f} ms, first-start to last-end {wall:.3f} ms; "
             f"vendor fills/copies in the step: "
             f"{sum(v for k, v in n.items() if 'rocclr' in k)}",
             "", "| ms | % | calls | kernel |", "|---:|---:|---:|---|"]
    for k, v in sorted(t.items(), key=lambda kv: -kv[1])[: a.top]:
        name = k.replace("pda::(anonymous namespace)::", "").replace("(anonymous namespace)::", "")[:140]
        lines.append(f"| {v:.3f} | {100 * v / total:.1f} | {n[k]} | `{name}` |")
    text = "\n".join(lines)
    print(text)
    if a.out:
        open(a.out, "w").write(text + "\n")


if __name__ == "__main__":
    main()
