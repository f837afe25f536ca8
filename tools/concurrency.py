"""For each kernel family matching a substring in a rocprofv3 kernel trace: mean duration, and the
share of its time during which a kernel of ANOTHER stream / queue was running (a kernel that runs
slower in a training step than in isolation is usually sharing the CUs).

    python tools/concurrency.py <kernel_trace.csv> <substring> [more substrings ...]
"""
import bisect
import csv
import sys


def main():
    path, subs = sys.argv[1], sys.argv[2:]
    rows = []
    for r in csv.DictReader(open(path)):
        q = r.get("Stream_Id") or r.get("Queue_Id") or "0"
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), q, r["Kernel_Name"]))
    rows.sort()
    starts = [r[0] for r in rows]
    for s in subs:
        sel = [r for r in rows if s in r[3]]
        if not sel:
            print(f"{s}: none")
            continue
        tot = ov = 0
        for (a, b, q, _n) in sel:
            tot += b - a
            # intervals of other queues that intersect [a, b)
            segs = []
            i = bisect.bisect_left(starts, a - 50_000_000)
            for (c, d, q2, _n2) in rows[i:]:
                if c >= b:
                    break
                if q2 != q and d > a:
                    segs.append((max(a, c), min(b, d)))
            segs.sort()
            cur_a = cur_b = None
            for (c, d) in segs:
                if cur_b is None or c > cur_b:
                    if cur_b is not None:
                        ov += cur_b - cur_a
                    cur_a, cur_b = c, d
                else:
                    cur_b = max(cur_b, d)
            if cur_b is not None:
                ov += cur_b - cur_a
        print(f"{s}: {len(sel)} launches, mean {tot / len(sel) / 1e3:.1f} us, {100 * ov / max(tot, 1):.0f} % of the time beside another queue's kernel")


if __name__ == "__main__":
    main()
