"""How much of the communication kernels' time runs beside compute kernels, from a rocprofv3 kernel trace
(``*_kernel_trace.csv``, default multi-stream run): for every RCCL kernel, the time during which at least
one non-RCCL kernel was also executing.  The evidence for "the P2P / collective is off the critical
path" (pipeline sends must not make the compute stream wait).

    python tools/overlap_report.py TRACE.csv [--comm nccl] [--skip-first N] [--json]
"""
import argparse
import csv
import json


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--comm", default="nccl", help="substring (case-insensitive) naming communication kernels")
    ap.add_argument("--skip-first", type=int, default=0, help="ignore the first N communication kernels (warm-up)")
    ap.add_argument("--json", action="store_true")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows]
    ks.sort()
    comm = [k for k in ks if a.comm.lower() in k[2].lower()][a.skip_first:]
    comp = [k for k in ks if a.comm.lower() not in k[2].lower()]
    total = overl = 0
    n_over = 0
    for s, e, _ in comm:
        total += e - s
        # union of compute intervals clipped to [s, e]
        iv = sorted((max(s, cs), min(e, ce)) for cs, ce, _ in comp if cs < e and ce > s)
        cov, cur_s, cur_e = 0, None, None
        for x, y in iv:
            if cur_e is None or x > cur_e:
                if cur_e is not None:
                    cov += cur_e - cur_s
                cur_s, cur_e = x, y
            else:
                cur_e = max(cur_e, y)
        if cur_e is not None:
            cov += cur_e - cur_s
        overl += cov
        n_over += cov > 0
    out = {"comm_kernels": len(comm), "comm_ms": total / 1e6, "overlapped_ms": overl / 1e6,
           "overlapped_frac": (overl / total) if total else 0.0, "kernels_with_overlap": n_over}
    print(json.dumps(out) if a.json else "\n".join(f"{k}: {v}" for k, v in out.items()))


if __name__ == "__main__":
    main()
