"""Summarise rocprofv3 kernel statistics: per-step ms, % and calls per kernel (top N).

Input: the ``*_kernel_stats.csv`` of ``rocprofv3 --stats --output-format csv`` or the rocpd SQLite
database (``*_results.db``) that rocprofv3 writes by default.

    python tools/prof_summary.py <csv|db> <profiled_steps> [top] [out.md]
"""
import csv
import sqlite3
import sys


def short(n: str) -> str:
    for a, b in [("pda::(anonymous namespace)::", ""), ("at::native::", ""), ("(anonymous namespace)::", "")]:
        n = n.replace(a, b)
    return n[:140]


def load_rows(path):
    """[(name, total_ns, calls)] sorted by total time."""
    if path.endswith(".db"):
        con = sqlite3.connect(path)
        q = ("SELECT S.display_name, SUM(K.end - K.start), COUNT(*) FROM rocpd_kernel_dispatch K "
             "JOIN rocpd_info_kernel_symbol S ON S.id = K.kernel_id AND S.guid = K.guid "
             "GROUP BY S.display_name ORDER BY 2 DESC")
        return [(n, float(t), int(c)) for n, t, c in con.execute(q)]
    rows = list(csv.DictReader(open(path)))
    return [(r["Name"], float(r["TotalDurationNs"]), int(r["Calls"])) for r in rows]


def main(path, steps, top=40, out=None):
    rows = load_rows(path)
    tot = sum(t for _, t, _ in rows)
    lines = [f"# kernel time per step (rocprofv3 --kernel-trace --stats), {steps:g} profiled steps",
             f"# total GPU kernel time per step: {tot / steps / 1e6:.3f} ms", "",
             "| ms/step | % | calls/step | kernel |", "|---:|---:|---:|---|"]
    for n, t, c in rows[:top]:
        lines.append(f"| {t / steps / 1e6:.3f} | {100.0 * t / tot:.1f} | {c / steps:.1f} | `{short(n)}` |")
    text = "\n".join(lines) + "\n"
    if out:
        open(out, "w").write(text)
    print(text)


if __name__ == "__main__":
    main(sys.argv[1], float(sys.argv[2]), int(sys.argv[3]) if len(sys.argv) > 3 else 40,
         sys.argv[4] if len(sys.argv) > 4 else None)
