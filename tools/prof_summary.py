"""Summarise a rocprofv3 --stats kernel CSV: per-step ms, % and calls per kernel (top N)."""
import csv
import sys


def short(n: str) -> str:
    for a, b in [("pda::(anonymous namespace)::", ""), ("at::native::", ""), ("(anonymous namespace)::", "")]:
        n = n.replace(a, b)
    return n[:140]


def main(path, steps, top=40, out=None):
    rows = list(csv.DictReader(open(path)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    lines = [f"# kernel time per step (rocprofv3 --kernel-trace --stats), {steps} profiled steps",
             f"# total GPU kernel time per step: {tot / steps / 1e6:.3f} ms", "",
             "| ms/step | % | calls/step | kernel |", "|---:|---:|---:|---|"]
    for r in rows[:top]:
        lines.append(f"| {float(r['TotalDurationNs']) / steps / 1e6:.3f} | {float(r['Percentage']):.1f} | "
                     f"{int(r['Calls']) / steps:.1f} | `{short(r['Name'])}` |")
    text = "\n".join(lines) + "\n"
    if out:
        open(out, "w").write(text)
    print(text)


if __name__ == "__main__":
    main(sys.argv[1], float(sys.argv[2]), int(sys.argv[3]) if len(sys.argv) > 3 else 40,
         sys.argv[4] if len(sys.argv) > 4 else None)
