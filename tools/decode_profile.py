"""Per-decode-step kernel breakdown from a rocprofv3 kernel trace of bench/llama_serve.py: kernels after
the last prefill attention, grouped by name, divided by the number of decode steps.

    python tools/decode_profile.py <prof_kernel_trace.csv> <n_layers> [out.md]
"""
import collections
import csv
import sys


def main(path, n_layers, out=None):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    last_pre = max(i for i, r in enumerate(rows) if "attn_fwd" in r["Kernel_Name"])
    j = next(i for i in range(last_pre, len(rows)) if "decode_attn_kernel" in rows[i]["Kernel_Name"])
    dec = rows[j:]
    steps = sum(1 for r in dec if "decode_attn_kernel" in r["Kernel_Name"]) / n_layers
    t0, t1 = int(dec[0]["Start_Timestamp"]), int(dec[-1]["End_Timestamp"])
    agg = collections.defaultdict(lambda: [0, 0])
    for r in dec:
        n = r["Kernel_Name"][:110]
        agg[n][0] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        agg[n][1] += 1
    tot = sum(v[0] for v in agg.values())
    lines = [f"# decode step kernels, {steps:.0f} steps after the last prefill",
             f"# wall per step {(t1 - t0) / steps / 1e6:.3f} ms, kernel time per step {tot / steps / 1e6:.3f} ms", "",
             "| ms/step | % | calls/step | kernel |", "|---:|---:|---:|---|"]
    for n, (t, c) in sorted(agg.items(), key=lambda x: -x[1][0])[:18]:
        lines.append(f"| {t / steps / 1e6:.3f} | {100 * t / tot:.1f} | {c / steps:.1f} | `{n}` |")
    text = "\n".join(lines) + "\n"
    if out:
        open(out, "w").write(text)
    print(text)


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]), sys.argv[3] if len(sys.argv) > 3 else None)
