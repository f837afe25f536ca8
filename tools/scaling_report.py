"""Scaling table from bench JSON lines (SURVEY §5.5 ``scaling_report``): reads one or more files of
``bench.py`` output lines (e.g. the N=1,2,4,8 runs), prints per-N value, ms/step and weak-scaling
efficiency value(N) / (N * value(1)).

    python tools/scaling_report.py profiles/*.jsonl [--markdown]
"""
from __future__ import annotations

import argparse
import json
import sys


def load(paths):
    rows = {}
    for p in paths:
        with open(p) as fh:
            for line in fh:
                line = line.strip()
                if not line.startswith("{"):
                    continue
                try:
                    r = json.loads(line)
                except json.JSONDecodeError:
                    continue
                if "n_gpus" in r and "value" in r:
                    rows.setdefault(r.get("metric", "?"), {})[int(r["n_gpus"])] = r
    return rows


def report(rows, markdown=False):
    out = []
    for metric, by_n in rows.items():
        base = by_n.get(1)
        out.append(f"## {metric}" if markdown else metric)
        if markdown:
            out += ["", "| GPUs | value | ms/step | efficiency |", "|---:|---:|---:|---:|"]
        for n in sorted(by_n):
            r = by_n[n]
            eff = r["value"] / (n * base["value"]) if base else None
            effs = f"{eff * 100:.1f}%" if eff is not None else "n/a"
            if markdown:
                out.append(f"| {n} | {r['value']:.1f} | {r.get('ms_per_step', float('nan')):.2f} | {effs} |")
            else:
                out.append(f"  N={n}: {r['value']:.1f} {r.get('unit', '')}  {r.get('ms_per_step', 0):.2f} ms/step  eff {effs}")
        out.append("")
    return "\n".join(out)


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("files", nargs="+")
    ap.add_argument("--markdown", action="store_true")
    a = ap.parse_args(argv)
    print(report(load(a.files), a.markdown))
    return 0


if __name__ == "__main__":
    sys.exit(main())
