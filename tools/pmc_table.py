"""Per-kernel hardware-counter table for a whole training step from three rocprofv3 --pmc passes.

    python tools/pmc_table.py <sq_dir> <fetch_dir> <write_dir> [top] [out.md]

Each dir holds the ``*_counter_collection.csv`` and ``*_kernel_trace.csv`` of one
``rocprofv3 --pmc ... --kernel-trace --output-format csv`` pass over the same program.  Counters are
summed over every dispatch of a kernel name; time comes from the SQ pass's kernel trace.
Derived columns:
  mfma/CU-cyc   SQ_VALU_MFMA_BUSY_CYCLES / (256 CUs * GRBM_GUI_ACTIVE / 8): MFMA-busy cycles per CU per
                GPU cycle (GRBM_GUI_ACTIVE is summed over the 8 XCDs); 4.0 would be all 4 SIMDs busy
  lds-confl     SQ_LDS_BANK_CONFLICT / SQ_INSTS_LDS (conflict cycles per LDS instruction)
  HBM GB/s      (2 * FETCH_SIZE + WRITE_SIZE) * 1024 B / kernel time; FETCH_SIZE doubled because on gfx950
                it tallies half the bytes of a wide streaming read (MI355X_MICROARCH.md, HBM section)
"""
import collections
import csv
import glob
import os
import sys


def _one(d, suffix):
    hits = glob.glob(os.path.join(d, "**", f"*{suffix}"), recursive=True)
    if not hits:
        raise SystemExit(f"no *{suffix} under {d}")
    return hits[0]


def counters(d):
    out = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(_one(d, "counter_collection.csv"))):
        out[r["Kernel_Name"]][r["Counter_Name"]] += float(r["Counter_Value"])
    return out


def durations(d):
    out = collections.defaultdict(lambda: [0.0, 0])
    for r in csv.DictReader(open(_one(d, "kernel_trace.csv"))):
        e = out[r["Kernel_Name"]]
        e[0] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
        e[1] += 1
    return out


def short(n):
    for a in ("pda::(anonymous namespace)::", "at::native::", "(anonymous namespace)::"):
        n = n.replace(a, "")
    return n.split("(")[0][:90]


def main(sq_dir, fetch_dir, write_dir, top=25, out=None):
    sq, fe, wr, du = counters(sq_dir), counters(fetch_dir), counters(write_dir), durations(sq_dir)
    total = sum(v[0] for v in du.values())
    lines = [f"# per-kernel counters over the profiled steps (3 rocprofv3 --pmc passes); kernel time total "
             f"{total * 1e3:.1f} ms", "",
             "| ms | % | calls | mfma/CU-cyc | lds-confl/inst | HBM GB/s | kernel |",
             "|---:|---:|---:|---:|---:|---:|---|"]
    for name, (t, n) in sorted(du.items(), key=lambda kv: -kv[1][0])[:top]:
        c = sq.get(name, {})
        gui = c.get("GRBM_GUI_ACTIVE", 0.0)
        mf = c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / (256 * gui / 8) if gui else float("nan")
        li = c.get("SQ_INSTS_LDS", 0.0)
        lc = c.get("SQ_LDS_BANK_CONFLICT", 0.0) / li if li else float("nan")
        by = (2 * fe.get(name, {}).get("FETCH_SIZE", 0.0) + wr.get(name, {}).get("WRITE_SIZE", 0.0)) * 1024
        gbs = by / t / 1e9 if t else float("nan")
        lines.append(f"| {t * 1e3:.2f} | {100 * t / total:.1f} | {n} | {mf:.2f} | {lc:.2f} | {gbs:,.0f} | `{short(name)}` |")
    text = "\n".join(lines) + "\n"
    if out:
        open(out, "w").write(text)
    print(text)


if __name__ == "__main__":
    a = sys.argv[1:]
    main(a[0], a[1], a[2], int(a[3]) if len(a) > 3 else 25, a[4] if len(a) > 4 else None)
