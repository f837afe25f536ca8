"""Aggregate a rocprofv3 --pmc counter_collection.csv per kernel (last dispatch of each kernel name)
and print counters plus per-wave / per-MFMA ratios."""
import collections
import csv
import sys


def main(path, match=""):
    rows = list(csv.DictReader(open(path)))
    per = collections.OrderedDict()
    for r in rows:
        name = r["Kernel_Name"]
        if match and match not in name:
            continue
        d = per.setdefault(name, {}).setdefault(r["Dispatch_Id"], collections.defaultdict(float))
        d[r["Counter_Name"]] += float(r["Counter_Value"])
        d["_vgpr"] = float(r.get("VGPR_Count") or 0)
        d["_agpr"] = float(r.get("Accum_VGPR_Count") or 0)
        d["_lds"] = float(r.get("LDS_Block_Size") or 0)
    for name, disp in per.items():
        last = list(disp.values())[-1]
        print(name[:120])
        for k in sorted(last):
            print(f"   {k:32s} {last[k]:,.0f}")
        mf = last.get("SQ_INSTS_VALU_MFMA_BF16") or last.get("SQ_INSTS_MFMA")
        if mf:
            for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM", "SQ_INSTS_SMEM"):
                if k in last:
                    print(f"   {k + ' per MFMA':32s} {last[k] / mf:.2f}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "")
