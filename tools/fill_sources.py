"""Which HIP runtime calls launch the vendor fill / copy kernels (``__amd_rocclr_fillBuffer*`` /
``__amd_rocclr_copyBuffer*``) of a run: joins a rocprofv3 kernel trace with its HIP API trace on the
correlation id.

    rocprofv3 --hip-trace --kernel-trace --output-format csv -d OUT -o run -- python ...
    python tools/fill_sources.py OUT
"""
import collections
import csv
import glob
import os
import sys


def main(d):
    kt = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    ht = glob.glob(os.path.join(d, "**", "*hip_api_trace.csv"), recursive=True)[0]
    api = {}
    for r in csv.DictReader(open(ht)):
        api[r.get("Correlation_Id")] = r.get("Function") or r.get("Operation") or "?"
    cnt = collections.Counter()
    for r in csv.DictReader(open(kt)):
        name = r["Kernel_Name"]
        if "rocclr" in name:
            cnt[(name[:40], api.get(r.get("Correlation_Id"), "?"))] += 1
    for (k, f), n in cnt.most_common():
        print(f"{n:6d}  {k:40s}  {f}")


if __name__ == "__main__":
    main(sys.argv[1])
