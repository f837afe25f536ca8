"""Per-kernel register / scratch / occupancy table of a HIP source compiled for gfx950.

    python tools/kernel_resources.py csrc/kernels/gemm_conv.hip [--filter wide]

Runs hipcc's device-only compile with ``-Rpass-analysis=kernel-resource-usage`` and condenses the
remarks — the quick check that an epilogue change did not push a kernel into scratch spills.
"""
import argparse
import os
import re
import subprocess
import tempfile


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("src")
    ap.add_argument("--filter", default="")
    a = ap.parse_args()
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    with tempfile.TemporaryDirectory() as td:
        r = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
                            f"-I{root}/csrc/include", "--offload-device-only",
                            "-Rpass-analysis=kernel-resource-usage", "-c", a.src, "-o", os.path.join(td, "k.o")],
                           capture_output=True, text=True)
    rows, cur = [], None
    for line in r.stderr.splitlines():
        m = re.search(r"remark: \s*(.+?): (\S+) \[-Rpass", line)
        if not m:
            continue
        k, v = m.group(1).strip(), m.group(2).strip()
        if k == "Function Name":
            cur = {"name": subprocess.run(["c++filt"], input=v, capture_output=True, text=True).stdout.strip()}
            rows.append(cur)
        elif cur is not None:
            cur[k] = v
    for c in rows:
        n = re.sub(r"pda::\(anonymous namespace\)::", "", c["name"])
        if a.filter in n:
            print(f"{c.get('VGPRs', '?'):>4} {c.get('AGPRs', '?'):>4} scratch={c.get('ScratchSize [bytes/lane]', '?'):>4}"
                  f" occ={c.get('Occupancy [waves/SIMD]', '?'):>2}  {n[:150]}")
    if r.returncode:
        print(r.stderr[-2000:])


if __name__ == "__main__":
    main()
