"""Where a kernel's scratch traffic and full vmcnt drains sit relative to its loops, from a device
assembly listing (``hipcc --offload-arch=gfx950 --cuda-device-only -S -o k.s src.hip``).

    python tools/asm_loops.py k.s [name-substring ...]

For each matching kernel prints its length, each loop (backward branch target .. branch), the scratch
instructions and ``s_waitcnt vmcnt(0)`` lines inside every loop — the check that a register-pressure
change kept the main loop clean (cdna_hip_programming.md: spills outside the steady state are cheap,
inside it they serialise the pipeline).  Only loops that issue MFMAs are listed.
"""
import re
import sys


def main():
    path, subs = sys.argv[1], sys.argv[2:]
    lines = open(path).read().split("\n")
    starts = [(i, l.split(":")[0]) for i, l in enumerate(lines) if re.match(r"^_Z\w+:", l)]
    for k, (i, name) in enumerate(starts):
        if subs and not all(s in name for s in subs):
            continue
        end = starts[k + 1][0] if k + 1 < len(starts) else len(lines)
        body = lines[i:end]
        labels = {}
        for j, l in enumerate(body):
            m = re.match(r"^(\.LBB\w+):", l)
            if m:
                labels[m.group(1)] = j
        loops = []
        for j, l in enumerate(body):
            m = re.search(r"s_(?:cbranch_\w+|branch)\s+(\.LBB\w+)", l)
            if m and m.group(1) in labels and labels[m.group(1)] < j:
                loops.append((labels[m.group(1)], j))
        scratch = [j for j, l in enumerate(body) if "scratch_" in l]
        print(f"{name}: {len(body)} lines, {len(scratch)} scratch ops")
        for (a, b) in loops:
            inner = [j for j in scratch if a <= j <= b]
            drains = [j for j in range(a, b + 1) if "vmcnt(0)" in body[j]]
            mfma = sum(1 for j in range(a, b + 1) if "v_mfma" in body[j])
            if not mfma:
                continue  # epilogue / copy loops
            print(f"  loop {a}..{b}: {mfma} mfma, {len(inner)} scratch {inner[:8]}, vmcnt(0) at {drains[:8]}")


if __name__ == "__main__":
    main()
