"""Which Python lines launch a benchmark's housekeeping kernels (fills, copies, casts): runs a bench
module's main() under a TorchDispatchMode that records, for every matching aten op on a GPU tensor, the
innermost framework frames of the Python stack, and prints the calls / bytes per call site.

    python tools/op_attrib.py pytorchdistributed_amd.bench.llama_fsdp --steps 2 --warmup 1 \
        [--ops fill_,copy_,zero_,_to_copy,zeros,new_zeros] [--top 20]
"""
import argparse
import collections
import importlib
import os
import sys
import traceback

import torch
from torch.utils._python_dispatch import TorchDispatchMode

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


class _Rec(TorchDispatchMode):
    def __init__(self, ops):
        super().__init__()
        self.ops = ops
        self.hits = collections.defaultdict(lambda: [0, 0])

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        out = func(*args, **(kwargs or {}))
        name = func._overloadpacket.__name__
        if name in self.ops:
            t = out if isinstance(out, torch.Tensor) else (args[0] if args and isinstance(args[0], torch.Tensor) else None)
            if t is not None and t.is_cuda:
                frames = [f for f in traceback.extract_stack()[:-1] if "pytorchdistributed_amd" in f.filename
                          and "_python_dispatch" not in f.filename]
                site = " <- ".join(f"{os.path.relpath(f.filename, ROOT)}:{f.lineno}" for f in frames[::-1][:4])
                h = self.hits[(name, str(t.dtype), site)]
                h[0] += 1
                h[1] += t.numel() * t.element_size()
        return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("module")
    ap.add_argument("--ops", default="fill_,copy_,zero_,_to_copy,zeros,new_zeros,zeros_like,clone")
    ap.add_argument("--top", type=int, default=20)
    a, rest = ap.parse_known_args()
    mod = importlib.import_module(a.module)
    rec = _Rec(set(a.ops.split(",")))
    # backward on the calling thread, so the mode also sees the ops autograd runs (a dispatch mode is
    # not active on the engine's device threads)
    with rec, torch.autograd.set_multithreading_enabled(False):
        mod.main(rest)
    rows = sorted(rec.hits.items(), key=lambda kv: -kv[1][1])
    for (name, dt, site), (n, b) in rows[: a.top]:
        print(f"{b / 2 ** 30:9.2f} GiB {n:6d} x {name:10s} {dt:15s} {site}")


if __name__ == "__main__":
    main()
