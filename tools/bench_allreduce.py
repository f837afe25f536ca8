"""All-reduce bandwidth sweep over bucket sizes: RCCL (torch.distributed
"nccl") vs the one-shot, two-shot and ring xGMI IPC kernels (with the copy into the exchange buffer) and
the zero-copy two-shot / ring on a registered buffer (the DDP bucket path), bf16, per size: time,
algorithm bandwidth and bus bandwidth (2(N-1)/N x bytes / time).  ``--gloo`` rehearses the sweep with
several ranks on one GPU (gloo carries the control plane; no RCCL column).  ``--write-table PATH`` (default: the per-node location
``parallel.xgmi.default_table_path``) stores the per-size winner of RCCL / one-shot / two-shot as the
crossover table that ``PDA_ALLREDUCE=ipc`` (DDP buckets) then follows.  Run on one node:

    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 tools/bench_allreduce.py --write-table
"""
import argparse
import json
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pytorchdistributed_amd.distributed as pd  # noqa: E402
from pytorchdistributed_amd.parallel.xgmi import XgmiAllReduce, default_table_path, table_from_sweep  # noqa: E402

SIZES_MB = [0.25, 1, 2, 4, 8, 16, 32, 64, 128]


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    dist.barrier()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    ms = torch.tensor([s.elapsed_time(e) / iters], device="cuda")
    dist.all_reduce(ms, op=dist.ReduceOp.MAX)
    return ms.item()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--write-table", nargs="?", const="", default=None,
                    help="write the RCCL / one-shot / two-shot crossover table (optional path)")
    ap.add_argument("--gloo", action="store_true", help="one-GPU rehearsal: ranks share cuda:0, no RCCL column")
    ap.add_argument("--sizes", default="", help="comma-separated MB sizes (default: the full sweep)")
    ap.add_argument("--only", default="", help="comma-separated arm names to run (default: all)")
    args = ap.parse_args()
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gloo:
        torch.cuda.set_device(0)
        pd.init_process_group("gloo")
    else:
        torch.cuda.set_device(local)
        pd.init_process_group("nccl", device_id=local)
    world, rank = dist.get_world_size(), dist.get_rank()
    sizes = [float(v) for v in args.sizes.split(",")] if args.sizes else SIZES_MB
    xg = XgmiAllReduce(capacity_mb=max(sizes) + 1)
    flat = torch.randn(int(max(sizes) * 2 ** 20 / 2) // 8 * 8, device="cuda", dtype=torch.bfloat16)
    reg = xg.register(flat)  # zero-copy: a registered flat buffer, buckets are slices of it
    records = []
    for mb in sizes:
        n = int(mb * 2 ** 20 / 2) // 8 * 8
        t = torch.randn(n, device="cuda", dtype=torch.bfloat16)
        rec = {"size_mb": mb, "world": world}
        arms = [] if args.gloo else [("rccl", lambda: dist.all_reduce(t))]
        arms += [("xgmi_oneshot", lambda: xg(t, algo="oneshot")), ("xgmi_twoshot", lambda: xg(t, algo="twoshot")),
                 ("xgmi_ring", lambda: xg(t, algo="ring")),
                 ("xgmi_zc_twoshot", lambda: xg.all_reduce_registered(reg, flat[:n], 0, algo="twoshot")),
                 ("xgmi_zc_ring", lambda: xg.all_reduce_registered(reg, flat[:n], 0, algo="ring"))]
        if args.only:
            arms = [a for a in arms if a[0] in args.only.split(",")]
        for name, fn in arms:
            ms = timeit(fn)
            alg = n * 2 / (ms * 1e-3) / 1e9
            rec[name] = {"ms": round(ms, 4), "alg_GBps": round(alg, 1),
                         "bus_GBps": round(alg * 2 * (world - 1) / world, 1)}
        records.append(rec)
        if rank == 0:
            print(json.dumps(rec), flush=True)
    xg.check()
    if args.write_table is not None and rank == 0 and not args.gloo:
        path = args.write_table or default_table_path(world)
        os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        with open(path, "w") as f:
            json.dump(table_from_sweep(records, world), f, indent=1)
        print(f"crossover table -> {path}", flush=True)
    pd.destroy_process_group()


if __name__ == "__main__":
    main()
