"""Shared benchmark plumbing: distributed setup from the torchrun / pda-run env contract and the
timed-window protocol (barrier + synchronize on both sides, MAX over ranks)."""
from __future__ import annotations

import datetime
import json
import os
import sys

import torch
import torch.distributed as dist

from .. import distributed as pdist
from ..utils.timing import StepTimer


_FORCE_ENVS = ("PDA_DDP_FORCE_COMM", "PDA_FSDP_FORCE_COMM", "PDA_PP_FORCE_COMM")


def _self_command() -> list:
    """The command line that re-runs this benchmark in a worker (``-m module`` or the script path)."""
    main = sys.modules.get("__main__")
    spec = getattr(main, "__spec__", None)
    if spec is not None and spec.name and spec.name != "__main__":
        return [sys.executable, "-u", "-m", spec.name] + sys.argv[1:]
    return [sys.executable, "-u", os.path.abspath(sys.argv[0])] + sys.argv[1:]


def launch_ranks(n_gpus: int) -> None:
    """``--gpus N`` without a launcher: start N ranks of this same command and exit with their code.

    The reference's scripts launch one process per GPU themselves (`02 DDP基本概念/ddp_gpus.py:94-98`,
    ``mp.spawn(main, nprocs=world_size)``); so does every benchmark here.  Runs in the parent before
    anything touches the GPU (no HIP call is made in this process): the framework's launcher
    (:func:`..launch.run_workers`) hosts the native rendezvous store on a free port, exports the
    torchrun env contract (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 / MASTER_PORT) to
    each worker, supervises them and tears the group down on the first failure.  Rank 0 prints the
    JSON line on the inherited stdout; the exit code is the first failing rank's (0 if all succeed).
    """
    from ..launch import run_workers

    env = {"PDA_BENCH_LAUNCHED": "1"}
    rc = run_workers(_self_command(), nproc_per_node=n_gpus, master_addr="127.0.0.1", master_port=0,
                     extra_env=env)
    if rc != 0:
        sys.stderr.write(f"[bench] a rank of the {n_gpus}-rank run failed (exit code {rc})\n")
    sys.exit(rc)


def _verify_group(n_gpus: int, backend: str, device) -> None:
    """Every rank checks the live group: size == --gpus and (RCCL) one distinct GPU per rank."""
    world = dist.get_world_size()
    if world != n_gpus:
        raise SystemExit(f"--gpus {n_gpus} but the process group has {world} rank(s)")
    if world == 1:
        return
    on = device if backend == "nccl" else torch.device("cpu")
    mine = torch.tensor([device.index if device.type == "cuda" else -1], dtype=torch.int64, device=on)
    every = [torch.zeros_like(mine) for _ in range(world)]
    dist.all_gather(every, mine)
    idx = [int(t.item()) for t in every]
    if backend == "nccl" and len(set(idx)) != world:
        raise SystemExit(f"RCCL ranks must own distinct GPUs, got device indices {idx}")


def group_info(device) -> dict:
    """Facts about the live group for the JSON line (the driver checks n_gpus against them)."""
    if not dist.is_initialized():
        return {"world": 1, "backend": None, "rccl_world": 0}
    b = dist.get_backend()
    return {"world": dist.get_world_size(), "backend": b, "rccl_world": dist.get_world_size() if b == "nccl" else 0}


def setup(n_gpus: int, one_rank_group: bool = False):
    """Rank / world / local rank / device from the env contract; initialises the default group.

    Without a launcher (``WORLD_SIZE`` unset) and ``n_gpus > 1`` this process becomes the launcher:
    :func:`launch_ranks` starts ``n_gpus`` ranks of the same command and never returns.

    ``PDA_DIST_BACKEND`` overrides the backend (default ``nccl`` = RCCL on a GPU, ``gloo`` on CPU).
    Rehearsal mode: with ``PDA_DIST_BACKEND=gloo`` more ranks than GPUs may share the visible GPUs
    (rank r on GPU r % count) — the whole multi-rank DDP path (hooks, buckets, collectives, timing
    protocol) runs on the native kernels of a one-GPU box; RCCL itself refuses two ranks per GPU.
    """
    # a hung collective must end the run with stacks and an ncclCommAbort well inside the driver's own
    # limit on a benchmark (600 s): the collective watchdog fires at 180 s, c10d's own timeout at 300 s
    if "PDA_COLLECTIVE_TIMEOUT_S" not in os.environ:
        os.environ["PDA_COLLECTIVE_TIMEOUT_S"] = "180"
        from .. import config as _config

        _config.set_config(None)  # re-resolve if an earlier import already loaded the config
    os.environ.setdefault("PDA_TRACK_COMM", "1")
    if n_gpus > 1 and "WORLD_SIZE" not in os.environ:
        launch_ranks(n_gpus)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if n_gpus != world:
        raise SystemExit(f"--gpus {n_gpus} but WORLD_SIZE={world} (refusing to run a different rank count)")
    use_gpu = torch.cuda.is_available()
    backend = os.environ.get("PDA_DIST_BACKEND", "nccl" if use_gpu else "gloo")
    gpu = local
    if use_gpu:
        count = torch.cuda.device_count()
        if local >= count:
            if backend == "nccl":
                raise SystemExit(f"LOCAL_RANK {local} but only {count} GPU(s) visible (RCCL needs one GPU per "
                                 f"rank; PDA_DIST_BACKEND=gloo rehearses with shared GPUs)")
            gpu = local % count
        torch.cuda.set_device(gpu)
    # PDA_DDP_FORCE_COMM=1 at N=1: a one-rank RCCL group, so the bucket all-reduces of the multi-GPU
    # path run (and are timed) on a single GPU
    # (``one_rank_group``: the headline bench defaults to it, so N=1 times the same DDP path as N>1)
    if one_rank_group and use_gpu:
        os.environ.setdefault("PDA_DDP_FORCE_COMM", "1")
    # (PDA_FSDP_FORCE_COMM / PDA_PP_FORCE_COMM likewise run FSDP's and the pipeline's collectives over it)
    force = any(os.environ.get(k) == "1" for k in _FORCE_ENVS) and use_gpu and backend == "nccl"
    if (world > 1 or force) and not dist.is_initialized():
        pdist.init_process_group(backend, rank=rank, world_size=world,
                                 device_id=gpu if use_gpu and backend == "nccl" else None,
                                 timeout=datetime.timedelta(seconds=_c10d_timeout_s()))
    device = torch.device("cuda", gpu) if use_gpu else torch.device("cpu")
    if dist.is_initialized():
        _verify_group(n_gpus, backend, device)
    return rank, world, local, device


def _c10d_timeout_s() -> float:
    return float(os.environ.get("PDA_BENCH_C10D_TIMEOUT_S", "300"))


def timed(step_fn, steps: int, warmup: int, on_start=None) -> float:
    """Run ``warmup`` untimed steps, then time exactly ``steps``; returns max-over-ranks seconds.
    ``on_start`` runs between the two (e.g. resetting communication counters)."""
    for _ in range(warmup):
        step_fn()
    if on_start is not None:
        on_start()
    t = StepTimer()
    t.start()
    for _ in range(steps):
        step_fn()
    secs = t.stop()
    return t.max_over_ranks(secs)


def comm_record(mod, steps: int) -> dict:
    """Per-step communication figures of a DDP / FSDP module for the JSON line: bytes and
    collective calls per step, and — tracking on (PDA_TRACK_COMM, default 1 in the benchmarks) — the
    compute-stream time per step spent waiting on the collectives (``exposed_comm_ms``), so a multi-GPU
    run separates exposed communication from kernel slowdown."""
    if mod is None or not hasattr(mod, "comm_stats"):
        return {}
    st = mod.comm_stats(reset=True)
    out = {"comm_mb_per_step": round(st.get("comm_bytes", 0) / 2 ** 20 / max(steps, 1), 2),
           "comm_calls_per_step": round(st.get("comm_calls", 0) / max(steps, 1), 2)}
    if "exposed_comm_ms" in st:
        out["exposed_comm_ms_per_step"] = round(st["exposed_comm_ms"] / max(steps, 1), 3)
    return out


def mem_record(device) -> dict:
    """Caching-allocator figures for the JSON line: peak allocated / reserved GiB and the number of
    allocation retries (a retry frees the cache and synchronises the device: a step that needs them
    is allocator-bound, not compute- or comm-bound)."""
    if device is None or getattr(device, "type", "cpu") != "cuda":
        return {}
    st = torch.cuda.memory_stats(device)
    gib = 2 ** 30
    return {"peak_alloc_gib": round(st.get("allocated_bytes.all.peak", 0) / gib, 1),
            "peak_reserved_gib": round(st.get("reserved_bytes.all.peak", 0) / gib, 1),
            "alloc_retries": int(st.get("num_alloc_retries", 0))}


def emit(record: dict, rank: int):
    if rank == 0:
        print(json.dumps(record), flush=True)


def teardown():
    if dist.is_initialized():
        pdist.destroy_process_group()
