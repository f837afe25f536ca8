"""Process launchers.

* :func:`spawn` — ``mp.spawn``-compatible (reference `ddp_gpus.py:98`
  ``mp.spawn(main, args=(world_size, ...), nprocs=world_size)``): calls ``fn(rank, *args)`` in
  ``nprocs`` fresh interpreters.  The parent hosts the native C++ rendezvous store, exports the
  torchrun env contract (RANK / LOCAL_RANK / WORLD_SIZE / LOCAL_WORLD_SIZE / MASTER_ADDR / MASTER_PORT)
  to every child, watches them, tears the whole group down on the first failure and re-raises the
  child's exception with its traceback.
* :func:`run_workers` — the engine behind the ``pda-run`` CLI (:mod:`.run`).
"""
from __future__ import annotations

import multiprocessing as mp
import os
import signal
import subprocess
import sys
import time
import traceback
from typing import Callable, Dict, List, Optional, Sequence

from . import distributed as pdist


class ProcessRaisedException(RuntimeError):
    def __init__(self, msg: str, rank: int, exitcode: Optional[int] = None):
        super().__init__(msg)
        self.rank = rank
        self.exitcode = exitcode


def _child(fn, rank: int, args: tuple, env: Dict[str, str], errq):
    os.environ.update(env)
    import faulthandler

    faulthandler.enable()  # a worker that dies on a signal leaves its Python stack on stderr
    try:
        fn(rank, *args)
    except KeyboardInterrupt:
        sys.exit(130)
    except BaseException:  # noqa: BLE001 - forwarded to the parent
        errq.put((rank, traceback.format_exc()))
        sys.exit(1)


def worker_env(rank: int, local_rank: int, world: int, local_world: int, master_addr: str, master_port: int,
               node_rank: int = 0, hosted: bool = True) -> Dict[str, str]:
    env = {
        "RANK": str(rank),
        "LOCAL_RANK": str(local_rank),
        "WORLD_SIZE": str(world),
        "LOCAL_WORLD_SIZE": str(local_world),
        "GROUP_RANK": str(node_rank),
        "MASTER_ADDR": master_addr,
        "MASTER_PORT": str(master_port),
    }
    if hosted:
        env["PDA_STORE_HOSTED"] = "1"
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
    return env


def _terminate(procs, grace: float = 5.0):
    for p in procs:
        if p.is_alive():
            p.terminate()
    deadline = time.time() + grace
    for p in procs:
        p.join(max(0.0, deadline - time.time()))
    for p in procs:
        if p.is_alive():
            p.kill()
            p.join()


def spawn(fn: Callable, args: Sequence = (), nprocs: int = 1, join: bool = True, master_addr: str = "127.0.0.1",
          master_port: Optional[int] = None, timeout: Optional[float] = None):
    """Run ``fn(rank, *args)`` in ``nprocs`` processes with a framework-hosted rendezvous store."""
    ctx = mp.get_context("spawn")
    server = pdist.start_store_server("0.0.0.0", master_port or 0)
    port = server.port
    errq = ctx.SimpleQueue()
    procs = []
    try:
        for r in range(nprocs):
            env = worker_env(r, r, nprocs, nprocs, master_addr, port)
            p = ctx.Process(target=_child, args=(fn, r, tuple(args), env, errq), daemon=False)
            p.start()
            procs.append(p)
        if not join:
            return procs, server
        t0 = time.time()
        while True:
            alive = [p for p in procs if p.is_alive()]
            failed = [(i, p) for i, p in enumerate(procs) if not p.is_alive() and p.exitcode not in (0, None)]
            if failed:
                rank, p = failed[0]
                _terminate(procs)
                msg = f"process {rank} terminated with exit code {p.exitcode}"
                while not errq.empty():
                    r, tb = errq.get()
                    if r == rank or "Traceback" in tb:
                        msg = f"-- process {r} terminated with the following error:\n{tb}"
                        rank = r
                        break
                raise ProcessRaisedException(msg, rank, p.exitcode)
            if not alive:
                return None
            if timeout is not None and time.time() - t0 > timeout:
                _terminate(procs)
                raise TimeoutError(f"spawn: workers did not finish within {timeout}s")
            time.sleep(0.05)
    finally:
        if join:
            server.stop()


def run_workers(cmd: List[str], nproc_per_node: int, nnodes: int = 1, node_rank: int = 0,
                master_addr: str = "127.0.0.1", master_port: int = 29500, max_restarts: int = 0,
                monitor_interval: float = 0.1, extra_env: Optional[Dict[str, str]] = None,
                grace: float = 10.0, profile_dir: Optional[str] = None) -> int:
    """Launch ``cmd`` once per local rank, supervise, tear down on failure; returns the exit code.

    ``profile_dir``: wrap every rank in ``rocprofv3 --kernel-trace --stats`` writing
    ``<profile_dir>/rank<r>/`` (the program itself follows ``--``)."""
    server = None
    if node_rank == 0:
        server = pdist.start_store_server("0.0.0.0", master_port)
        master_port = server.port  # master_port=0: the store picked a free port
    world = nproc_per_node * nnodes
    if "OMP_NUM_THREADS" not in os.environ and nproc_per_node > 1:
        sys.stderr.write(
            "*****************************************\n"
            "Setting OMP_NUM_THREADS environment variable for each process to be 1 in default, to avoid your "
            "system being overloaded, please further tune the variable for optimal performance in your "
            "application as needed.\n*****************************************\n")
    attempt = 0
    try:
        while True:
            procs = []
            for lr in range(nproc_per_node):
                env = dict(os.environ)
                env.setdefault("OMP_NUM_THREADS", "1")
                env.update(worker_env(node_rank * nproc_per_node + lr, lr, world, nproc_per_node, master_addr,
                                      master_port, node_rank))
                env["PDA_RESTART_COUNT"] = str(attempt)
                env["TORCHELASTIC_RESTART_COUNT"] = str(attempt)
                if extra_env:
                    env.update(extra_env)
                rcmd = cmd
                if profile_dir:
                    rank = node_rank * nproc_per_node + lr
                    rcmd = ["rocprofv3", "--kernel-trace", "--stats", "-d", os.path.join(profile_dir, f"rank{rank}"),
                            "-o", "trace", "--output-format", "csv", "--"] + list(cmd)
                procs.append(subprocess.Popen(rcmd, env=env, start_new_session=True))
            rc = _supervise(procs, monitor_interval, grace)
            if rc == 0:
                return 0
            if attempt >= max_restarts:
                return rc
            attempt += 1
            sys.stderr.write(f"[pda-run] worker group failed (rc={rc}); restart {attempt}/{max_restarts}\n")
    finally:
        if server is not None:
            server.stop()


def _supervise(procs: List[subprocess.Popen], interval: float, grace: float) -> int:
    try:
        while True:
            codes = [p.poll() for p in procs]
            bad = [c for c in codes if c not in (None, 0)]
            if bad:
                _kill_group(procs, grace)
                return bad[0]
            if all(c == 0 for c in codes):
                return 0
            time.sleep(interval)
    except KeyboardInterrupt:
        _kill_group(procs, grace)
        return 130


def _kill_group(procs: List[subprocess.Popen], grace: float):
    for p in procs:
        if p.poll() is None:
            try:
                os.killpg(p.pid, signal.SIGTERM)
            except ProcessLookupError:
                pass
    deadline = time.time() + grace
    for p in procs:
        try:
            p.wait(timeout=max(0.0, deadline - time.time()))
        except subprocess.TimeoutExpired:
            try:
                os.killpg(p.pid, signal.SIGKILL)
            except ProcessLookupError:
                pass
            p.wait()
