"""``pda-run``: torchrun-compatible launcher (reference transcript
`02_ddp.ipynb` cell "!torchrun --nproc-per-node=2 --master_port=12355 ddp_gpus_torchrun.py ...").

    python -m pytorchdistributed_amd.run --nproc-per-node=2 --master-port=12355 train.py --max_epochs 5

Accepts both ``--nproc-per-node`` and ``--nproc_per_node`` spellings, ``--nnodes``, ``--node-rank``,
``--master-addr``, ``--master-port``, ``--standalone``, ``--max-restarts``, plus ``--profile-dir``
(per-rank rocprofv3 kernel traces), ``--metrics-dir``, ``--debug-collectives`` and
``--collective-timeout``.  Node 0's launcher hosts the
native rendezvous store; workers get the torchrun env contract.  On the first non-zero worker exit
the launcher SIGTERMs the whole local group (SIGKILL after ``--grace`` seconds) and, with
``--max-restarts N``, relaunches it (workers resume from their latest snapshot, see
:class:`pytorchdistributed_amd.train.Trainer`).
"""
from __future__ import annotations

import argparse
import sys

from .distributed import free_port
from .launch import run_workers


def _parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(prog="pda-run", description=__doc__, formatter_class=argparse.RawTextHelpFormatter)
    p.add_argument("--nproc-per-node", "--nproc_per_node", type=int, default=1)
    p.add_argument("--nnodes", type=int, default=1)
    p.add_argument("--node-rank", "--node_rank", type=int, default=0)
    p.add_argument("--master-addr", "--master_addr", default="127.0.0.1")
    p.add_argument("--master-port", "--master_port", type=int, default=29500)
    p.add_argument("--standalone", action="store_true", help="single node, pick a free port")
    p.add_argument("--max-restarts", "--max_restarts", type=int, default=0)
    p.add_argument("--monitor-interval", "--monitor_interval", type=float, default=0.1)
    p.add_argument("--grace", type=float, default=10.0, help="seconds between SIGTERM and SIGKILL on teardown")
    p.add_argument("-m", "--module", action="store_true", help="run the target as a python module")
    p.add_argument("--profile-dir", default=None, help="wrap each rank in rocprofv3 --kernel-trace --stats")
    p.add_argument("--metrics-dir", default=None, help="per-rank metrics JSONL directory (PDA_METRICS_DIR)")
    p.add_argument("--debug-collectives", action="store_true", help="PDA_DEBUG=collectives fingerprint checks")
    p.add_argument("--collective-timeout", type=float, default=None, help="watchdog deadline per collective (s)")
    p.add_argument("script")
    p.add_argument("script_args", nargs=argparse.REMAINDER)
    return p


def main(argv=None) -> int:
    a = _parser().parse_args(argv)
    if a.standalone:
        a.nnodes, a.node_rank, a.master_addr, a.master_port = 1, 0, "127.0.0.1", free_port()
    cmd = [sys.executable] + (["-m", a.script] if a.module else [a.script]) + list(a.script_args)
    extra = {}
    if a.metrics_dir:
        extra["PDA_METRICS_DIR"] = a.metrics_dir
    if a.debug_collectives:
        extra["PDA_DEBUG"] = "collectives"
    if a.collective_timeout:
        extra["PDA_COLLECTIVE_TIMEOUT_S"] = str(a.collective_timeout)
    return run_workers(cmd, a.nproc_per_node, a.nnodes, a.node_rank, a.master_addr, a.master_port,
                       a.max_restarts, a.monitor_interval, extra_env=extra or None, grace=a.grace,
                       profile_dir=a.profile_dir)


if __name__ == "__main__":
    sys.exit(main())
