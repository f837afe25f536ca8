"""Collective consistency checker — ``PDA_DEBUG=collectives`` (the analogue of torch's
``TORCH_DISTRIBUTED_DEBUG=DETAIL``).  The reference has no race or mismatch detection at all; a rank
that issues a different collective (other op, dtype or size, or one collective too few) leaves RCCL
hanging or silently reducing garbage.

When enabled, every collective of ``torch.distributed`` is preceded by a fingerprint exchange over
the rendezvous store: each member of the group publishes ``(seq, op, dtype, numel/shape, root,
call site)`` under ``pda_dbg/<group>/<seq>/<rank>`` and reads every peer's.  Any difference raises
:class:`CollectiveMismatchError` on every rank with a per-rank table, *before* the collective is
issued; a peer that never arrives shows up as a store timeout naming the missing rank and the
collective it was expected to join.
"""
from __future__ import annotations

import functools
import json
import os
import traceback
from datetime import timedelta
from typing import Dict, List, Optional

import torch
import torch.distributed as dist

_OPS = ("all_reduce", "broadcast", "all_gather", "all_gather_into_tensor", "reduce_scatter",
        "reduce_scatter_tensor", "reduce", "gather", "scatter", "all_to_all_single", "all_to_all", "barrier")


class CollectiveMismatchError(RuntimeError):
    pass


def _describe(x):
    if isinstance(x, torch.Tensor):
        return {"dtype": str(x.dtype).replace("torch.", ""), "shape": list(x.shape), "dev": x.device.type}
    if isinstance(x, (list, tuple)) and x and isinstance(x[0], torch.Tensor):
        return {"list": len(x), **_describe(x[0])}
    return None


def _call_site() -> str:
    for fr in reversed(traceback.extract_stack()[:-3]):
        f = fr.filename
        if "torch/distributed" in f or f.endswith("parallel/debug.py"):
            continue
        return f"{os.path.basename(f)}:{fr.lineno}"
    return "?"


class CollectiveChecker:
    def __init__(self, store=None, timeout_s: float = 300.0):
        self.store = store
        self.timeout_s = timeout_s
        self.seq: Dict[str, int] = {}
        self.checked = 0
        self._orig: Dict[str, object] = {}

    # ------------------------------------------------------------------ fingerprints
    def _store(self):
        if self.store is None:
            self.store = dist.distributed_c10d._get_default_store()
        return self.store

    @staticmethod
    def _group_ranks(group) -> List[int]:
        if group is None or group is dist.group.WORLD:
            return list(range(dist.get_world_size()))
        return sorted(dist.get_process_group_ranks(group))

    def fingerprint(self, op: str, args, kwargs) -> dict:
        tensors = [a for a in args if isinstance(a, (torch.Tensor, list, tuple))]
        fp = {"op": op, "tensors": [_describe(t) for t in tensors[:2]]}
        for key in ("op", "src", "dst"):
            v = kwargs.get(key)
            if v is not None:
                fp["arg_" + key] = str(v)
        if op in ("broadcast", "reduce") and len(args) > 1 and isinstance(args[1], int):
            fp["root"] = args[1]
        if op == "all_reduce" and len(args) > 1 and not isinstance(args[1], torch.Tensor):
            fp["arg_op"] = str(args[1])
        return fp

    @staticmethod
    def _comparable(fp: dict) -> dict:
        # the list length of an all_gather output and the device kind must agree; call sites may differ
        return {k: v for k, v in fp.items() if k not in ("site", "rank")}

    def check(self, op: str, args, kwargs):
        group = kwargs.get("group")
        ranks = self._group_ranks(group)
        if len(ranks) <= 1:
            return
        me = dist.get_rank()
        gid = "-".join(map(str, ranks)) if len(ranks) < 16 else f"{ranks[0]}..{ranks[-1]}x{len(ranks)}"
        seq = self.seq.get(gid, 0) + 1
        self.seq[gid] = seq
        fp = self.fingerprint(op, args, kwargs)
        fp["seq"] = seq
        mine = dict(fp, rank=me, site=_call_site())
        store = self._store()
        base = f"pda_dbg/{gid}/{seq}/"
        store.set(base + str(me), json.dumps(mine))
        peers = {}
        for r in ranks:
            try:
                store.wait([base + str(r)], timedelta(seconds=self.timeout_s))
                peers[r] = json.loads(store.get(base + str(r)))
            except Exception as e:  # noqa: BLE001
                raise CollectiveMismatchError(
                    f"rank {me}: rank {r} did not reach collective #{seq} of group [{gid}] "
                    f"({op} at {mine['site']}) within {self.timeout_s:.0f}s: {type(e).__name__}") from None
        ref = self._comparable(mine)
        bad = [r for r, p in peers.items() if self._comparable(p) != ref]
        if bad:
            lines = [f"collective mismatch at #{seq} of group [{gid}] (seen on rank {me}):"]
            for r in ranks:
                p = peers[r]
                lines.append(f"  rank {r}: {p['op']} {p.get('tensors')} "
                             f"{ {k: v for k, v in p.items() if k.startswith('arg_') or k == 'root'} } at {p['site']}")
            raise CollectiveMismatchError("\n".join(lines))
        if seq > 2:  # keep the store small: our key of two collectives ago is no longer read by anyone
            try:
                store.delete_key(f"pda_dbg/{gid}/{seq - 2}/{me}")
            except Exception:  # noqa: BLE001
                pass
        self.checked += 1

    # ------------------------------------------------------------------ patching
    def enable(self):
        for name in _OPS:
            fn = getattr(dist, name, None)
            if fn is None or name in self._orig:
                continue
            self._orig[name] = fn

            def make(name, fn):
                @functools.wraps(fn)
                def wrapper(*args, **kwargs):
                    self.check(name, args, kwargs)
                    return fn(*args, **kwargs)
                return wrapper
            setattr(dist, name, make(name, fn))
        return self

    def disable(self):
        for name, fn in self._orig.items():
            setattr(dist, name, fn)
        self._orig.clear()


_CHECKER: Optional[CollectiveChecker] = None


def enabled_by_env() -> bool:
    flags = [s.strip().lower() for s in os.environ.get("PDA_DEBUG", "").split(",")]
    return "collectives" in flags or os.environ.get("PDA_DEBUG_COLLECTIVES", "0").lower() in ("1", "true", "yes")


def enable_collective_checks(store=None, timeout_s: float = 300.0) -> CollectiveChecker:
    global _CHECKER
    if _CHECKER is None:
        _CHECKER = CollectiveChecker(store, timeout_s).enable()
    return _CHECKER


def disable_collective_checks():
    global _CHECKER
    if _CHECKER is not None:
        _CHECKER.disable()
    _CHECKER = None


def maybe_enable(store=None):
    if enabled_by_env():
        return enable_collective_checks(store)
    return None
