"""Typed configuration / flag system.

The reference configures itself with two argparse flags (``--max_epochs``, ``--batch_size``;
`02 DDP基本概念/ddp_gpus.py:86-98`, `ddp_gpus_torchrun.py:86-102`), the torchrun env contract
(``RANK``/``LOCAL_RANK``/``WORLD_SIZE``/``MASTER_ADDR``/``MASTER_PORT``) and notebook constants.
Those keep working unchanged; the framework's own knobs live in one dataclass resolved with the
precedence **CLI > environment (``PDA_*``) > config file (JSON/YAML) > defaults**.

    cfg = Config.load(argv)          # or Config.load(file="run.yaml")
    cfg.bucket_mb, cfg.allreduce, cfg.debug_collectives, ...

Every field maps to an env var ``PDA_<FIELD_UPPER>`` (e.g. ``bucket_mb`` <- ``PDA_BUCKET_MB``) and a
CLI flag ``--<field-with-dashes>``.
"""
from __future__ import annotations

import argparse
import dataclasses
import json
import os
from dataclasses import dataclass, field, fields
from typing import Any, Dict, List, Optional, Sequence

_CHOICES = {
    "allreduce": ("auto", "rccl", "ring", "host", "ipc", "oneshot", "twoshot"),
    "precision": ("bf16", "fp32"),
    "schedule": ("gpipe", "1f1b"),
}


@dataclass
class Config:
    # --- reference CLI flags (same names and defaults as ddp_gpus_torchrun.py)
    max_epochs: int = 10
    batch_size: int = 32
    save_every: int = 0
    snapshot_path: str = "snapshot.pt"
    # --- DDP communication (buckets sized for 7 xGMI links)
    bucket_mb: float = 32.0
    first_bucket_mb: float = 2.0
    allreduce: str = "auto"          # auto -> RCCL for device tensors, host ring for CPU tensors; oneshot/twoshot -> IPC xGMI kernels, ipc -> size-picked
    comm_priority: bool = True       # high-priority HIP stream for communication
    broadcast_buffers: bool = True
    # --- pipeline / FSDP
    split_size: int = 20
    num_microbatches: int = 0        # 0: derived from split_size
    schedule: str = "1f1b"
    recompute: bool = False
    fsdp_prefetch: bool = True
    # --- numerics
    precision: str = "bf16"
    # --- observability / robustness
    debug_collectives: bool = False  # PDA_DEBUG_COLLECTIVES=1: cross-rank fingerprint check per collective
    collective_timeout_s: float = 600.0
    watchdog: bool = True
    metrics_dir: str = ""            # per-rank metrics JSONL when set
    profile: bool = False
    log_rank0_only: bool = False
    extra: Dict[str, Any] = field(default_factory=dict)

    # ------------------------------------------------------------------ resolution
    @classmethod
    def env_name(cls, name: str) -> str:
        return "PDA_" + name.upper()

    @staticmethod
    def _coerce(tp, raw):
        if isinstance(raw, str):
            if tp in (bool, "bool"):
                return raw.strip().lower() in ("1", "true", "yes", "on")
            if tp in (int, "int"):
                return int(raw)
            if tp in (float, "float"):
                return float(raw)
        return raw

    @classmethod
    def _types(cls) -> Dict[str, Any]:
        return {f.name: f.type for f in fields(cls) if f.name != "extra"}

    @classmethod
    def from_file(cls, path: str) -> Dict[str, Any]:
        with open(path) as fh:
            text = fh.read()
        if path.endswith((".yaml", ".yml")):
            import yaml

            data = yaml.safe_load(text) or {}
        else:
            data = json.loads(text)
        if not isinstance(data, dict):
            raise ValueError(f"config file {path} must hold a mapping")
        return data

    @classmethod
    def add_arguments(cls, ap: argparse.ArgumentParser) -> argparse.ArgumentParser:
        for name, tp in cls._types().items():
            flag = "--" + name.replace("_", "-")
            alt = "--" + name  # the reference spells --max_epochs / --batch_size with underscores
            opts = [flag] if alt == flag else [flag, alt]
            kw: Dict[str, Any] = dict(dest=name, default=None)
            if tp in (bool, "bool"):
                kw["type"] = lambda s: s.strip().lower() in ("1", "true", "yes", "on")
                kw["nargs"] = "?"
                kw["const"] = True
            else:
                kw["type"] = {"int": int, "float": float}.get(tp if isinstance(tp, str) else tp.__name__, str)
            if name in _CHOICES:
                kw["choices"] = _CHOICES[name]
            ap.add_argument(*opts, **kw)
        ap.add_argument("--config", dest="config_file", default=None, help="JSON/YAML config file")
        return ap

    @classmethod
    def load(cls, argv: Optional[Sequence[str]] = None, file: Optional[str] = None,
             env: Optional[Dict[str, str]] = None, parse_known: bool = True) -> "Config":
        env = os.environ if env is None else env
        values: Dict[str, Any] = {}
        cli: Dict[str, Any] = {}
        if argv is not None:
            ap = cls.add_arguments(argparse.ArgumentParser(add_help=False))
            ns, _ = ap.parse_known_args(list(argv)) if parse_known else (ap.parse_args(list(argv)), None)
            cli = {k: v for k, v in vars(ns).items() if v is not None}
            file = cli.pop("config_file", None) or file
        file = file or env.get("PDA_CONFIG")
        types = cls._types()
        extra: Dict[str, Any] = {}
        if file:
            for k, v in cls.from_file(file).items():
                (values if k in types else extra)[k] = v
        for name, tp in types.items():
            ev = env.get(cls.env_name(name))
            if ev is not None and ev != "":
                values[name] = cls._coerce(tp, ev)
        values.update(cli)
        for name, tp in types.items():
            if name in values:
                values[name] = cls._coerce(tp, values[name])
        cfg = cls(**values)
        cfg.extra.update(extra)
        cfg.validate()
        return cfg

    def validate(self):
        for name, allowed in _CHOICES.items():
            if getattr(self, name) not in allowed:
                raise ValueError(f"{name}={getattr(self, name)!r}; expected one of {allowed}")
        if self.bucket_mb <= 0 or self.first_bucket_mb <= 0:
            raise ValueError("bucket sizes must be positive")
        if self.collective_timeout_s <= 0:
            raise ValueError("collective_timeout_s must be positive")

    def to_env(self) -> Dict[str, str]:
        """Env vars that reproduce this config in child processes (used by the launcher)."""
        out = {}
        for name in self._types():
            v = getattr(self, name)
            out[self.env_name(name)] = ("1" if v else "0") if isinstance(v, bool) else str(v)
        return out

    def asdict(self) -> Dict[str, Any]:
        return dataclasses.asdict(self)


_CURRENT: Optional[Config] = None


def get_config() -> Config:
    """Process-wide config (env + ``PDA_CONFIG`` file), resolved once; ``set_config`` overrides."""
    global _CURRENT
    if _CURRENT is None:
        _CURRENT = Config.load()
    return _CURRENT


def set_config(cfg: Optional[Config]):
    global _CURRENT
    _CURRENT = cfg


def env_flag_list(name: str) -> List[str]:
    raw = os.environ.get(name, "")
    return [s for s in raw.replace(";", ",").split(",") if s]
