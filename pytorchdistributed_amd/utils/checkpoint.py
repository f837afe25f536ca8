"""Checkpoint / resume.

Layout (stock-PyTorch compatible, loads without this framework):
``{"MODEL_STATE": model.module.state_dict() (no ``module.`` prefix), "OPTIMIZER_STATE": ...,
"EPOCHS_RUN": int, "RNG": {...}}`` written by rank 0 with an atomic rename.  Sharded (FSDP) runs write
``shard_{rank:05d}.pt`` + ``meta.json`` (see :mod:`pytorchdistributed_amd.parallel.fsdp`).
Loading always uses ``weights_only=True``.
"""
from __future__ import annotations

import os
import random

import torch


def unwrap(model):
    return model.module if hasattr(model, "module") else model


def rng_state():
    st = {"torch": torch.get_rng_state(), "python": random.getstate()}
    if torch.cuda.is_available():
        st["cuda"] = torch.cuda.get_rng_state_all()
    return st


def set_rng_state(st):
    if not st:
        return
    torch.set_rng_state(st["torch"])
    if "python" in st:
        random.setstate(st["python"])
    if "cuda" in st and torch.cuda.is_available():
        torch.cuda.set_rng_state_all(st["cuda"])


def save_snapshot(path: str, model, optimizer=None, epochs_run: int = 0, extra: dict | None = None):
    """Models with a reference layout (``reference_state_dict()``, e.g. the channels-last ResNet-50 ->
    torchvision's OIHW / top-level ``conv1``) are saved in it, tagged ``"LAYOUT": "reference"``."""
    m = unwrap(model)
    if hasattr(m, "reference_state_dict"):
        snap = {"MODEL_STATE": m.reference_state_dict(), "LAYOUT": "reference", "EPOCHS_RUN": epochs_run}
    else:
        snap = {"MODEL_STATE": m.state_dict(), "EPOCHS_RUN": epochs_run}
    if optimizer is not None:
        snap["OPTIMIZER_STATE"] = optimizer.state_dict()
    snap["RNG"] = rng_state()
    if extra:
        snap.update(extra)
    tmp = path + ".tmp"
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    torch.save(snap, tmp)
    os.replace(tmp, path)


def load_snapshot(path: str, model, optimizer=None, map_location="cpu") -> int:
    snap = torch.load(path, map_location=map_location, weights_only=True)
    m = unwrap(model)
    if snap.get("LAYOUT") == "reference" and hasattr(m, "load_reference_state_dict"):
        m.load_reference_state_dict(snap["MODEL_STATE"])
    else:
        m.load_state_dict(snap["MODEL_STATE"])
    if optimizer is not None and "OPTIMIZER_STATE" in snap:
        optimizer.load_state_dict(snap["OPTIMIZER_STATE"])
        sync = getattr(optimizer, "sync_from_state", None)
        if sync is not None:
            sync()
    return int(snap.get("EPOCHS_RUN", 0))
