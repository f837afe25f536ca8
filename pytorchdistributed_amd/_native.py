"""Loader for the native extension ``pytorchdistributed_amd._C``.

GPU code paths call :func:`C` which raises loudly when the extension is missing (a silent eager
fallback on a GPU box would hide that the HIP kernels never ran).  CPU-only paths (tests, the gloo
plumbing config) use :func:`maybe` and fall back to PyTorch reference math.
"""
from __future__ import annotations

import importlib
import os

_mod = None
_err: Exception | None = None


def _load():
    global _mod, _err
    if _mod is not None or _err is not None:
        return
    try:
        _mod = importlib.import_module("pytorchdistributed_amd._C")
    except Exception as e:  # pragma: no cover - depends on the build state
        if os.environ.get("PDA_AUTOBUILD", "1") == "1":
            try:
                from . import _build

                _build.build()
                _mod = importlib.import_module("pytorchdistributed_amd._C")
                return
            except Exception as e2:  # noqa: BLE001
                _err = e2
                return
        _err = e


def available() -> bool:
    _load()
    return _mod is not None


def C():
    """Return the native module or raise (used on every GPU path)."""
    _load()
    if _mod is None:
        raise RuntimeError(
            "pytorchdistributed_amd._C is not built/loadable; run `python -m pytorchdistributed_amd._build` "
            f"(original error: {_err!r})"
        )
    return _mod


def maybe():
    _load()
    return _mod
