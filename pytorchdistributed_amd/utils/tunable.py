"""Per-shape selection of vendor-library GEMM solutions (PyTorch TunableOp over hipBLASLt/rocBLAS).

Since round 4 no framework GEMM goes to the vendor library: every bf16 Linear / conv GEMM runs on the
native kernels (ops/linear.py, csrc/kernels/gemm_pp.hip), so this only matters for PyTorch ops a user
script calls directly (``torch.mm`` / ``F.linear`` on GPU tensors).  The tables tuned on MI355X for the
transformer configs while their Linears still used hipBLASLt stay under
``pytorchdistributed_amd/tuning/tunableop_<model>.csv``; a run only reads a table (no tuning).

``PDA_TUNABLEOP``: ``0`` (default) off, ``1`` use the table when it exists, ``tune`` re-tune and write
``PDA_TUNABLEOP_OUT`` (torch appends the device ordinal to the file name).
"""
from __future__ import annotations

import os

import torch

TABLE_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tuning")


def use_tuned_gemms(tag: str) -> str:
    """Enable TunableOp for this process with the committed table of ``tag``; returns the mode used."""
    mode = os.environ.get("PDA_TUNABLEOP", "0")
    if mode == "0" or not torch.cuda.is_available():
        return "off"
    from torch.cuda import tunable

    path = os.path.join(TABLE_DIR, f"tunableop_{tag}.csv")
    if mode == "tune":
        tunable.enable(True)
        tunable.tuning_enable(True)
        tunable.set_max_tuning_duration(int(os.environ.get("PDA_TUNABLEOP_MS", "20")))
        tunable.set_max_tuning_iterations(int(os.environ.get("PDA_TUNABLEOP_ITERS", "10")))
        tunable.set_filename(os.environ.get("PDA_TUNABLEOP_OUT", path))
        return "tune"
    if not os.path.exists(path):
        return "off"
    import tempfile

    tunable.enable(True)
    tunable.tuning_enable(False)
    # results are only read; anything torch writes back at exit goes to a scratch file, never the table
    tunable.set_filename(os.path.join(tempfile.gettempdir(), f"pda_tunableop_{tag}_{os.getpid()}.csv"))
    tunable.read_file(path)
    return "table"
