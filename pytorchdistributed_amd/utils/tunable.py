"""Per-shape selection of the vendor library GEMM solutions (PyTorch TunableOp over hipBLASLt/rocBLAS).

Plain linear GEMMs of the transformer models go to hipBLASLt through ``torch.mm`` (ops/linear.py).
The library's default heuristic pick is weak on some training shapes — e.g. the GPT-2-medium weight
gradient 1024 x 1024 x 16384 runs at ~350 TFLOP/s with it — so each model's GEMM shapes were timed
over all candidate solutions once on an MI355X and the winners are committed under
``pytorchdistributed_amd/tuning/tunableop_<model>.csv``; a run only reads that table (no tuning).

``PDA_TUNABLEOP``: ``1`` (default) use the table when it exists, ``0`` off, ``tune`` re-tune and write
``PDA_TUNABLEOP_OUT`` (torch appends the device ordinal to the file name).
"""
from __future__ import annotations

import os

import torch

TABLE_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tuning")


def use_tuned_gemms(tag: str) -> str:
    """Enable TunableOp for this process with the committed table of ``tag``; returns the mode used."""
    mode = os.environ.get("PDA_TUNABLEOP", "1")
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
