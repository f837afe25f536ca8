"""One-shot IPC all-reduce (csrc/kernels/xgmi.hip) with 2 ranks sharing the one GPU of the test box:
exchange buffers and flags are IPC-mapped between the two processes exactly as between the GPUs of
a node; results vs the sum / mean of the inputs, several epochs, fp32 and bf16."""
import os

import pytest
import torch

import _workers  # noqa: F401  (path setup for spawned children)
from pytorchdistributed_amd.launch import spawn

pytestmark = pytest.mark.gpu


def test_xgmi_oneshot_two_processes_one_gpu(tmp_path):
    spawn(_workers.xgmi_worker, args=(2, str(tmp_path)), nprocs=2, timeout=300)
    for r in range(2):
        assert (tmp_path / f"ok{r}").read_text() == "ok"
