"""IPC all-reduce over xGMI (csrc/kernels/xgmi.hip: one-shot and two-shot) with several ranks sharing
the one GPU of the test box: exchange buffers and flags are IPC-mapped between the processes exactly as
between the GPUs of a node; results vs the sum / mean of the inputs over several epochs, fp32 and
bf16, sizes that leave two-shot chunks ragged or empty, and algorithm switches between calls."""
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


@pytest.mark.parametrize("world", [2, 4])
def test_xgmi_twoshot_processes_one_gpu(tmp_path, world):
    spawn(_workers.xgmi_worker, args=(world, str(tmp_path), ("twoshot", "oneshot", "twoshot", "auto")),
          nprocs=world, timeout=300)
    for r in range(world):
        assert (tmp_path / f"ok{r}").read_text() == "ok"


def test_xgmi_barrier_timeout_is_reported(tmp_path):
    spawn(_workers.xgmi_timeout_worker, args=(2, str(tmp_path)), nprocs=2, timeout=300)
    assert (tmp_path / "ok0").read_text() == "raised"


@pytest.mark.parametrize("world", [2, 3])
def test_ddp_buckets_over_xgmi_ipc(tmp_path, world):
    spawn(_workers.ddp_xgmi_gpu_worker, args=(world, str(tmp_path)), nprocs=world, timeout=300)
    for r in range(world):
        assert (tmp_path / f"ok{r}").read_text() == "ok"
