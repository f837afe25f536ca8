"""IPC collectives over xGMI (csrc/kernels/xgmi.hip: one-shot / two-shot / ring all-reduce, all-gather,
reduce-scatter) with several ranks sharing
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


@pytest.mark.parametrize("world", [2, 3, 4])
def test_xgmi_ring_allreduce(tmp_path, world):
    """The tutorial's ring (N-1 reduce-scatter + N-1 all-gather neighbour steps) on the GPU, switching
    with the direct algorithms on the same buffers; world 3 leaves the last chunk ragged."""
    spawn(_workers.xgmi_worker, args=(world, str(tmp_path), ("ring", "oneshot", "ring", "twoshot")),
          nprocs=world, timeout=300)
    for r in range(world):
        assert (tmp_path / f"ok{r}").read_text() == "ok"


@pytest.mark.parametrize("world", [2, 4])
def test_xgmi_allgather_reduce_scatter(tmp_path, world):
    spawn(_workers.xgmi_collectives_worker, args=(world, str(tmp_path)), nprocs=world, timeout=300)
    for r in range(world):
        assert (tmp_path / f"ok{r}").read_text() == "ok"


def test_fsdp_over_xgmi_ipc_matches_unsharded(tmp_path):
    """PDA_FSDP_COMM=ipc: unit all-gathers and gradient reduce-scatters on the IPC kernels (2 ranks)."""
    spawn(_workers.fsdp_llama_gpu_worker, args=(2, str(tmp_path), "ipc"), nprocs=2, timeout=300)
    for r in range(2):
        assert (tmp_path / f"ok{r}").read_text().startswith("ok")


def test_xgmi_barrier_timeout_is_reported(tmp_path):
    spawn(_workers.xgmi_timeout_worker, args=(2, str(tmp_path)), nprocs=2, timeout=300)
    assert (tmp_path / "ok0").read_text() == "raised"


@pytest.mark.parametrize("world,zero_copy", [(2, True), (3, True), (2, False)])
def test_ddp_buckets_over_xgmi_ipc(tmp_path, world, zero_copy):
    spawn(_workers.ddp_xgmi_gpu_worker, args=(world, str(tmp_path), zero_copy), nprocs=world, timeout=300)
    for r in range(world):
        assert (tmp_path / f"ok{r}").read_text() == "ok"


@pytest.mark.parametrize("world", [2, 4])
def test_xgmi_zero_copy_registered(tmp_path, world):
    """Zero-copy mode: registered tensors read in place by peers (no copy-in; exchange buffer smaller than
    every message), all-reduce (two-shot / ring) on slices of a registered flat buffer, all-gather of a
    registered shard, reduce-scatter of a registered full buffer, vs fp32 sums."""
    spawn(_workers.xgmi_zero_copy_worker, args=(world, str(tmp_path)), nprocs=world, timeout=300)
    for r in range(world):
        assert (tmp_path / f"ok{r}").read_text() == "ok"
