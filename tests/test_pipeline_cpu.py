"""Pipeline parallelism tests on CPU/gloo: schedule invariants, GPipe / 1F1B
gradients equal to single-process training, recompute, PP x DP groups."""
import pytest
import torch
import torch.nn.functional as F

import _workers
from pytorchdistributed_amd.launch import spawn
from pytorchdistributed_amd.parallel.pipeline import (check_schedule, partition_layers, schedule_1f1b,
                                                      schedule_gpipe)


@pytest.mark.parametrize("S", [1, 2, 3, 4, 8])
@pytest.mark.parametrize("M", [1, 2, 4, 7, 16])
def test_schedules_complete_and_are_well_formed(S, M):
    for fn in (schedule_gpipe, schedule_1f1b):
        assert check_schedule(fn, S, M)
        for s in range(S):
            acts = fn(S, M, s)
            assert sorted(a for a in acts if a[0] == "F") == [("F", i) for i in range(M)]
            assert sorted(a for a in acts if a[0] == "B") == [("B", i) for i in range(M)]
            for i in range(M):  # forward of a micro-batch precedes its backward
                assert acts.index(("F", i)) < acts.index(("B", i))


def test_1f1b_bounds_in_flight_activations():
    S, M = 4, 16
    for s in range(S):
        live = peak = 0
        for kind, _ in schedule_1f1b(S, M, s):
            live += 1 if kind == "F" else -1
            peak = max(peak, live)
        assert peak <= S - s  # vs M for GPipe


def test_partition_layers():
    assert partition_layers(48, 4) == [(0, 12), (12, 24), (24, 36), (36, 48)]
    assert partition_layers(5, 2) == [(0, 3), (3, 5)]


def _reference_grads(dp):
    full = _workers._tiny_stack(4)
    g = torch.Generator().manual_seed(1)
    X = torch.randn(dp * 8, 16, generator=g)
    Y = torch.randn(dp * 8, 16, generator=g)
    # per-replica mean over 4 micro-batches of 2 == mean over the replica batch; then DP average
    F.mse_loss(full(X), Y).backward()
    return full


@pytest.mark.parametrize("pp,dp,schedule,recompute", [(2, 1, "gpipe", False), (2, 1, "1f1b", False),
                                                      (4, 1, "1f1b", True), (2, 2, "1f1b", False)])
def test_pipeline_grads_match_single_process(tmp_path, pp, dp, schedule, recompute):
    world = pp * dp
    spawn(_workers.pipeline_worker, args=(world, pp, dp, schedule, recompute, str(tmp_path)), nprocs=world,
          timeout=180)
    ref = _reference_grads(dp)
    ref_blocks = [ref[3 * i: 3 * i + 3] for i in range(4)]
    for r in range(world):
        d = torch.load(tmp_path / f"{r}.pt", weights_only=True)
        lo = d["lo"]
        stage = r % pp
        hi = partition_layers(4, pp)[stage][1]
        ref_stage = torch.nn.Sequential(*ref_blocks[lo:hi])
        for (n, p) in ref_stage.named_parameters():
            assert torch.allclose(d["grads"][n], p.grad, atol=1e-5, rtol=1e-4), (r, n)
