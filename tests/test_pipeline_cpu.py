"""Pipeline parallelism tests on CPU/gloo: schedule invariants, GPipe / 1F1B
gradients equal to single-process training, recompute, PP x DP groups."""
import pytest
import torch
import torch.nn.functional as F

import _workers
from pytorchdistributed_amd.launch import spawn
from pytorchdistributed_amd.parallel.pipeline import (check_schedule, partition_layers, plan_interleaved,
                                                      schedule_1f1b, schedule_gpipe, schedule_interleaved)


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


@pytest.mark.parametrize("pp,dp,schedule,recompute,dp_mode", [
    (2, 1, "gpipe", False, "none"), (2, 1, "1f1b", False, "none"), (4, 1, "1f1b", True, "none"),
    (2, 2, "1f1b", True, "ddp"), (2, 2, "1f1b", False, "ddp"), (2, 2, "gpipe", True, "ddp")])
def test_pipeline_grads_match_single_process(tmp_path, pp, dp, schedule, recompute, dp_mode):
    """``dp_mode="ddp"``: the DP average runs through the stage's DDP over its DP group, launched during
    the last micro-batch's backward (no_sync before), reporting the exposed communication time."""
    world = pp * dp
    spawn(_workers.pipeline_worker, args=(world, pp, dp, schedule, recompute, str(tmp_path), dp_mode),
          nprocs=world, timeout=180)
    if dp_mode == "ddp":
        for r in range(world):
            st = torch.load(tmp_path / f"{r}.pt", weights_only=True)["stats"]
            assert st["comm_calls"] > 0 and "exposed_comm_ms" in st, st
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


@pytest.mark.parametrize("S", [1, 2, 3, 4])
@pytest.mark.parametrize("v", [1, 2, 3])
@pytest.mark.parametrize("k", [1, 2, 4])
def test_interleaved_schedule_well_formed(S, v, k):
    M = k * S
    for s in range(S):
        acts = schedule_interleaved(S, M, s, v)
        units = {(c, mb) for c in range(v) for mb in range(M)}
        assert sorted((c, mb) for kind, c, mb in acts if kind == "F") == sorted(units)
        assert sorted((c, mb) for kind, c, mb in acts if kind == "B") == sorted(units)
        for c, mb in units:
            assert acts.index(("F", c, mb)) < acts.index(("B", c, mb))
    ticks = plan_interleaved(S, M, v)  # raises if the ranks' unit lists deadlock
    # the fill/drain bubble (ticks beyond the 2*M*v units of work) shrinks with v in stage-time units
    assert len(ticks) - 2 * M * v <= 2 * (S - 1) + (v - 1) * S + 2 * S


def test_interleaved_bubble_shrinks_with_chunks():
    S, M = 4, 16
    stage_time = {v: len(plan_interleaved(S, M, v)) / v for v in (1, 2, 4)}
    assert stage_time[4] < stage_time[2] < stage_time[1]


def test_interleaved_needs_divisible_microbatches():
    with pytest.raises(ValueError):
        schedule_interleaved(4, 6, 0, 2)


@pytest.mark.parametrize("world,chunks,n_layers,n_micro,recompute", [(2, 2, 4, 4, False), (2, 2, 8, 2, True),
                                                                     (4, 2, 8, 4, False), (1, 3, 3, 2, False)])
def test_interleaved_pipeline_grads_match_single_process(tmp_path, world, chunks, n_layers, n_micro, recompute):
    spawn(_workers.pipeline_interleaved_worker, args=(world, chunks, n_layers, n_micro, recompute, str(tmp_path)),
          nprocs=world, timeout=180)
    full = _workers._tiny_stack(n_layers)
    g = torch.Generator().manual_seed(1)
    X = torch.randn(n_micro * 2, 16, generator=g)
    Y = torch.randn(n_micro * 2, 16, generator=g)
    loss = F.mse_loss(full(X), Y)
    loss.backward()
    per = n_layers // (world * chunks)
    blocks = [full[3 * i: 3 * i + 3] for i in range(n_layers)]
    for r in range(world):
        d = torch.load(tmp_path / f"{r}.pt", weights_only=True)
        if r == world - 1:
            assert torch.allclose(d["loss"], loss.detach(), atol=1e-6)
        for c in range(chunks):
            vs = c * world + r
            ref = torch.nn.Sequential(*[m for b in blocks[vs * per:(vs + 1) * per] for m in b])
            for n, p in ref.named_parameters():
                assert torch.allclose(d["grads"][f"{c}.{n}"], p.grad, atol=1e-5, rtol=1e-4), (r, c, n)


def test_interleaved_pipeline_ddp_grads_match_single_process(tmp_path):
    """Interleaved schedule x DDP: 2 stages x 2 chunks x 2 DP replicas on gloo; the DP
    average runs through each rank's DDP wrapper (multi-pass buckets)."""
    pp, dp, chunks, n_layers, n_micro = 2, 2, 2, 8, 4
    spawn(_workers.pipeline_interleaved_ddp_worker, args=(pp * dp, pp, dp, chunks, n_layers, n_micro, str(tmp_path)),
          nprocs=pp * dp, timeout=180)
    full = _workers._tiny_stack(n_layers)
    g = torch.Generator().manual_seed(1)
    B = n_micro * 2
    X = torch.randn(dp * B, 16, generator=g)
    Y = torch.randn(dp * B, 16, generator=g)
    # the replicas' losses are means over their own half: the DP-averaged gradient is that of the mean
    # of the two half-batch means = the full-batch mean (equal halves)
    loss = F.mse_loss(full(X), Y)
    loss.backward()
    per = n_layers // (pp * chunks)
    blocks = [full[3 * i: 3 * i + 3] for i in range(n_layers)]
    for r in range(pp * dp):
        d = torch.load(tmp_path / f"{r}.pt", weights_only=True)
        s = d["stage"]
        assert d["stats"]["comm_calls"] > 0
        for c in range(chunks):
            vs = c * pp + s
            ref = torch.nn.Sequential(*[m for b in blocks[vs * per:(vs + 1) * per] for m in b])
            for n, p in ref.named_parameters():
                assert torch.allclose(d["grads"][f"{c}.{n}"], p.grad, atol=1e-5, rtol=1e-4), (r, c, n)


@pytest.mark.parametrize("world,chunks", [(2, 1), (2, 2), (4, 1)])
def test_pipeline_checkpoint_roundtrip_and_consolidate(tmp_path, world, chunks):
    """PP checkpoint layout: stage files + partition map, reload, consolidation."""
    spawn(_workers.pipeline_ckpt_worker, args=(world, chunks, str(tmp_path)), nprocs=world, timeout=180)
    for r in range(world):
        assert (tmp_path / f"ok{r}").read_text() == "ok"
    assert sorted(p.name for p in (tmp_path / "ckpt").iterdir()) == \
        ["pipeline.json"] + [f"stage_{s:03d}.pt" for s in range(world)]


@pytest.mark.parametrize("find_unused", [False, True])
def test_interleaved_ddp_unused_parameter_is_reported(tmp_path, find_unused):
    """a chunk parameter that gets no gradient must not leave the multi-pass DDP step with
    unlaunched buckets; Pipeline finalizes through DDP.finish_multi_pass after its last backward."""
    import os

    spawn(_workers.pipeline_interleaved_unused_worker, args=(1, find_unused, str(tmp_path)), nprocs=1, timeout=120)
    out = torch.load(os.path.join(tmp_path, "0.pt"), weights_only=False)
    if find_unused:
        assert out["error"] is None and out["unused_grad_zero"] and out["pending"] == [0] and not out["open"]
    else:
        assert out["error"] is not None and "received no gradient" in out["error"]
