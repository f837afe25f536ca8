"""FSDP full-shard on CPU/gloo (SURVEY §4.2 T3 analogue): sharded training equals unsharded training;
sharded checkpoint consolidates to the same state dict."""
import torch
import torch.nn.functional as F

import _workers
from pytorchdistributed_amd.launch import spawn
from pytorchdistributed_amd.parallel.fsdp import consolidate


def test_fsdp_matches_unsharded(tmp_path):
    world = 2
    spawn(_workers.fsdp_worker, args=(world, str(tmp_path)), nprocs=world, timeout=180)
    torch.manual_seed(0)
    ref = _workers._Net()
    opt = torch.optim.AdamW(ref.parameters(), lr=1e-2, weight_decay=0.1)
    g = torch.Generator().manual_seed(3)
    for step in range(3):
        X = torch.randn(world * 4, 8, generator=g)
        Y = torch.randint(0, 4, (world * 4,), generator=g)
        opt.zero_grad()
        F.cross_entropy(ref(X), Y).backward()
        opt.step()
    sd = torch.load(tmp_path / "full.pt", weights_only=True)
    ref_sd = ref.state_dict()
    assert set(sd) == set(ref_sd)
    for k, v in ref_sd.items():
        assert torch.allclose(sd[k], v, atol=1e-5), k
    merged = consolidate(str(tmp_path / "ckpt"))
    for k, v in ref_sd.items():
        assert torch.allclose(merged[k], v, atol=1e-5), k


def test_fsdp_sharded_checkpoint_resumes_exactly(tmp_path):
    """Sharded checkpoint with the optimizer state (fp32 master / Adam moments / step per shard): 3 steps,
    save, resume in fresh processes, 3 more steps == 6 uninterrupted steps, bit for bit; the
    consolidated snapshot is the stock {"MODEL_STATE", "OPTIMIZER_STATE"} layout."""
    from pytorchdistributed_amd.parallel.fsdp import consolidate_snapshot

    world = 2
    for phase in ("full", "first", "resume"):
        spawn(_workers.fsdp_resume_worker, args=(world, str(tmp_path), phase), nprocs=world, timeout=180)
    for r in range(world):
        full = torch.load(tmp_path / f"full{r}.pt", weights_only=True)
        res = torch.load(tmp_path / f"resume{r}.pt", weights_only=True)
        for a, b in zip(full["losses"][3:], res["losses"]):
            assert torch.equal(a, b), (full["losses"], res["losses"])
        for k in full["state"]:
            assert torch.equal(full["state"][k], res["state"][k]), k
    snap = consolidate_snapshot(str(tmp_path / "ckpt"), str(tmp_path / "snapshot.pt"))
    loaded = torch.load(tmp_path / "snapshot.pt", weights_only=True)
    assert set(loaded) >= {"MODEL_STATE", "OPTIMIZER_STATE", "EPOCHS_RUN"}
    ref = _workers._Net()
    ref.load_state_dict(snap["MODEL_STATE"])  # loads into the unsharded model as is
    opt = torch.optim.AdamW(ref.parameters(), lr=1e-2, weight_decay=0.1)
    opt.load_state_dict(snap["OPTIMIZER_STATE"])  # torch's own optimizer accepts the consolidated state
    names = list(snap["MODEL_STATE"])
    st = snap["OPTIMIZER_STATE"]["state"]
    assert st[0]["exp_avg"].shape == snap["MODEL_STATE"][names[0]].shape


def test_fsdp_deferred_init_matches_eager(tmp_path):
    """Meta-device construction: each rank materialises one unit at a time and keeps its
    1/world shard; peak construction memory <= the rank's shards + one unit; losses and shards after three
    AdamW steps are bit-identical to FSDP over the eagerly built model (world 4, gloo), and to the run
    without the gathered-buffer ring (PDA_FSDP_RING=0)."""
    world = 4
    spawn(_workers.fsdp_deferred_init_worker, args=(world, str(tmp_path)), nprocs=world, timeout=240)
    for r in range(world):
        out = torch.load(tmp_path / f"{r}.pt", weights_only=True)
        e, d = out["eager"], out["deferred"]
        assert torch.equal(e["losses"], d["losses"]), (e["losses"], d["losses"])
        assert all(torch.equal(a, b) for a, b in zip(e["shards"], d["shards"]))
        # the preallocated gathered-buffer ring (on from step 2) changes no bit against the allocator path
        nr = out["noring"]
        assert torch.equal(e["losses"], nr["losses"]) and all(torch.equal(a, b) for a, b in zip(e["shards"], nr["shards"]))
        assert e["peak"] == 0 < d["peak"]
        assert d["peak"] <= d["shard_bytes"] + d["unit_max"]
        assert d["peak"] <= d["model_bytes"] / world + d["unit_max"]
