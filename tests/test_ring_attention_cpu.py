"""Ring attention / context parallelism (parallel/ring_attention.py) on gloo, CPU fp32: output and input
gradients of every rank's sequence shard == full causal GQA attention."""
import pytest

import _workers
from pytorchdistributed_amd.launch import spawn


@pytest.mark.parametrize("world", [2, 3, 4])
def test_ring_attention_matches_full_attention(tmp_path, world):
    spawn(_workers.ulysses_worker, args=(world, "cpu", str(tmp_path), "ring"), nprocs=world, timeout=240)
    for r in range(world):
        assert (tmp_path / f"ok{r}").read_text() == "ok"
