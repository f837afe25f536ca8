"""Expert parallelism (parallel/expert_parallel.py) on gloo, CPU fp32: uneven all-to-all token
dispatch / combine with autograd == a dense all-experts oracle (outputs, expert and router grads)."""
import pytest

import _workers
from pytorchdistributed_amd.launch import spawn


@pytest.mark.parametrize("world", [2, 4])
def test_moe_expert_parallel_matches_dense(tmp_path, world):
    spawn(_workers.moe_ep_worker, args=(world, str(tmp_path)), nprocs=world, timeout=240)
    for r in range(world):
        assert (tmp_path / f"ok{r}").read_text() == "ok"
