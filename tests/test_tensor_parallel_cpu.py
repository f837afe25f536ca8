"""Tensor parallelism (parallel/tensor_parallel.py) on gloo, CPU fp32: a TP-sharded Llama computes the
full model's logits / loss / gradients (gradient shards == slices of the full gradients), with and
without sequence parallelism, and serves KV-cached generation identical to the full model."""
import pytest

import _workers
from pytorchdistributed_amd.launch import spawn


@pytest.mark.parametrize("sp", [False, True])
def test_tp_llama_matches_full_model(tmp_path, sp):
    spawn(_workers.tp_llama_worker, args=(2, sp, str(tmp_path)), nprocs=2, timeout=240)
    for r in range(2):
        assert (tmp_path / f"ok{r}").read_text() == "ok"
