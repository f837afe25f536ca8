"""Tensor-parallel Llama on the native HIP kernels (2 ranks sharing the test box's GPU over gloo)."""
import pytest

import _workers
from pytorchdistributed_amd.launch import spawn

pytestmark = pytest.mark.gpu


def test_tp2_llama_bf16_native(tmp_path):
    spawn(_workers.tp_llama_gpu_worker, args=(2, str(tmp_path)), nprocs=2, timeout=300)
    for r in range(2):
        assert (tmp_path / f"ok{r}").read_text() == "ok"
