"""Expert-parallel MoE on the native kernels (2 ranks sharing the test GPU over gloo)."""
import pytest

import _workers
from pytorchdistributed_amd.launch import spawn

pytestmark = pytest.mark.gpu


def test_moe_ep_native_two_ranks(tmp_path):
    spawn(_workers.moe_ep_gpu_worker, args=(2, str(tmp_path)), nprocs=2, timeout=300)
    for r in range(2):
        assert (tmp_path / f"ok{r}").read_text() == "ok"
