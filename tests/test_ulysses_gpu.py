"""Ulysses SP attention on the native flash-attention kernels (2 ranks sharing the test GPU, gloo)."""
import pytest

import _workers
from pytorchdistributed_amd.launch import spawn

pytestmark = pytest.mark.gpu


def test_ulysses_native_two_ranks(tmp_path):
    spawn(_workers.ulysses_worker, args=(2, "cuda", str(tmp_path)), nprocs=2, timeout=300)
    for r in range(2):
        assert (tmp_path / f"ok{r}").read_text() == "ok"


def test_ring_attention_native_two_ranks(tmp_path):
    spawn(_workers.ulysses_worker, args=(2, "cuda", str(tmp_path), "ring"), nprocs=2, timeout=300)
    for r in range(2):
        assert (tmp_path / f"ok{r}").read_text() == "ok"
