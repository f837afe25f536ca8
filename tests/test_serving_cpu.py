"""Serving path on CPU (reference math): KV-cached generation == uncached full forward, for Llama-3
(GQA + RoPE) and GPT-2 (learned positions, tied head); placement map; sampling determinism."""
import pytest
import torch

from pytorchdistributed_amd.models.gpt2 import gpt2
from pytorchdistributed_amd.models.llama import llama
from pytorchdistributed_amd.serving import KVCache, generate, place


def _tiny(kind):
    torch.manual_seed(0)
    if kind == "llama":
        return llama("llama3-tiny", dtype=torch.float32).eval()
    return gpt2("gpt2", n_layer=2, n_embd=128, n_head=2, vocab_size=500, n_positions=128, dtype=torch.float32).eval()


@pytest.mark.parametrize("kind", ["llama", "gpt2"])
def test_cached_generation_matches_full_forward(kind):
    m = _tiny(kind)
    g = torch.Generator().manual_seed(1)
    prompt = torch.randint(0, 500, (2, 7), generator=g)
    toks, logits = generate(m, prompt, max_new_tokens=6, return_logits=True)
    assert toks.shape == (2, 13) and torch.equal(toks[:, :7], prompt)
    with torch.no_grad():
        for i in range(6):
            full = m(toks[:, : 7 + i])
            full = full[..., :logits.shape[-1]]
            assert torch.allclose(logits[:, i], full[:, -1].float(), atol=1e-4, rtol=1e-4), i
            # greedy: the emitted token is the argmax of the full-forward logits
            assert torch.equal(toks[:, 7 + i], full[:, -1].argmax(-1))


def test_sampling_is_seeded_and_eos_sticks():
    m = _tiny("llama")
    prompt = torch.randint(0, 500, (3, 4), generator=torch.Generator().manual_seed(2))
    a = generate(m, prompt, 8, temperature=0.8, top_k=20, generator=torch.Generator().manual_seed(5))
    b = generate(m, prompt, 8, temperature=0.8, top_k=20, generator=torch.Generator().manual_seed(5))
    assert torch.equal(a, b)
    first = generate(m, prompt, 1)[:, -1]
    eos = int(first[0])
    out = generate(m, prompt, 6, eos_token=eos)
    assert (out[0, 4:] == eos).all()


def test_kv_cache_sizing_and_placement_map():
    m = _tiny("llama")
    c = KVCache(m, batch=2, max_len=16)
    assert c.k[0].shape == (2, 16, 1, 128) and c.nbytes() == 2 * 2 * 2 * 16 * 128 * 4
    assert KVCache.bytes_per_token(m, torch.bfloat16) == 2 * 2 * 1 * 128 * 2
    dmap = place(m, devices=["cpu"], max_memory={"cpu": 1 << 40})
    assert dmap["layers.0"] == torch.device("cpu") and dmap["output"] == torch.device("cpu")
    # Llama-3-8B: 128 KiB of bf16 KV cache per token (32 layers x 8 KV heads x 128 x 2)
    big = llama("llama3-8b", device="meta")
    assert KVCache.bytes_per_token(big) == 131072


def test_int8_weight_only_quantization_cpu():
    from pytorchdistributed_amd.ops import quantize_int8, quantize_linears

    w = torch.randn(64, 256)
    q, s = quantize_int8(w)
    assert q.dtype == torch.int8 and (q.abs() <= 127).all()
    assert ((q.float() * s[:, None] - w).abs() <= s[:, None] / 2 + 1e-6).all()
    m = _tiny("llama")
    prompt = torch.randint(0, 500, (2, 6), generator=torch.Generator().manual_seed(4))
    toks, ref = generate(m, prompt, 4, return_logits=True)
    assert quantize_linears(m, head=True) == 2 * 4 + 1
    # teacher-forced on the float model's tokens: a greedy near-tie flipping under int8 must not
    # turn the comparison into one between two different continuations
    with torch.no_grad():
        got = m(toks[:, :-1])[:, prompt.shape[1] - 1:, :ref.shape[-1]].float()
    assert ((got - ref).norm() / ref.norm()).item() < 0.05
    _, got_gen = generate(m, prompt, 4, return_logits=True)
    assert torch.allclose(got_gen[:, 0], got[:, 0], atol=1e-4, rtol=1e-4)
    lin = m.layers[0].wqkv  # .weight is the dequantised float weight, never the raw int8 codes
    assert lin.weight.dtype == torch.float32 and lin.device == lin.q.device
    assert torch.equal(lin.weight, lin.q.float() * lin.scale[:, None])


def test_batching_engine_and_http_front_end():
    import threading

    from fastapi.testclient import TestClient

    from pytorchdistributed_amd.serving import BatchingEngine, create_app

    m = _tiny("llama")
    eng = BatchingEngine(m, max_batch=8, window_ms=50)
    try:
        g = torch.Generator().manual_seed(9)
        prompts = [torch.randint(0, 500, (6,), generator=g).tolist() for _ in range(5)]
        futs = [eng.submit(p, 4) for p in prompts]
        res = [f.result(timeout=60) for f in futs]
        ref = generate(m, torch.tensor(prompts), 4)[:, 6:].tolist()
        assert [r["tokens"] for r in res] == ref
        assert max(r["batch"] for r in res) > 1  # requests were batched together
        client = TestClient(create_app(eng))
        out = {}

        def call(i):
            out[i] = client.post("/generate", json={"prompt": prompts[i], "max_new_tokens": 4}).json()

        ts = [threading.Thread(target=call, args=(i,)) for i in range(3)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        assert [out[i]["tokens"] for i in range(3)] == ref[:3]
        assert client.get("/health").json()["status"] == "ok"
        assert client.post("/generate", json={"prompt": []}).status_code == 400
    finally:
        eng.close()


def test_batching_engine_close_fails_pending_and_rejects_new():
    from concurrent.futures import Future

    from pytorchdistributed_amd.serving import BatchingEngine

    m = _tiny("llama")
    eng = BatchingEngine(m, max_batch=8, window_ms=5)
    eng._stop.set()  # worker exits without serving: whatever is queued must fail, not hang
    eng._thread.join(timeout=10)
    fut = Future()
    eng.q.put(((3, 2, 0.0, None), [1, 2, 3], fut))
    eng.close()
    with pytest.raises(RuntimeError, match="engine closed"):
        fut.result(timeout=5)
    with pytest.raises(RuntimeError, match="engine closed"):
        eng.submit([1, 2, 3], 2)


def test_batching_engine_worker_sets_its_device(monkeypatch):
    """The current HIP device is per thread: the worker must select the engine's device (cuda:N,
    N != 0) before it captures decode graphs there."""
    from pytorchdistributed_amd.serving import BatchingEngine

    seen = []
    monkeypatch.setattr(torch.cuda, "set_device", lambda d: seen.append(torch.device(d)))
    m = _tiny("llama")
    eng = BatchingEngine(m, graph=False, device=torch.device("cuda", 3))
    eng.close()
    assert seen == [torch.device("cuda", 3)]
