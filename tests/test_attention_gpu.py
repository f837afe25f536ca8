"""Flash-attention / embedding / RoPE kernels vs fp32 PyTorch references, and small GPT-2 / Llama
models end to end on the native path."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu


def rel_err(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


@pytest.mark.parametrize("B,T,Hq,Hkv,D,causal", [(2, 128, 4, 4, 64, True), (1, 200, 4, 2, 128, True),
                                                  (2, 64, 2, 2, 128, False), (1, 256, 8, 1, 64, True),
                                                  (1, 96, 2, 2, 64, False), (1, 200, 4, 2, 64, True),
                                                  (2, 72, 2, 1, 64, True), (1, 330, 2, 2, 64, False)])
@pytest.mark.parametrize("use_rope", [False, True])
def test_flash_attention_fwd_bwd(B, T, Hq, Hkv, D, causal, use_rope):
    from pytorchdistributed_amd.ops.attention import attention_qkv, attention_ref, rope_tables

    torch.manual_seed(0)
    qkv = torch.randn(B, T, Hq + 2 * Hkv, D).to(torch.bfloat16)
    rope = rope_tables(T, D, 10000.0) if use_rope else None
    ref_in = qkv.float().clone().requires_grad_()
    q, k, v = ref_in[:, :, :Hq], ref_in[:, :, Hq:Hq + Hkv], ref_in[:, :, Hq + Hkv:]
    o_ref = attention_ref(q, k, v, causal, 1 / math.sqrt(D), rope)
    do = torch.randn_like(o_ref)
    o_ref.backward(do)
    g_in = qkv.cuda().requires_grad_()
    rope_g = tuple(t.cuda() for t in rope) if rope is not None else None
    o = attention_qkv(g_in, Hq, Hkv, causal=causal, rope=rope_g)
    o.backward(do.cuda().to(torch.bfloat16))
    assert rel_err(o.cpu(), o_ref.detach()) < 2e-2
    g = g_in.grad.cpu().float()
    r = ref_in.grad
    assert rel_err(g[:, :, :Hq], r[:, :, :Hq]) < 3e-2            # dq
    assert rel_err(g[:, :, Hq:Hq + Hkv], r[:, :, Hq:Hq + Hkv]) < 3e-2  # dk
    assert rel_err(g[:, :, Hq + Hkv:], r[:, :, Hq + Hkv:]) < 3e-2      # dv


@pytest.mark.parametrize("B,T,Hq,Hkv,D,causal", [(2, 128, 4, 4, 64, True), (1, 200, 4, 2, 128, True),
                                                  (2, 64, 2, 2, 128, False), (1, 256, 8, 1, 64, True),
                                                  (1, 96, 2, 2, 64, False), (1, 200, 4, 2, 64, True),
                                                  (2, 72, 2, 1, 64, True), (1, 330, 2, 2, 64, False),
                                                  (1, 520, 4, 1, 128, True), (2, 384, 4, 4, 64, True)])
def test_flash_attention_bwd_fused_dq(B, T, Hq, Hkv, D, causal):
    """Fused key-stationary backward (dQ through the fp32 atomic accumulator, PDA_ATTN_BWD_FUSED) vs
    the fp32 reference and vs the two-kernel path."""
    from pytorchdistributed_amd._native import C
    from pytorchdistributed_amd.ops.attention import attention_qkv, attention_ref

    torch.manual_seed(1)
    qkv = torch.randn(B, T, Hq + 2 * Hkv, D).to(torch.bfloat16)
    ref_in = qkv.float().clone().requires_grad_()
    q, k, v = ref_in[:, :, :Hq], ref_in[:, :, Hq:Hq + Hkv], ref_in[:, :, Hq + Hkv:]
    o_ref = attention_ref(q, k, v, causal, 1 / math.sqrt(D), None)
    do = torch.randn_like(o_ref)
    o_ref.backward(do)
    grads = {}
    old = C().attn_bwd_fused_mode()
    try:
        for mode in (0, 3):
            C().set_attn_bwd_fused(mode)
            g_in = qkv.cuda().requires_grad_()
            o = attention_qkv(g_in, Hq, Hkv, causal=causal)
            o.backward(do.cuda().to(torch.bfloat16))
            grads[mode] = g_in.grad.cpu().float()
    finally:
        C().set_attn_bwd_fused(old)
    g, r = grads[3], ref_in.grad
    assert torch.isfinite(g).all()
    for sl in (slice(0, Hq), slice(Hq, Hq + Hkv), slice(Hq + Hkv, Hq + 2 * Hkv)):  # dq, dk, dv
        assert rel_err(g[:, :, sl], r[:, :, sl]) < 3e-2
        assert rel_err(g[:, :, sl], grads[0][:, :, sl]) < 1e-2


def test_embedding_and_rope_kernels():
    from pytorchdistributed_amd._native import C
    from pytorchdistributed_amd.ops import embedding
    from pytorchdistributed_amd.ops.attention import _rope_ref, rope_tables

    torch.manual_seed(1)
    table = torch.randn(100, 64).to(torch.bfloat16)
    idx = torch.randint(0, 100, (3, 17))
    tg = table.cuda().requires_grad_()
    out = embedding(idx.cuda(), tg)
    assert torch.equal(out.cpu(), table[idx])
    dy = torch.randn(3, 17, 64).to(torch.bfloat16)
    out.backward(dy.cuda())
    ref = torch.zeros(100, 64).index_add_(0, idx.reshape(-1), dy.float().reshape(-1, 64))
    assert rel_err(tg.grad.cpu(), ref) < 1e-2
    x = torch.randn(2, 9, 3, 64).to(torch.bfloat16)
    cs, sn = rope_tables(9, 64)
    y = C().rope(x.cuda(), cs.cuda(), sn.cuda(), False, None)
    assert rel_err(y.cpu(), _rope_ref(x, cs, sn)) < 1e-2
    back = C().rope(y, cs.cuda(), sn.cuda(), True, None)
    assert rel_err(back.cpu(), x) < 2e-2
    # strided input (head slice of a fused buffer) written into a strided output slice
    big = torch.randn(2, 9, 5, 64).to(torch.bfloat16)
    out = torch.zeros(2, 9, 7, 64, dtype=torch.bfloat16).cuda()
    C().rope(big.cuda()[:, :, 1:4], cs.cuda(), sn.cuda(), False, out[:, :, 2:5])
    assert rel_err(out[:, :, 2:5].cpu(), _rope_ref(big[:, :, 1:4], cs, sn)) < 1e-2
    assert out[:, :, :2].abs().sum().item() == 0 and out[:, :, 5:].abs().sum().item() == 0


def test_attention_kernel_inline_rope():
    """The kernels' in-load rotary path (rope_cos/rope_sin arguments) against the reference."""
    from pytorchdistributed_amd._native import C
    from pytorchdistributed_amd.ops.attention import attention_ref, rope_tables

    torch.manual_seed(3)
    q, k, v = (torch.randn(1, 128, h, 64).to(torch.bfloat16) for h in (4, 2, 2))
    cs, sn = rope_tables(128, 64)
    o, _ = C().attn_fwd(q.cuda(), k.cuda(), v.cuda(), 0.125, True, cs.cuda(), sn.cuda())
    ref = attention_ref(q.float(), k.float(), v.float(), True, 0.125, (cs, sn))
    assert rel_err(o.cpu(), ref) < 2e-2


def test_gpt2_small_native_vs_reference():
    import copy

    from pytorchdistributed_amd.models.gpt2 import GPT2, config

    torch.manual_seed(0)
    cfg = config("gpt2", n_layer=2, n_embd=256, n_head=4, n_positions=128, vocab_size=1000)
    ref = GPT2(cfg, dtype=torch.bfloat16)
    gpu = copy.deepcopy(ref).cuda()
    idx = torch.randint(0, 1000, (2, 128))
    tgt = torch.randint(0, 1000, (2, 128))
    l_ref = ref(idx, tgt)
    l_ref.backward()
    l = gpu(idx.cuda(), tgt.cuda())
    l.backward()
    assert abs(l.item() - l_ref.item()) < 2e-2
    for n in ["wte", "h.0.c_attn.weight", "h.1.mlp_proj.weight", "ln_f.weight"]:
        g = dict(gpu.named_parameters())[n].grad.float().cpu().flatten()
        r = dict(ref.named_parameters())[n].grad.float().flatten()
        assert torch.nn.functional.cosine_similarity(g, r, dim=0) > 0.98, n


def test_llama_tiny_native_vs_reference():
    import copy

    from pytorchdistributed_amd.models.llama import Llama, config

    torch.manual_seed(0)
    cfg = config("llama3-tiny", dim=256, n_heads=2, n_kv_heads=1, ffn_dim=512)
    ref = Llama(cfg, dtype=torch.bfloat16)
    gpu = copy.deepcopy(ref).cuda()
    gpu._rope_cache = {}
    idx = torch.randint(0, cfg.vocab_size, (2, 128))
    tgt = torch.randint(0, cfg.vocab_size, (2, 128))
    l_ref = ref(idx, tgt)
    l_ref.backward()
    l = gpu(idx.cuda(), tgt.cuda())
    l.backward()
    assert abs(l.item() - l_ref.item()) < 2e-2
    for n in ["tok_embeddings", "layers.0.wqkv.weight", "layers.1.w13.weight", "output.weight"]:
        g = dict(gpu.named_parameters())[n].grad.float().cpu().flatten()
        r = dict(ref.named_parameters())[n].grad.float().flatten()
        assert torch.nn.functional.cosine_similarity(g, r, dim=0) > 0.98, n


def test_deterministic_mode_transformer_bit_identical(monkeypatch):
    """PDA_DETERMINISTIC=1 also covers the transformer path — the fused attention backward (dQ
    by fp32 atomics) gives way to the atomic-free dQ + dK/dV pair and the embedding backward sums each
    token's rows in sorted order.  Two GPT-2 training steps from the same state are bit-identical, and the
    deterministic embedding gradient equals the fp32 reference."""
    import copy

    from pytorchdistributed_amd.models.gpt2 import GPT2, config

    monkeypatch.setenv("PDA_DETERMINISTIC", "1")
    torch.manual_seed(0)
    cfg = config("gpt2", n_layer=2, n_embd=256, n_head=4, n_positions=512, vocab_size=1000)
    base = GPT2(cfg, dtype=torch.bfloat16).cuda()
    idx = torch.randint(0, 50, (4, 512), device="cuda")  # many repeated tokens: contended embedding rows
    tgt = torch.randint(0, 1000, (4, 512), device="cuda")

    def run():
        m = copy.deepcopy(base)
        loss = m(idx, tgt)
        loss.backward()
        torch.cuda.synchronize()
        return loss.detach().clone(), [p.grad.detach().clone() for p in m.parameters()]

    l1, g1 = run()
    l2, g2 = run()
    assert torch.equal(l1, l2)
    assert all(torch.equal(a, b) for a, b in zip(g1, g2))
    # the sorted embedding backward against fp32 index_add
    from pytorchdistributed_amd.ops import embedding

    table = torch.randn(100, 64).to(torch.bfloat16)
    ids = torch.randint(0, 7, (5, 33))
    dy = torch.randn(5, 33, 64).to(torch.bfloat16)
    tg = table.cuda().requires_grad_()
    embedding(ids.cuda(), tg).backward(dy.cuda())
    ref = torch.zeros(100, 64).index_add_(0, ids.reshape(-1), dy.float().reshape(-1, 64))
    assert rel_err(tg.grad.cpu(), ref) < 1e-2
    assert tg.grad[7:].abs().sum().item() == 0
