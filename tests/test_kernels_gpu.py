"""Numerics of every HIP kernel against a plain PyTorch fp32 reference of the same op.

Run on the MI355X box: ``python -m pytest tests -m gpu``.  All tests here are single-process.
"""
import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = "cuda"


def C():
    from pytorchdistributed_amd._native import C as _C

    return _C()


def rel_err(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


def bf(x):
    return x.to(DEV, torch.bfloat16).contiguous()


# ----------------------------------------------------------------------------- GEMM
@pytest.mark.parametrize("M,N,K", [(128, 128, 64), (300, 200, 136), (1024, 1000, 2048), (77, 64, 520),
                                   (4096, 256, 64), (16, 8, 8)])
@pytest.mark.parametrize("ak,bk", [(True, True), (True, False), (False, True), (False, False)])
def test_gemm_layouts(M, N, K, ak, bk):
    if not ak and M % 8:
        pytest.skip("M-major A needs M % 8 == 0")
    torch.manual_seed(0)
    A = torch.randn(M, K)
    B = torch.randn(K, N)
    a_store = bf(A) if ak else bf(A.t().contiguous())
    b_store = bf(B.t().contiguous()) if bk else bf(B)
    lda = K if ak else M
    ldb = K if bk else N
    out = torch.empty(M, N, device=DEV, dtype=torch.float32)
    C().gemm(a_store, ak, lda, b_store, bk, ldb, out, N, M, N, K, None, False, True)
    ref = A.to(torch.bfloat16).float() @ B.to(torch.bfloat16).float()
    assert rel_err(out.cpu(), ref) < 1e-5


def test_gemm_identity_asymmetric():
    # A = I with an asymmetric B catches a transposed C write (cdna guide §3)
    n = 64
    A = torch.eye(n)
    B = torch.arange(n * n, dtype=torch.float32).reshape(n, n) % 97
    out = torch.empty(n, n, device=DEV)
    C().gemm(bf(A), True, n, bf(B.t().contiguous()), True, n, out, n, n, n, n, None, False, False)
    assert torch.equal(out.cpu(), B.to(torch.bfloat16).float())


def test_gemm_big_tile_path():
    """Long-K GEMM with >= 512 tiles: the 256x128 three-stage kernel, bias + ReLU epilogue, ragged edges."""
    M, N, K = 16400, 1032, 2056
    A, W, b = torch.randn(M, K), torch.randn(N, K) * 0.05, torch.randn(N)
    out = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    C().gemm(bf(A), True, K, bf(W), True, K, out, N, M, N, K, b.to(DEV), True, False)
    ref = torch.relu(A.to(torch.bfloat16).float() @ W.to(torch.bfloat16).float().t() + b)
    assert rel_err(out.cpu(), ref) < 1e-2


@pytest.fixture
def force_wide():
    C().set_gemm_paths(2)
    yield
    C().set_gemm_paths(-1)


@pytest.mark.parametrize("M,N,K", [(700, 520, 200), (256, 256, 64), (1100, 296, 2056), (4096, 4096, 512)])
def test_gemm_wide_tile_path(M, N, K, force_wide):
    """256x256 wide-tile kernel (forced): ragged M/N/K, bias + ReLU epilogue, bf16 output."""
    torch.manual_seed(5)
    A, W, b = torch.randn(M, K), torch.randn(N, K) * 0.05, torch.randn(N)
    out = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    C().gemm(bf(A), True, K, bf(W), True, K, out, N, M, N, K, b.to(DEV), True, True)
    ref = torch.relu(A.to(torch.bfloat16).float() @ W.to(torch.bfloat16).float().t() + b)
    assert rel_err(out.cpu(), ref) < 1e-2


@pytest.mark.parametrize("case", [(4, 15, 15, 64, 256, 3, 1, 1), (4, 14, 14, 256, 512, 3, 2, 1),
                                  (3, 9, 9, 512, 272, 1, 1, 0)])
def test_conv_wide_tile_path(case, force_wide):
    """Conv fwd, (phased, row-remapped, addend-fused) dgrad and split-K wgrad through the wide tile."""
    N, H, W, Cin, Cout, k, s, p = case
    torch.manual_seed(6)
    x = torch.randn(N, H, W, Cin).to(torch.bfloat16).float().requires_grad_()
    w = (torch.randn(Cout, k, k, Cin) / math.sqrt(Cin * k * k)).to(torch.bfloat16).float().requires_grad_()
    y = _conv_ref(x, w, s, p)
    dy = torch.randn_like(y).to(torch.bfloat16).float()
    y.backward(dy)
    yg = C().conv_fwd(bf(x.detach()), bf(w.detach()), s, p, 1, None, False)
    assert rel_err(yg.cpu(), y.detach()) < 1e-2
    add = torch.randn(N, H, W, Cin).to(torch.bfloat16)
    dx = C().conv_dgrad(bf(dy), bf(w.detach()), H, W, s, p, 1, add.to(DEV))
    assert rel_err(dx.cpu(), x.grad + add.float()) < 1e-2
    # wgrad: MN-major operands (dy^T, im2col(x)^T) with split-K slabs through the wide tile
    dw = C().conv_wgrad(bf(dy), bf(x.detach()), k, k, s, p, 1, True, None)
    assert rel_err(dw.cpu(), w.grad) < 1e-3
    dwb = C().conv_wgrad(bf(dy), bf(x.detach()), k, k, s, p, 1, False, None)
    assert rel_err(dwb.cpu(), w.grad) < 1e-2


@pytest.mark.parametrize("M,N,K,split", [(320, 384, 8192, True), (264, 512, 4160, True), (512, 256, 64, False),
                                         (776, 264, 1032, False)])
@pytest.mark.parametrize("ak,bk", [(True, True), (True, False), (False, True), (False, False)])
def test_gemm_wide_layouts(M, N, K, split, ak, bk, force_wide):
    """Wide tile with every operand major-ness (MN-major halves read with ds_read_b64_tr), fp32
    output, and split-K fp32 slabs + reduction when ``split``."""
    torch.manual_seed(9)
    A = torch.randn(M, K)
    B = torch.randn(K, N)
    a_store = bf(A) if ak else bf(A.t().contiguous())
    b_store = bf(B.t().contiguous()) if bk else bf(B)
    out = torch.empty(M, N, device=DEV, dtype=torch.float32)
    C().gemm(a_store, ak, K if ak else M, b_store, bk, K if bk else N, out, N, M, N, K, None, False, split)
    ref = A.to(torch.bfloat16).float() @ B.to(torch.bfloat16).float()
    assert rel_err(out.cpu(), ref) < 1e-5


@pytest.mark.parametrize("M,N,K", [(1000, 264, 136), (256, 520, 72), (296, 256, 1600), (8, 8, 8), (512, 768, 4096),
                                   (2048, 2048, 1024)])
@pytest.mark.parametrize("ak,bk", [(True, True), (True, False), (False, False)])
@pytest.mark.parametrize("variant", [0, 3, 6, 10, 100, 200])
def test_gemm_pp_variants(M, N, K, ak, bk, variant):
    """Pipelined 256x256 GEMM (gemm_pp.hip) through its lab entry: every operand layout used in training
    (fwd K x K, dgrad K x MN, wgrad MN x MN), ragged M / N / K (rows past the operand and K past the end
    read zero through the buffer descriptors), the plain (0), ping-pong + setprio (3), DMA-first (6),
    two-phase (10) schedules, the persistent tile walk (100) and the 4-wave 128x128-per-wave tile (200,
    K-major x K-major; the other layouts fall back to the default schedule), bias."""
    torch.manual_seed(21)
    A = torch.rand(M, K) * 2 - 1
    B = torch.rand(K, N) * 2 - 1
    bias = torch.rand(N) - 0.5
    a_store = bf(A) if ak else bf(A.t().contiguous())
    b_store = bf(B.t().contiguous()) if bk else bf(B)
    out = torch.full((M, N), float("nan"), device=DEV, dtype=torch.bfloat16)
    C().gemm_pp_lab(a_store, ak, K if ak else M, b_store, bk, K if bk else N, out, N, M, N, K, bf(bias), variant)
    ref = A.to(torch.bfloat16).float() @ B.to(torch.bfloat16).float() + bias.to(torch.bfloat16).float()
    assert torch.isfinite(out).all()
    assert rel_err(out.cpu(), ref) < 1e-2


def test_gemm_pp_matches_wide_kernel_bitwise_fp32_slabs():
    """The pipelined and the 2-stage wide kernel accumulate every output in the same MFMA order over K
    tiles, so with split-K fp32 slabs (no bf16 rounding of partials) both paths give the same fp32 C."""
    M, N, K = 512, 512, 8192
    torch.manual_seed(22)
    A, B = bf(torch.randn(M, K)), bf(torch.randn(N, K))
    outs = []
    for pp in (1, 0):
        C().set_gemm_pp(pp)
        C().set_gemm_paths(2)
        try:
            o = torch.empty(M, N, device=DEV, dtype=torch.float32)
            C().gemm(A, True, K, B, True, K, o, N, M, N, K, None, False, True)
            outs.append(o)
        finally:
            C().set_gemm_paths(-1)
            C().set_gemm_pp(-1)
    ref = A.float().cpu() @ B.float().cpu().t()
    assert rel_err(outs[0].cpu(), ref) < 1e-5 and rel_err(outs[1].cpu(), ref) < 1e-5
    assert rel_err(outs[0], outs[1]) < 1e-6


@pytest.mark.parametrize("M,N,K,f32", [(320, 384, 8192, True), (1024, 1024, 16384, False), (264, 520, 4160, True)])
def test_splitk_fixup_matches_reduce_launch(M, N, K, f32):
    """Split-K weight-gradient layout (MN-major x MN-major) on the pipelined tile: the in-kernel fix-up (the
    last split of each tile sums the slabs) against the separate reduce launch and fp32; the fix-up sums in
    split order whoever arrives last, so repeated launches (tickets re-zeroed by each launch) are bitwise
    identical."""
    torch.manual_seed(31)
    A, B = torch.randn(K, M), torch.randn(K, N)
    Ab, Bb = bf(A), bf(B)
    ref = A.to(torch.bfloat16).float().t() @ B.to(torch.bfloat16).float()
    outs = {}
    C().set_gemm_paths(2)
    try:
        for fix in (0, 1):
            C().set_splitk_fixup(fix)
            runs = []
            for _ in range(3 if fix else 1):
                o = torch.full((M, N), float("nan"), device=DEV, dtype=torch.float32 if f32 else torch.bfloat16)
                for _ in range(5):  # back-to-back launches reuse the ticket pool
                    C().gemm(Ab, False, M, Bb, False, N, o, N, M, N, K, None, False, True)
                runs.append(o.clone())
            outs[fix] = runs
    finally:
        C().set_splitk_fixup(-1)
        C().set_gemm_paths(-1)
    tol = 1e-5 if f32 else 1e-2
    for fix, runs in outs.items():
        assert torch.isfinite(runs[0].float()).all(), fix
        assert rel_err(runs[0].float().cpu(), ref) < tol, (fix, rel_err(runs[0].float().cpu(), ref))
    assert all(torch.equal(outs[1][0], r) for r in outs[1][1:])
    assert rel_err(outs[0][0].float(), outs[1][0].float()) < (1e-6 if f32 else 1e-2)


@pytest.mark.parametrize("fix", [1, 0])
@pytest.mark.parametrize("T,Nout,Kin", [(4096, 1024, 1024), (2048, 512, 768), (3000, 296, 264), (64, 64, 64)])
def test_gemm_wgrad_db_fused(T, Nout, Kin, fix):
    """Linear weight gradient with the bias gradient folded in: dW = dY^T X and db = sum_t dY
    from one pipelined GEMM (split-K: fp32 atomics + cast; no split: direct bf16 store); small shapes
    that do not take the 256x256 path report False and leave db to the caller."""
    torch.manual_seed(23)
    dy = torch.randn(T, Nout) * 0.1
    x = torch.randn(T, Kin)
    dw = torch.empty(Nout, Kin, device=DEV, dtype=torch.bfloat16)
    db = torch.full((Nout,), float("nan"), device=DEV, dtype=torch.bfloat16)
    C().set_splitk_fixup(fix)  # split-K: the in-kernel fix-up (1) or the reduce launch (0)
    try:
        done = C().gemm_wgrad_db(bf(dy), bf(x), dw, db)
    finally:
        C().set_splitk_fixup(-1)
    dyb, xb = dy.to(torch.bfloat16).float(), x.to(torch.bfloat16).float()
    assert rel_err(dw.cpu(), dyb.t() @ xb) < 1e-2
    if (T, Nout, Kin) == (4096, 1024, 1024):
        assert done  # 16 output tiles: split-K on the pipelined tile
    if done:
        assert rel_err(db.cpu(), dyb.sum(0)) < 1e-2
    else:
        assert torch.isnan(db.float()).all()


def _gelu_grad_ref(h):
    k0, k1 = 0.7978845608028654, 0.044715
    t = torch.tanh(k0 * (h + k1 * h ** 3))
    return 0.5 * (1 + t) + 0.5 * h * (1 - t * t) * k0 * (1 + 3 * k1 * h * h)


@pytest.mark.parametrize("M,N,K", [(300, 520, 136), (4096, 1024, 512), (1000, 4096, 256)])
@pytest.mark.parametrize("wide", [-1, 0, 2])
def test_gemm_gelu_epilogues(M, N, K, wide):
    """GEMM with the fused GELU epilogues (128 / 256x128 / 256x256 tiles): act 1 writes
    gelu(A B + bias) and the pre-activation, act 2 multiplies A B by gelu'(aux)."""
    torch.manual_seed(11)
    A, W, b = torch.randn(M, K), torch.randn(N, K) * 0.05, torch.randn(N)
    C().set_gemm_paths(wide)
    try:
        g = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
        h = torch.empty_like(g)
        C().gemm_act(bf(A), True, K, bf(W), True, K, g, N, M, N, K, b.to(DEV), 1, h)
        pre = A.to(torch.bfloat16).float() @ W.to(torch.bfloat16).float().t() + b
        assert rel_err(h.cpu(), pre) < 1e-2
        assert rel_err(g.cpu(), F.gelu(pre, approximate="tanh")) < 1e-2
        # backward form: dH = (dY W) * gelu'(h), dY [M, K'] K-major, W [K', N] read MN-major
        Kp = 128
        dY, W2 = torch.randn(M, Kp), torch.randn(Kp, N) * 0.05
        dh = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
        C().gemm_act(bf(dY), True, Kp, bf(W2), False, N, dh, N, M, N, Kp, None, 2, h)
        ref = (dY.to(torch.bfloat16).float() @ W2.to(torch.bfloat16).float()) * _gelu_grad_ref(h.cpu().float())
        assert rel_err(dh.cpu(), ref) < 1e-2
    finally:
        C().set_gemm_paths(-1)


def test_mlp_gelu_fused_matches_unfused(monkeypatch):
    """ops.mlp_gelu (GELU inside the GEMM epilogues, PDA_MLP_FUSED=1) == linear -> gelu_tanh -> linear,
    values and all five gradients."""
    from pytorchdistributed_amd import ops
    from pytorchdistributed_amd.ops.act import gelu_tanh
    from pytorchdistributed_amd.ops.linear import mlp_fused_ok

    monkeypatch.setenv("PDA_MLP_FUSED", "1")

    torch.manual_seed(12)
    d, f, T = 256, 1024, 2 * 384
    x0 = torch.randn(T, d, device=DEV).to(torch.bfloat16)
    p0 = [torch.randn(f, d, device=DEV) * 0.05, torch.randn(f, device=DEV) * 0.1,
          torch.randn(d, f, device=DEV) * 0.03, torch.randn(d, device=DEV) * 0.1]
    p0 = [t.to(torch.bfloat16) for t in p0]
    dy = torch.randn(T, d, device=DEV).to(torch.bfloat16)
    assert mlp_fused_ok(x0, p0[0], p0[2])
    outs, grads = [], []
    for fused in (True, False):
        x = x0.clone().requires_grad_()
        ps = [t.clone().requires_grad_() for t in p0]
        if fused:
            y = ops.mlp_gelu(x.view(2, T // 2, d), *ps)
        else:
            y = ops.linear(gelu_tanh(ops.linear(x.view(2, T // 2, d), ps[0], ps[1])), ps[2], ps[3])
        y.backward(dy.view(2, T // 2, d))
        torch.cuda.synchronize()
        outs.append(y.detach().float().reshape(T, d))
        grads.append([x.grad.float()] + [p.grad.float() for p in ps])
    assert rel_err(outs[0], outs[1]) < 1e-2
    for a, b in zip(grads[0], grads[1]):
        assert rel_err(a, b) < 2e-2


def test_gemm_bias_relu_bf16_out():
    M, N, K = 257, 136, 96
    A, W, b = torch.randn(M, K), torch.randn(N, K), torch.randn(N)
    out = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    C().gemm(bf(A), True, K, bf(W), True, K, out, N, M, N, K, b.to(DEV), True, False)
    ref = torch.relu(A.to(torch.bfloat16).float() @ W.to(torch.bfloat16).float().t() + b)
    assert rel_err(out.cpu(), ref) < 1e-2


# ----------------------------------------------------------------------------- conv
CONV_CASES = [
    # N, H, W, C, Cout, k, stride, pad
    (2, 16, 16, 64, 64, 1, 1, 0),
    (2, 16, 16, 64, 128, 3, 1, 1),
    (2, 15, 15, 128, 64, 3, 2, 1),
    (2, 16, 16, 256, 512, 1, 2, 0),
    (2, 32, 32, 8, 64, 7, 2, 3),
    (3, 7, 7, 512, 2048, 1, 1, 0),
    (1, 9, 11, 24, 40, 3, 1, 1),
    (8, 28, 28, 64, 64, 1, 1, 0),       # deep split-K wgrad, 64-row tiles
    (2, 14, 14, 64, 128, 3, 2, 1),      # even size, stride-2 phases
    (2, 13, 10, 32, 48, 3, 3, 1),       # stride 3: 9 phases, some with no taps
    (2, 12, 12, 32, 64, 3, 1, 2, 2),    # dilation 2 (stride-1 phased dgrad)
    (2, 13, 13, 32, 64, 3, 2, 2, 2),    # dilation 2 + stride 2: folded dgrad
    (16, 56, 56, 64, 256, 1, 1, 0),     # >= 256 tiles: 256x128 three-stage kernel (fwd)
    (16, 56, 56, 256, 64, 1, 1, 0),     # ... and for the dgrad (with and without the fused addend)
    (8, 57, 57, 128, 128, 3, 1, 1),     # big tiles with ragged M and 3x3 gathers
    (6, 7, 7, 128, 128, 3, 1, 1),       # 3x3 halo path: 128-pixel tiles spanning 3 images
    (2, 28, 28, 128, 128, 3, 1, 1),     # 3x3 halo path (layer2 shape), 2 source-channel chunks
    (3, 9, 13, 64, 128, 3, 1, 1),       # halo fwd (its dgrad, 64 out channels, stays implicit GEMM)
    (2, 5, 30, 64, 64, 3, 1, 1),        # all-taps 3x3 wgrad: 2 rows per K-step, a 1-row last group
    (3, 4, 56, 128, 64, 3, 1, 1),       # all-taps 3x3 wgrad: 1 row per K-step, 2 input-channel blocks
    (2, 35, 35, 16, 64, 4, 1, 0),       # stem (4x4 valid over the space-to-depth image): band wgrad kernel
    (2, 20, 40, 16, 128, 4, 1, 0),      # stem wgrad with two output-channel tiles, rows of 37 pixels
    (2, 115, 115, 16, 64, 4, 1, 0),     # the ResNet-50 stem shape (112-pixel rows padded to 128)
    (4, 14, 14, 1024, 256, 1, 1, 0),    # 1x1 dgrad on the transposed weight (K-major B), wide tile
    # 3x3 weight gradient v2 (conv3x3_wg_kernel): every ResNet-50 3x3 layer shape (small batch), the
    # strided ones included, 64- and 128-channel output tiles, ragged last row groups
    (3, 56, 56, 64, 64, 3, 1, 1),       # 2 rows (112 px) per K-step, 64-channel tile (pixel-half parities)
    # persistent 64 -> 64 3x3 fwd / dgrad (conv3x3_res64_kernel): > 256 tiles so workgroups walk several
    # tiles with the next band in flight; bands crossing image boundaries; ragged last tile
    (16, 56, 56, 64, 64, 3, 1, 1),
    (70, 17, 29, 64, 64, 3, 1, 1),
    (2, 28, 28, 128, 128, 3, 1, 1),     # 4 rows per step, 128-channel tile, 2 ci blocks
    (3, 14, 14, 256, 256, 3, 1, 1),     # 9 + 5 rows per image
    (4, 7, 7, 512, 512, 3, 1, 1),       # one image per step (49 px)
    (2, 56, 56, 128, 128, 3, 2, 1),     # stride 2: 2 output rows, a 5-row band of 58 pixels
    (2, 28, 28, 256, 256, 3, 2, 1),
    (3, 14, 14, 512, 512, 3, 2, 1),
    (2, 9, 13, 64, 192, 3, 2, 1),       # odd sizes, 64-channel output tiles x 3
]


def _conv_ref(x, w, stride, pad, dil=1):
    return F.conv2d(x.permute(0, 3, 1, 2), w.permute(0, 3, 1, 2), None, stride, pad, dil).permute(0, 2, 3, 1)


@pytest.mark.parametrize("case", CONV_CASES)
def test_conv_fwd_dgrad_wgrad(case):
    N, H, W, Cin, Cout, k, s, p = case[:8]
    d = case[8] if len(case) > 8 else 1
    torch.manual_seed(1)
    x = torch.randn(N, H, W, Cin).to(torch.bfloat16).float().requires_grad_()
    w = (torch.randn(Cout, k, k, Cin) / math.sqrt(Cin * k * k)).to(torch.bfloat16).float().requires_grad_()
    y = _conv_ref(x, w, s, p, d)
    dy = torch.randn_like(y).to(torch.bfloat16).float()
    y.backward(dy)
    yg = C().conv_fwd(bf(x.detach()), bf(w.detach()), s, p, d, None, False)
    assert yg.shape == y.shape
    assert rel_err(yg.cpu(), y.detach()) < 1e-2
    dx = C().conv_dgrad(bf(dy), bf(w.detach()), H, W, s, p, d, None)
    assert rel_err(dx.cpu(), x.grad) < 1e-2
    add = torch.randn(N, H, W, Cin).to(torch.bfloat16)
    dx2 = C().conv_dgrad(bf(dy), bf(w.detach()), H, W, s, p, d, add.to(DEV))  # fused gradient accumulation
    assert rel_err(dx2.cpu(), x.grad + add.float()) < 1e-2
    # bit-masked addend (a bottleneck's residual gradient dz * relu_mask read from dz + the 1-bit mask)
    mask = torch.rand(N, H, W, Cin) > 0.5
    bits = (mask.reshape(-1, 8).to(torch.uint8) << torch.arange(8, dtype=torch.uint8)).sum(1).to(torch.uint8)
    dx3 = C().conv_dgrad(bf(dy), bf(w.detach()), H, W, s, p, d, add.to(DEV), bits.to(DEV))
    assert rel_err(dx3.cpu(), x.grad + add.float() * mask) < 1e-2
    dw = C().conv_wgrad(bf(dy), bf(x.detach()), k, k, s, p, d, True, None)
    assert rel_err(dw.cpu(), w.grad) < 1e-3
    dwb = C().conv_wgrad(bf(dy), bf(x.detach()), k, k, s, p, d, False, None)
    assert rel_err(dwb.cpu(), w.grad) < 1e-2


@pytest.mark.parametrize("case", [(2, 16, 16, 64, 64, 1, 1, 0), (3, 15, 15, 32, 136, 3, 2, 1), (1, 7, 7, 64, 2048, 1, 1, 0),
                                  (8, 28, 28, 64, 256, 1, 1, 0), (4, 14, 14, 256, 512, 3, 1, 1),
                                  (2, 35, 35, 16, 64, 4, 1, 0), (3, 115, 115, 16, 64, 4, 1, 0)])  # stem kernels
@pytest.mark.parametrize("wide", [-1, 0, 2])
def test_conv_fwd_epilogue_bn_sums(case, wide):
    """BN statistics accumulated by the conv epilogue (128-tile, wide-tile and auto paths) == sums over
    the stored bf16 output; the BN finalize that consumes the table leaves it zeroed."""
    N, H, W, Cin, Cout, k, s, p = case
    torch.manual_seed(4)
    x = torch.randn(N, H, W, Cin).to(torch.bfloat16)
    w = (torch.randn(Cout, k, k, Cin) / math.sqrt(Cin * k * k)).to(torch.bfloat16)
    shift = torch.randn(Cout) * 0.1
    rows = 5  # odd row count: tiles wrap onto rows unevenly
    table = torch.zeros(rows, 2, Cout, device=DEV)
    C().set_gemm_paths(wide)
    try:
        y = C().conv_fwd_stats(x.to(DEV), w.to(DEV), s, p, 1, shift.to(DEV), table)
        y_plain = C().conv_fwd(x.to(DEV), w.to(DEV), s, p, 1, None, False)
    finally:
        C().set_gemm_paths(-1)
    assert torch.equal(y, y_plain)
    d = y.float().cpu().reshape(-1, Cout) - shift
    ref = torch.stack([d.sum(0), (d * d).sum(0)])
    assert rel_err(table.sum(0).cpu(), ref) < 1e-4
    # BN from the epilogue sums == BN with its own statistics pass; the finalize re-zeroes the table
    g, b = torch.rand(Cout) + 0.5, torch.randn(Cout)
    rm1, rv1 = shift.clone().to(DEV), torch.ones(Cout, device=DEV)
    rm2, rv2 = shift.clone().to(DEV), torch.ones(Cout, device=DEV)
    nbt = torch.zeros((), dtype=torch.long, device=DEV)
    ya, ma, ia, ssa, _ = C().bn_fwd_train_sums(y, table, rm1.clone(), None, g.to(DEV), b.to(DEV), rm1, rv1, 0.1,
                                               1e-5, True, False, nbt)
    assert not table.any()
    yb, mb, ib, ssb, _ = C().bn_fwd_train(y, None, g.to(DEV), b.to(DEV), rm2, rv2, 0.1, 1e-5, True, False, nbt)
    assert nbt.item() == 2  # num_batches_tracked is bumped by each training finalize
    assert rel_err(ma.cpu(), mb.cpu()) < 1e-4 and rel_err(ia.cpu(), ib.cpu()) < 1e-4
    assert rel_err(ya.cpu(), yb.cpu()) < 1e-2 and rel_err(rv1.cpu(), rv2.cpu()) < 1e-4


# ----------------------------------------------------------------------------- batch norm
@pytest.mark.parametrize("shape", [(4, 8, 8, 64), (2, 7, 7, 2048), (3, 5, 5, 200), (2, 56, 56, 256),
                                   (64, 28, 28, 64),
                                   # partial last wave iteration (vectors % 256 != 0) with 1 and 2
                                   # coefficient sets per lane
                                   (3, 7, 7, 64), (1, 3, 7, 128), (1, 3, 5, 1024)])
@pytest.mark.parametrize("relu,res", [(False, False), (True, False), (True, True)])
def test_batchnorm_train(shape, relu, res):
    torch.manual_seed(2)
    Cc = shape[-1]
    x = (torch.randn(shape) * 3 + 1.5).to(torch.bfloat16).float()
    r = torch.randn(shape).to(torch.bfloat16).float() if res else None
    g = torch.rand(Cc) + 0.5
    b = torch.randn(Cc)
    rm, rv = torch.zeros(Cc), torch.ones(Cc)
    xr = x.clone().requires_grad_()
    gr, br = g.clone().requires_grad_(), b.clone().requires_grad_()
    rr = r.clone().requires_grad_() if res else None
    y = F.batch_norm(xr.reshape(-1, Cc), rm, rv, gr, br, True, 0.1, 1e-5).reshape(shape)
    if res:
        y = y + rr
    if relu:
        y = torch.relu(y)
    dy = torch.randn(shape).to(torch.bfloat16).float()
    y.backward(dy)

    rmg, rvg = torch.zeros(Cc, device=DEV), torch.ones(Cc, device=DEV)
    yg, mean, invstd, ss, bits = C().bn_fwd_train(bf(x), bf(r) if res else None, g.to(DEV), b.to(DEV), rmg, rvg,
                                                  0.1, 1e-5, relu, relu, None)
    assert rel_err(yg.cpu(), y.detach()) < 1e-2
    assert rel_err(rmg.cpu(), rm) < 1e-4 and rel_err(rvg.cpu(), rv) < 1e-4
    if relu:  # bit j of byte v is the ReLU mask of element 8v+j
        want = (yg.reshape(-1, 8).cpu().float() > 0).to(torch.int32)
        got = torch.stack([(bits.cpu().to(torch.int32) >> j) & 1 for j in range(8)], 1)
        assert torch.equal(got, want)
    # the ReLU mask from the saved output, from its bit mask, and (no residual) recomputed from x and
    # the saved scale/shift
    modes = ["y"] + (["bits"] if relu else []) + (["ss"] if relu and not res else [])
    for mode in modes:
        saved = {"y": yg, "bits": bits, "ss": None}[mode]
        dx, dres, dgamma, dbeta = C().bn_bwd(bf(dy), bf(x), saved, ss if mode == "ss" else None, mean,
                                             invstd, g.to(DEV), relu, res, None, None)
        assert rel_err(dx.cpu(), xr.grad) < 2e-2
        assert rel_err(dgamma.cpu(), gr.grad) < 1e-2
        assert rel_err(dbeta.cpu(), br.grad) < 1e-2
        if res:
            assert rel_err(dres.cpu(), rr.grad) < 1e-2


def test_batchnorm_bwd_fused_finalize_reuse():
    """The in-launch finalize's persistent [R][2][C] table and ticket must be left zero by every call:
    back-to-back backwards of different widths (table rows R = 8192 / C, clamped to 8..128) on the
    default stream and on a second stream (its own table) all match the fp32 reference."""
    torch.manual_seed(5)
    cases = []
    for shape in [(4, 6, 6, 64), (2, 7, 7, 2048), (3, 5, 5, 200), (4, 6, 6, 64), (1, 9, 9, 1024)]:
        Cc = shape[-1]
        x = (torch.randn(shape) * 2 + 0.5).to(torch.bfloat16).float()
        g = torch.rand(Cc) + 0.5
        dy = torch.randn(shape).to(torch.bfloat16).float()
        xr, gr, br = x.clone().requires_grad_(), g.clone().requires_grad_(), torch.zeros(Cc, requires_grad=True)
        y = F.batch_norm(xr.reshape(-1, Cc), None, None, gr, br, True, 0.1, 1e-5).reshape(shape)
        y.backward(dy)
        cases.append((x, g, dy, xr.grad, gr.grad, br.grad))
    side = torch.cuda.Stream()
    prev = C().bn_bwd_fused_max_c()
    C().set_bn_bwd_fused_max_c(2048)
    try:
        _fused_finalize_cases(cases, side)
    finally:
        C().set_bn_bwd_fused_max_c(prev)


def _fused_finalize_cases(cases, side):
    for rep in range(3):
        for i, (x, g, dy, dx_ref, dg_ref, db_ref) in enumerate(cases):
            Cc = x.shape[-1]
            stream = side if (rep + i) % 2 else torch.cuda.current_stream()
            with torch.cuda.stream(stream):
                _, mean, invstd, _, _ = C().bn_fwd_train(bf(x), None, g.to(DEV), torch.zeros(Cc, device=DEV),
                                                         torch.zeros(Cc, device=DEV), torch.ones(Cc, device=DEV),
                                                         0.1, 1e-5, False, False, None)
                dx, _, dgamma, dbeta = C().bn_bwd(bf(dy), bf(x), None, None, mean, invstd, g.to(DEV), False, False,
                                                  None, None)
            torch.cuda.synchronize()
            assert rel_err(dx.cpu(), dx_ref) < 2e-2, (rep, i)
            assert rel_err(dgamma.cpu(), dg_ref) < 1e-2, (rep, i)
            assert rel_err(dbeta.cpu(), db_ref) < 1e-2, (rep, i)


def test_batchnorm_eval():
    x = torch.randn(2, 4, 4, 64)
    g, b = torch.rand(64) + 0.5, torch.randn(64)
    rm, rv = torch.randn(64), torch.rand(64) + 0.5
    y = C().bn_fwd_eval(bf(x), None, g.to(DEV), b.to(DEV), rm.to(DEV), rv.to(DEV), 1e-5, True)
    ref = torch.relu(F.batch_norm(x.to(torch.bfloat16).float().reshape(-1, 64), rm, rv, g, b, False, 0.1, 1e-5))
    assert rel_err(y.cpu(), ref.reshape(x.shape)) < 1e-2


# ----------------------------------------------------------------------------- pooling
@pytest.mark.parametrize("H,W,k,s,p", [(17, 16, 3, 2, 1), (16, 17, 3, 2, 1), (56, 56, 3, 2, 1), (7, 7, 3, 2, 1),
                                      (1, 2, 3, 2, 1), (12, 13, 2, 2, 0), (9, 9, 3, 1, 1)])
def test_maxpool_fwd_bwd(H, W, k, s, p):
    """3x3/2/1 backward runs the 2x2-block gather kernel, the others the generic gather."""
    torch.manual_seed(3)
    x = torch.randn(2, H, W, 64).to(torch.bfloat16).float().requires_grad_()
    y = F.max_pool2d(x.permute(0, 3, 1, 2), k, s, p).permute(0, 2, 3, 1)
    dy = torch.randn_like(y).to(torch.bfloat16).float()
    y.backward(dy)
    yg, idx = C().maxpool_fwd(bf(x.detach()), k, s, p)
    assert torch.equal(yg.cpu().float(), y.detach())
    dx = C().maxpool_bwd(bf(dy), idx, H, W, k, s, p)
    assert rel_err(dx.cpu(), x.grad) < 1e-2


def test_avgpool_fwd_bwd():
    x = torch.randn(3, 7, 7, 128)
    y = C().avgpool_fwd(bf(x), False)
    assert rel_err(y.cpu(), x.to(torch.bfloat16).float().mean((1, 2))) < 1e-4
    dy = torch.randn(3, 128)
    dx = C().avgpool_bwd(dy.to(DEV), 7, 7)
    assert rel_err(dx.cpu(), (dy / 49)[:, None, None, :].expand(3, 7, 7, 128)) < 1e-2


# ----------------------------------------------------------------------------- cross entropy
@pytest.mark.parametrize("M,Cc,dtype", [(64, 1000, torch.float32), (33, 1000, torch.bfloat16), (8, 50257, torch.bfloat16),
                                        (32, 1, torch.float32)])
@pytest.mark.parametrize("kind", ["index", "prob", "smooth"])
def test_cross_entropy(M, Cc, dtype, kind):
    from pytorchdistributed_amd.ops import cross_entropy

    torch.manual_seed(4)
    logits = (torch.randn(M, Cc) * 3).to(dtype).float()
    if kind == "prob":
        tgt = torch.rand(M, Cc) if Cc > 1 else torch.rand(M, 1)
        ls = 0.0
    else:
        tgt = torch.randint(0, Cc, (M,))
        if M > 3:
            tgt[3] = -100
        ls = 0.1 if kind == "smooth" else 0.0
    lr = logits.clone().requires_grad_()
    ref = F.cross_entropy(lr, tgt, label_smoothing=ls)
    ref.backward()
    lg = logits.to(DEV, dtype).requires_grad_()
    out = cross_entropy(lg, tgt.to(DEV), label_smoothing=ls)
    out.backward()
    assert abs(out.item() - ref.item()) < 1e-3 * max(1.0, abs(ref.item()))
    assert rel_err(lg.grad.cpu(), lr.grad) < (1e-4 if dtype == torch.float32 else 2e-2) or lr.grad.norm() < 1e-12


# ----------------------------------------------------------------------------- optimizers
def test_sgd_flat_matches_torch():
    torch.manual_seed(5)
    p0 = torch.randn(1003)
    grads = [torch.randn(1003) for _ in range(3)]
    ref = p0.clone().requires_grad_()
    opt = torch.optim.SGD([ref], lr=0.1, momentum=0.9, weight_decay=1e-3, nesterov=True)
    master = p0.clone().to(DEV)
    mom = torch.zeros(1003, device=DEV)
    pb = torch.empty(1003, device=DEV, dtype=torch.bfloat16)
    for i, g in enumerate(grads):
        ref.grad = g.clone()
        opt.step()
        C().sgd_step(master, pb, g.to(DEV), mom, 0.1, 0.9, 0.0, 1e-3, True, i == 0, 1.0, None, None)
    assert rel_err(master.cpu(), ref.detach()) < 1e-6
    assert rel_err(pb.cpu(), ref.detach()) < 1e-2


@pytest.mark.parametrize("adamw", [False, True])
def test_adam_matches_torch(adamw):
    torch.manual_seed(6)
    p0 = torch.randn(517)
    ref = p0.clone().requires_grad_()
    cls = torch.optim.AdamW if adamw else torch.optim.Adam
    opt = cls([ref], lr=1e-2, betas=(0.9, 0.99), eps=1e-8, weight_decay=0.01)
    master = p0.clone().to(DEV)
    m, v = torch.zeros(517, device=DEV), torch.zeros(517, device=DEV)
    for t in range(1, 4):
        g = torch.randn(517).to(torch.bfloat16).float()
        ref.grad = g.clone()
        opt.step()
        C().adam_step(master, None, g.to(DEV, torch.bfloat16), m, v, 1e-2, 0.9, 0.99, 1e-8, 0.01, adamw, t,
                      1.0, None, None, None)
    assert rel_err(master.cpu(), ref.detach()) < 1e-5


def test_grad_norm():
    g = torch.randn(10001)
    out = C().grad_norm(g.to(DEV, torch.bfloat16), 0.5, 1.0).cpu()
    n = g.to(torch.bfloat16).float().norm() * 0.5
    assert abs(out[0].item() - n.item()) / n.item() < 1e-4
    assert abs(out[1].item() - min(1.0, 1.0 / (n.item() + 1e-6))) < 1e-5


# ----------------------------------------------------------------------------- norms / activations / simt
@pytest.mark.parametrize("rms", [False, True])
@pytest.mark.parametrize("D,rows", [(64, 37), (1024, 37), (1024, 2500), (1600, 37), (4096, 300), (8192, 130)])
def test_rownorm(rms, D, rows):
    from pytorchdistributed_amd.ops import layer_norm, rms_norm

    torch.manual_seed(7)
    x = (torch.randn(rows, D) * 2 + 0.3).to(torch.bfloat16).float()
    g = torch.rand(D) + 0.5
    b = torch.randn(D)
    xr = x.clone().requires_grad_()
    gr, br = g.clone().requires_grad_(), b.clone().requires_grad_()
    if rms:
        y = xr * torch.rsqrt(xr.pow(2).mean(-1, keepdim=True) + 1e-6) * gr
    else:
        y = F.layer_norm(xr, (D,), gr, br, 1e-5)
    dy = torch.randn_like(y)
    y.backward(dy)
    xg = x.to(DEV, torch.bfloat16).requires_grad_()
    gg = g.to(DEV).requires_grad_()
    bg = b.to(DEV).requires_grad_()
    yg = rms_norm(xg, gg, 1e-6) if rms else layer_norm(xg, gg, bg, 1e-5)
    yg.backward(dy.to(DEV, torch.bfloat16))
    assert rel_err(yg.cpu(), y.detach()) < 1e-2
    assert rel_err(xg.grad.cpu(), xr.grad) < 2e-2
    assert rel_err(gg.grad.cpu(), gr.grad) < 2e-2
    if not rms:
        assert rel_err(bg.grad.cpu(), br.grad) < 2e-2


@pytest.mark.parametrize("rms", [False, True])
@pytest.mark.parametrize("D,rows", [(64, 37), (1024, 2500), (1600, 37), (4096, 300)])
def test_add_norm_train(rms, D, rows):
    """Residual add fused into the norm, with autograd: h = x + r and norm(h) forward; backward
    dx = dr = norm_bwd(dn) + dh (the residual stream's own gradient added in the dx kernel)."""
    from pytorchdistributed_amd.ops import add_norm_train

    torch.manual_seed(8)
    x = (torch.randn(rows, D) * 2 + 0.3).to(torch.bfloat16).float()
    r = torch.randn(rows, D).to(torch.bfloat16).float()
    g = (torch.rand(D) + 0.5).to(torch.bfloat16).float()
    b = torch.randn(D).to(torch.bfloat16).float()
    xr, rr = x.clone().requires_grad_(), r.clone().requires_grad_()
    gr, br = g.clone().requires_grad_(), b.clone().requires_grad_()
    h = (xr + rr).to(torch.bfloat16).float()  # the fused kernel rounds h to bf16 like a separate add
    n = h * torch.rsqrt(h.pow(2).mean(-1, keepdim=True) + 1e-6) * gr if rms else F.layer_norm(h, (D,), gr, br, 1e-5)
    dh, dn = torch.randn_like(h), torch.randn_like(n)
    torch.autograd.backward([h, n], [dh, dn])
    xg, rg = x.to(DEV, torch.bfloat16).requires_grad_(), r.to(DEV, torch.bfloat16).requires_grad_()
    gg = g.to(DEV, torch.bfloat16).requires_grad_()
    bg = b.to(DEV, torch.bfloat16).requires_grad_()
    hg, ng = add_norm_train(xg, rg, gg, None if rms else bg, 1e-6 if rms else 1e-5, rms=rms)
    torch.autograd.backward([hg, ng], [dh.to(DEV, torch.bfloat16), dn.to(DEV, torch.bfloat16)])
    assert rel_err(hg.cpu(), h.detach()) < 1e-2
    assert rel_err(ng.cpu(), n.detach()) < 1e-2
    assert rel_err(xg.grad.cpu(), xr.grad) < 2e-2
    assert rel_err(rg.grad.cpu(), rr.grad) < 2e-2
    assert rel_err(gg.grad.cpu(), gr.grad) < 2e-2
    if not rms:
        assert rel_err(bg.grad.cpu(), br.grad) < 2e-2


@pytest.mark.parametrize("rows,cols", [(1, 8), (37, 64), (5000, 1024), (300, 1600), (64, 50304), (33, 5)])
def test_colsum(rows, cols):
    x = torch.randn(rows, cols)
    for dt in (torch.float32, torch.bfloat16):
        xd = x.to(dt)
        out = C().colsum(xd.to(DEV)).cpu()
        assert rel_err(out, xd.float().sum(0)) < 1e-5


def test_activations():
    from pytorchdistributed_amd.ops import gelu_tanh, relu, swiglu

    x = torch.randn(33, 64)
    for fn, ref in [(relu, torch.relu), (gelu_tanh, lambda t: F.gelu(t, approximate="tanh"))]:
        xr = x.clone().requires_grad_()
        y = ref(xr)
        y.backward(torch.ones_like(y))
        xg = x.to(DEV).requires_grad_()
        yg = fn(xg)
        yg.backward(torch.ones_like(yg))
        assert rel_err(yg.cpu(), y.detach()) < 1e-5
        assert rel_err(xg.grad.cpu(), xr.grad) < 1e-5
    gu = torch.randn(5, 128)
    gr = gu.clone().requires_grad_()
    g_, u_ = gr.chunk(2, -1)
    y = F.silu(g_) * u_
    y.backward(torch.ones_like(y))
    gg = gu.to(DEV).requires_grad_()
    yg = swiglu(gg)
    yg.backward(torch.ones_like(yg))
    assert rel_err(yg.cpu(), y.detach()) < 1e-5
    assert rel_err(gg.grad.cpu(), gr.grad) < 1e-5


@pytest.mark.parametrize("M,N,K", [(32, 1, 20), (16, 20, 10), (100, 37, 333)])
def test_simt_gemm_fp32(M, N, K):
    A, B = torch.randn(M, K), torch.randn(K, N)
    out = torch.empty(M, N, device=DEV)
    C().simt_gemm(A.to(DEV), K, 1, B.to(DEV), N, 1, out, N, 1, M, N, K, None, False, 0.0)
    assert rel_err(out.cpu(), A @ B) < 1e-5


def test_linear_op_all_paths():
    from pytorchdistributed_amd.ops import linear

    for dtype, fin, fout in [(torch.bfloat16, 64, 136), (torch.float32, 20, 1), (torch.bfloat16, 10, 20)]:
        torch.manual_seed(8)
        x = torch.randn(50, fin).to(dtype).float()
        w = (torch.randn(fout, fin) * 0.1).to(dtype).float()
        b = torch.randn(fout).to(dtype).float()
        xr, wr, br = (t.clone().requires_grad_() for t in (x, w, b))
        y = torch.relu(F.linear(xr, wr, br))
        y.backward(torch.ones_like(y))
        xg, wg, bg = (t.to(DEV, dtype).requires_grad_() for t in (x, w, b))
        yg = linear(xg, wg, bg, relu=True)
        yg.backward(torch.ones_like(yg))
        tol = 1e-5 if dtype == torch.float32 else 2e-2
        for a, r in [(yg, y), (xg.grad, xr.grad), (wg.grad, wr.grad), (bg.grad, br.grad)]:
            assert rel_err(a.cpu(), r.detach()) < tol


@pytest.mark.parametrize("fused_db", ["1", "0"])
def test_linear_gemm_native(fused_db, monkeypatch):
    """Plain bf16 Linear on the native MFMA kernels (no vendor-library path), fwd + bwd vs fp32, with the
    bias gradient from the weight-gradient GEMM (PDA_WGRAD_DB_FUSED=1) and from the column-sum kernel."""
    from pytorchdistributed_amd.ops import linear

    monkeypatch.setenv("PDA_WGRAD_DB_FUSED", fused_db)
    torch.manual_seed(9)
    x = torch.randn(300, 256).to(torch.bfloat16).float()
    w = (torch.randn(136, 256) * 0.05).to(torch.bfloat16).float()
    b = torch.randn(136).to(torch.bfloat16).float()
    xr, wr, br = (t.clone().requires_grad_() for t in (x, w, b))
    y = F.linear(xr, wr, br)
    dy = torch.randn_like(y).to(torch.bfloat16).float()
    y.backward(dy)
    xg, wg, bg = (t.to(DEV, torch.bfloat16).requires_grad_() for t in (x, w, b))
    yg = linear(xg, wg, bg)
    yg.backward(dy.to(DEV, torch.bfloat16))
    for a, r in [(yg, y), (xg.grad, xr.grad), (wg.grad, wr.grad), (bg.grad, br.grad)]:
        assert rel_err(a.cpu(), r.detach()) < 2e-2


def test_synth_fill_statistics():
    t = torch.empty(1 << 20, device=DEV)
    C().fill_random(t, 7, 0, 1, 0.0, 1.0)
    assert abs(t.mean().item()) < 0.01 and abs(t.std().item() - 1) < 0.01
    t2 = torch.empty(1 << 20, device=DEV)
    C().fill_random(t2, 7, 0, 1, 0.0, 1.0)
    assert torch.equal(t, t2)
    i = torch.empty(100000, device=DEV, dtype=torch.long)
    C().fill_randint(i, 1, 0, 0, 1000)
    assert i.min().item() >= 0 and i.max().item() < 1000


@pytest.mark.parametrize("wide", [0, 2])
@pytest.mark.parametrize("case", [(4, 28, 28, 256, 64, 1, 1, 0), (2, 14, 14, 512, 256, 3, 1, 1)])
def test_conv_dgrad_masked_addend_paths(case, wide):
    """dx = dgrad + addend * mask on the 128-tile and the wide 256x256-tile epilogues (the bottleneck's
    conv1 dgrad joining the residual gradient dz * relu_mask)."""
    N, H, W, Cin, Cout, k, s, p = case
    torch.manual_seed(3)
    w = (torch.randn(Cout, k, k, Cin) / math.sqrt(Cin * k * k)).to(torch.bfloat16)
    dy = torch.randn(N, H, W, Cout).to(torch.bfloat16)
    add = torch.randn(N, H, W, Cin).to(torch.bfloat16)
    mask = torch.rand(N, H, W, Cin) > 0.3
    bits = (mask.reshape(-1, 8).to(torch.uint8) << torch.arange(8, dtype=torch.uint8)).sum(1).to(torch.uint8)
    C().set_gemm_paths(wide)
    try:
        dx = C().conv_dgrad(dy.to(DEV), w.to(DEV), H, W, s, p, 1, add.to(DEV), bits.to(DEV))
        dx0 = C().conv_dgrad(dy.to(DEV), w.to(DEV), H, W, s, p, 1, None, None)
    finally:
        C().set_gemm_paths(-1)
    ref = dx0.float().cpu() + add.float() * mask
    assert rel_err(dx.cpu(), ref) < 1e-2


_WGRAD_BUDGET_SCRIPT = r"""
import math, torch, torch.nn.functional as F
from pytorchdistributed_amd._native import C
for N, H, W, Cin, Cout, k, s, p in [(8, 28, 28, 64, 64, 1, 1, 0), (2, 28, 28, 128, 128, 3, 1, 1),
                                    (4, 14, 14, 256, 512, 3, 1, 1), (3, 7, 7, 512, 2048, 1, 1, 0)]:
    torch.manual_seed(3)
    x = torch.randn(N, H, W, Cin).to(torch.bfloat16).float()
    w = (torch.randn(Cout, k, k, Cin) / math.sqrt(Cin * k * k)).to(torch.bfloat16).float().requires_grad_()
    y = F.conv2d(x.permute(0, 3, 1, 2), w.permute(0, 3, 1, 2), None, s, p).permute(0, 2, 3, 1)
    dy = torch.randn_like(y).to(torch.bfloat16).float()
    y.backward(dy)
    bf = lambda t: t.to("cuda", torch.bfloat16).contiguous()
    dw = C().conv_wgrad(bf(dy), bf(x), k, k, s, p, 1, True, None).cpu()
    err = ((dw - w.grad).norm() / w.grad.norm()).item()
    assert err < 1e-3, (N, H, W, Cin, Cout, k, err)
print("budget ok")
"""


@pytest.mark.parametrize("env", [{"PDA_WGRAD_CUS": "48"}, {"PDA_WGRAD_CUS": "256", "PDA_WGRAD_CUS_WG3": "32"}])
def test_conv_wgrad_cu_budgets(env):
    """Split-K weight gradients planned for other CU budgets (PDA_WGRAD_CUS*, read once per process:
    run in a child) — the split counts and the slab sizing must agree at every budget."""
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", _WGRAD_BUDGET_SCRIPT], cwd=root, env={**os.environ, **env},
                       capture_output=True, text=True, timeout=100)
    assert r.returncode == 0 and "budget ok" in r.stdout, r.stdout[-2000:] + r.stderr[-2000:]


_PP_REBASE_SCRIPT = r"""
import torch
from pytorchdistributed_amd._native import C
torch.manual_seed(5)
dev = "cuda"
def rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12)).item()
# K = 40 K tiles (not a multiple of the 2-tile rebase period), every MN-major layout, split and unsplit
for M, N, K in [(512, 520, 2560), (264, 256, 2600)]:
    for lay in ("nn", "tn", "mn"):
        ak, bk = lay == "nn", lay == "mn"
        a = (torch.rand(M, K, device=dev) * 2 - 1).bfloat16() if ak else (torch.rand(K, M, device=dev) * 2 - 1).bfloat16()
        b = (torch.rand(N, K, device=dev) * 2 - 1).bfloat16() if bk else (torch.rand(K, N, device=dev) * 2 - 1).bfloat16()
        ref = (a.float() if ak else a.float().t()) @ (b.float().t() if bk else b.float())
        for split in (False, True):
            o = torch.empty(M, N, device=dev, dtype=torch.bfloat16)  # bf16 C: the pipelined tile's output
            C().gemm(a, ak, K if ak else M, b, bk, K if bk else N, o, N, M, N, K, None, False, split)
            assert rel(o, ref) < 5e-3, (M, N, K, lay, split, rel(o, ref))
# the fused weight + bias gradient (row sums) across rebases
dy = (torch.rand(4096, 1024, device=dev) * 2 - 1).bfloat16()  # the shape test_gemm_wgrad_db_fused pins to the tile
x = (torch.rand(4096, 1024, device=dev) * 2 - 1).bfloat16()
dw = torch.empty(1024, 1024, device=dev, dtype=torch.bfloat16)
db = torch.empty(1024, device=dev, dtype=torch.float32)
done = C().gemm_wgrad_db(dy, x, dw, db)
assert rel(dw, dy.float().t() @ x.float()) < 5e-3
assert done and rel(db, dy.float().sum(0)) < 1e-5
print("rebase ok")
"""


def test_gemm_pp_descriptor_rebase():
    """MN-major operands re-base their buffer descriptor every 2^s K tiles so K spans past 2 GB (the LM-head
    weight gradients) keep 32-bit offsets; PDA_PP_RB_SHIFT=1 (read once per process: a child) forces a
    rebase every 2 K tiles on small GEMMs: every MN-major layout, split-K on and off, and the fused
    weight + bias gradient, against fp32."""
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", _PP_REBASE_SCRIPT], cwd=root, env={**os.environ, "PDA_PP_RB_SHIFT": "1"},
                       capture_output=True, text=True, timeout=100)
    assert r.returncode == 0 and "rebase ok" in r.stdout, r.stdout[-2000:] + r.stderr[-2000:]


@pytest.mark.parametrize("dual_bwd", [True, False])
# (768, 384): C = 1536 has no register-table layout -> the guard (bn_dual_ok) takes the separate-BN path
@pytest.mark.parametrize("inplanes,planes,stride", [(64, 64, 1), (256, 128, 2), (512, 256, 2), (1024, 512, 2),
                                                    (768, 384, 2)])
def test_dual_bn_bottleneck_matches_unfused(inplanes, planes, stride, dual_bwd, monkeypatch):
    """Downsample bottleneck: relu(bn3(z3) + bn_ds(z_ds)) in one kernel (PDA_DUAL_BN) vs the separate
    shortcut BN apply + residual BN, both against the fp32 block on the CPU: output, input / parameter
    gradients and running statistics (bf16 gradients of both paths sit ~6 % from fp32 at 588 rows per
    channel).  The fused path keeps the shortcut in fp32 (no bf16 rounding of
    bn_ds(z_ds) or of its gradient), so it must be at least as close to fp32 as the unfused one."""
    import copy

    from pytorchdistributed_amd.models import resnet as R
    from pytorchdistributed_amd.ops import norm as Nm

    monkeypatch.setattr(Nm, "_DUAL_BWD", dual_bwd)  # one-pass dual backward (C <= 1024) or two BN backwards
    torch.manual_seed(21)
    blk = R.Bottleneck(inplanes, planes, stride=stride, downsample=True, device=DEV, dtype=torch.bfloat16)
    with torch.no_grad():  # non-trivial affine parameters so both BNs' gamma / beta matter
        for m in blk.modules():
            if hasattr(m, "running_var") and m.weight is not None:
                m.weight.uniform_(0.5, 1.5)
                m.bias.uniform_(-0.3, 0.3)
    x0 = torch.randn(3, 14, 14, inplanes, device=DEV).to(torch.bfloat16)

    def run(b, x):
        x = x.clone().requires_grad_()
        y = b(x)
        y.backward(dy.to(y.device, y.dtype))
        return (y.detach().float().cpu(), x.grad.float().cpu(), [p.grad.float().cpu() for p in b.parameters()],
                [t.float().cpu() for n, t in b.named_buffers() if "running" in n])

    ref_blk = copy.deepcopy(blk).float().cpu()
    with torch.no_grad():
        dy = torch.randn_like(ref_blk(x0.float().cpu()))
    ref_blk = copy.deepcopy(blk).float().cpu()
    ref = run(ref_blk, x0.float().cpu())
    errs = {}
    for dual in (True, False):
        monkeypatch.setattr(R, "_DUAL_BN", dual)
        y, dx, g, r = run(copy.deepcopy(blk), x0)
        torch.cuda.synchronize()
        errs[dual] = [rel_err(y, ref[0]), rel_err(dx, ref[1])] + [rel_err(a, b) for a, b in zip(g, ref[2])]
        for a, b in zip(r, ref[3]):
            assert rel_err(a, b) < 1e-2
    for e_dual, e_sep in zip(errs[True], errs[False]):
        assert e_dual < 0.15 and e_dual <= 1.25 * e_sep + 2e-3, (errs[True], errs[False])


@pytest.mark.parametrize("fused_bwd", [True, False])
def test_stem_bn_relu_maxpool_matches_unfused(fused_bwd, monkeypatch):
    """ResNet stem with BN + ReLU applied inside the maxpool's loads (PDA_STEM_BN_POOL) == conv -> BN+ReLU
    apply -> maxpool: same rounding of the pooled values, so output, parameter gradients and running
    statistics agree to the float-atomic summation order of the conv-epilogue statistics."""
    import copy

    from pytorchdistributed_amd.models import resnet as R
    from pytorchdistributed_amd.ops import pool as Pl

    monkeypatch.setattr(Pl, "_FUSED_BWD", fused_bwd)  # pool gradient gathered inside the BN backward or stored
    torch.manual_seed(22)
    stem = R.Stem(device=DEV, dtype=torch.bfloat16)
    with torch.no_grad():
        stem.bn1.weight.uniform_(0.5, 1.5)
        stem.bn1.bias.uniform_(-0.3, 0.3)
    x = torch.randn(4, 3, 58, 62, device=DEV).to(torch.bfloat16)  # odd pooled sizes, NCHW input
    runs = []
    for fused in (True, False):
        monkeypatch.setattr(R, "_STEM_BN_POOL", fused)
        s = copy.deepcopy(stem)
        y = s(x)
        if not runs:
            dy = torch.randn_like(y)
        y.backward(dy)
        torch.cuda.synchronize()
        runs.append((y.float(), [p.grad.float() for p in s.parameters()],
                     [t.float() for n, t in s.named_buffers() if "running" in n]))
    (y1, g1, r1), (y2, g2, r2) = runs
    assert y1.shape == y2.shape == (4, 15, 16, 64)
    assert rel_err(y1, y2) < 1e-2
    for a, b in zip(g1, g2):
        assert rel_err(a, b) < 1e-2
    for a, b in zip(r1, r2):
        assert rel_err(a, b) < 1e-4


_ROWNORM_FUSED_SCRIPT = r"""
import torch, torch.nn.functional as F
from pytorchdistributed_amd.ops import layer_norm, rms_norm
def rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()
for rms in (False, True):
    for D, rows in [(64, 37), (1024, 2500), (1600, 37), (2048, 300)]:
        torch.manual_seed(7)
        x = (torch.randn(rows, D) * 2 + 0.3).to(torch.bfloat16).float()
        g, b = torch.rand(D) + 0.5, torch.randn(D)
        xr, gr, br = x.clone().requires_grad_(), g.clone().requires_grad_(), b.clone().requires_grad_()
        y = xr * torch.rsqrt(xr.pow(2).mean(-1, keepdim=True) + 1e-6) * gr if rms else F.layer_norm(xr, (D,), gr, br, 1e-5)
        dy = torch.randn_like(y)
        y.backward(dy)
        xg = x.to("cuda", torch.bfloat16).requires_grad_()
        gg, bg = g.cuda().requires_grad_(), b.cuda().requires_grad_()
        yg = rms_norm(xg, gg, 1e-6) if rms else layer_norm(xg, gg, bg, 1e-5)
        yg.backward(dy.to("cuda", torch.bfloat16))
        errs = [rel(xg.grad.cpu(), xr.grad), rel(gg.grad.cpu(), gr.grad)] + ([] if rms else [rel(bg.grad.cpu(), br.grad)])
        assert max(errs) < 2e-2, (rms, D, rows, errs)
print("fused ok")
"""


def test_rownorm_fused_bwd_path():
    """LayerNorm / RMSNorm backward with the parameter-gradient partials accumulated by the dx kernel
    (PDA_ROWNORM_FUSED_BWD=1, read once per process: run in a child) against the fp32 reference."""
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", _ROWNORM_FUSED_SCRIPT], cwd=root,
                       env={**os.environ, "PDA_ROWNORM_FUSED_BWD": "1"}, capture_output=True, text=True, timeout=100)
    assert r.returncode == 0 and "fused ok" in r.stdout, r.stdout[-2000:] + r.stderr[-2000:]


_STEM_FWD_SCRIPT = r"""
import torch, torch.nn.functional as F
from pytorchdistributed_amd._native import C
for N, H in [(2, 35), (16, 51), (13, 115)]:  # 1, 2 and 3 output rows per workgroup
    torch.manual_seed(1)
    x = torch.randn(N, H, H, 16).to(torch.bfloat16)
    w = (torch.randn(64, 4, 4, 16) / 16).to(torch.bfloat16)
    ref = F.conv2d(x.float().permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2)).permute(0, 2, 3, 1)
    ys = [C().conv_fwd(x.cuda(), w.cuda(), 1, 0, 1, None, False).cpu() for _ in range(3)]
    assert all(torch.equal(ys[0], y) for y in ys[1:]), (N, H)
    err = ((ys[0].float() - ref).norm() / ref.norm()).item()
    assert err < 1e-2, (N, H, err)
    shift = torch.randn(64) * 0.1
    table = torch.zeros(7, 2, 64, device="cuda")
    y = C().conv_fwd_stats(x.cuda(), w.cuda(), 1, 0, 1, shift.cuda(), table)
    d = y.float().cpu().reshape(-1, 64) - shift
    s = torch.stack([d.sum(0), (d * d).sum(0)])
    assert ((table.sum(0).cpu() - s).norm() / s.norm()).item() < 1e-4, (N, H)
print("stem fwd ok")
"""


def test_stem_fwd_kernel_rows_per_workgroup():
    """The stem forward band kernel (PDA_CONV_STEM_FWD=1 forced in a child: the flag is read once per
    process): fp32-reference numerics, bit-exact repeats and the epilogue BN sums at 1-3 output rows
    per workgroup (the conv tests above cover 1 only)."""
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", _STEM_FWD_SCRIPT], cwd=root,
                       env={**os.environ, "PDA_CONV_STEM_FWD": "1"}, capture_output=True, text=True, timeout=100)
    assert r.returncode == 0 and "stem fwd ok" in r.stdout, r.stdout[-2000:] + r.stderr[-2000:]


@pytest.mark.parametrize("fused", ["0", "1"])
@pytest.mark.parametrize("M,K,N", [(64, 40, 24), (300, 136, 200), (2048, 512, 512)])
def test_linear_grads_land_in_flat_slots_once(monkeypatch, fused, M, K, N):
    """each flat-buffer slot is claimed once per backward.  With the fused wgrad+db path off
    and on small shapes (db from a column sum) the weight / bias gradients must alias the flat buffer and
    the parameter must NOT be marked shared (a second claim reads as a tied weight and pushes the
    parameter off the side stream for good)."""
    monkeypatch.setenv("PDA_WGRAD_DB_FUSED", fused)
    from pytorchdistributed_amd.ops.linear import linear
    from pytorchdistributed_amd.parallel.flat import FlatGroup

    torch.manual_seed(0)
    w = torch.nn.Parameter((torch.randn(N, K) * 0.1).to(DEV, torch.bfloat16))
    b = torch.nn.Parameter((torch.randn(N) * 0.1).to(DEV, torch.bfloat16))
    fg = FlatGroup([w, b])
    x = bf(torch.randn(M, K))
    dy = bf(torch.randn(M, N))
    for _ in range(2):
        w.grad = b.grad = None
        w._pda_claimed = b._pda_claimed = False
        linear(x, w, b).backward(dy)
        torch.cuda.synchronize()
        assert not getattr(w, "_pda_shared", False) and not getattr(b, "_pda_shared", False)
        assert w.grad.data_ptr() == fg.grad_view(0).data_ptr()
        assert b.grad.data_ptr() == fg.grad_view(1).data_ptr()
    assert rel_err(w.grad, dy.float().t() @ x.float()) < 1e-2
    assert rel_err(b.grad, dy.float().sum(0)) < 1e-2


@pytest.mark.parametrize("M,Cin,Cout", [(640 * 56 * 56 // 64, 64, 256), (3000, 128, 512), (1000, 256, 1024), (37, 64, 64),
                                        (4100, 128, 192)])
def test_fwd_stream_matches_tile(M, Cin, Cout):
    """Streaming short-K 1x1 forward (fwd_stream.hip) against the 256 x 256 tile and fp32: the same bf16
    output (same MFMA k order), and BN sums over the stored output (ragged M, N = 64 / 192 column groups)."""
    torch.manual_seed(41)
    x = torch.randn(1, 1, M, Cin).to(torch.bfloat16)
    w = (torch.randn(Cout, 1, 1, Cin) / math.sqrt(Cin)).to(torch.bfloat16)
    shift = torch.randn(Cout) * 0.1
    outs = {}
    try:
        for mode in (0, 2):
            C().set_fwd_stream(mode)
            table = torch.zeros(3, 2, Cout, device=DEV)
            y = C().conv_fwd_stats(x.to(DEV), w.to(DEV), 1, 0, 1, shift.to(DEV), table)
            outs[mode] = (y, table.sum(0))
    finally:
        C().set_fwd_stream(-1)
    ref = x.float().reshape(M, Cin) @ w.float().reshape(Cout, Cin).t()
    for mode, (y, tab) in outs.items():
        assert rel_err(y.float().cpu().reshape(M, Cout), ref) < 1e-2, mode
        d = y.float().cpu().reshape(M, Cout) - shift
        assert rel_err(tab.cpu(), torch.stack([d.sum(0), (d * d).sum(0)])) < 1e-4, mode
    assert rel_err(outs[0][0].float(), outs[2][0].float()) < 1e-3
