"""fp32 training path (ops/fp32.py, csrc/kernels/fp32x3.hip) against fp64/fp32 CPU references.

The reference trains ResNet-50 in fp32 (`03 模型并行/03_model_parallel.ipynb` raw lines 369-391); every
kernel of the fp32 path must match a CPU fp32 computation of the same op to <= 1e-4 relative error
(norm-wise), the split-bf16 convs included (TF32 would sit near 1e-3).
"""
import copy

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = "cuda"


def rel_err(a, b):
    a, b = a.double(), b.double()
    return ((a - b).norm() / (b.norm() + 1e-30)).item()


def _ref_conv(x, w, stride, pad, dil=1):
    y = F.conv2d(x.permute(0, 3, 1, 2).double(), w.permute(0, 3, 1, 2).double(), None, stride, pad, dil)
    return y.permute(0, 2, 3, 1)


@pytest.mark.parametrize("N,H,C,Co,R,stride", [(4, 14, 64, 128, 1, 1), (4, 14, 64, 64, 3, 1), (3, 15, 32, 64, 3, 2),
                                               (2, 16, 128, 256, 1, 2), (2, 35, 16, 64, 4, 1),
                                               (2, 7, 512, 2048, 1, 1)])
def test_conv_fp32_fwd_dgrad_wgrad(N, H, C, Co, R, stride):
    from pytorchdistributed_amd.ops import fp32

    torch.manual_seed(0)
    pad = (R - 1) // 2 if R != 4 else 0
    x = torch.randn(N, H, H, C)
    w = torch.randn(Co, R, R, C) * (1.0 / (C * R * R) ** 0.5)
    xg = x.to(DEV).requires_grad_()
    wg = w.to(DEV).requires_grad_()
    y = fp32.conv2d(xg, wg, None, stride, pad)
    xr = x.double().requires_grad_()
    wr = w.double().requires_grad_()
    yr = _ref_conv(xr, wr, stride, pad)
    assert y.dtype == torch.float32
    assert rel_err(y.cpu(), yr) < 1e-4
    dy = torch.randn(yr.shape)
    y.backward(dy.to(DEV))
    yr.backward(dy.double())
    assert rel_err(xg.grad.cpu(), xr.grad) < 1e-4
    assert rel_err(wg.grad.cpu(), wr.grad) < 1e-4


def test_split_bf16_layouts():
    from pytorchdistributed_amd._native import C

    torch.manual_seed(0)
    x = torch.randn(6, 8, device=DEV) * 3.7
    hi = x.to(torch.bfloat16)
    lo = (x - hi.float()).to(torch.bfloat16)
    cols = C().split_bf16(x, 3, 0b100, False)  # hi, hi, lo side by side
    assert torch.equal(cols, torch.cat([hi, hi, lo], dim=1))
    stack = C().split_bf16(x, 3, 0b010, True)  # hi, lo, hi stacked
    assert torch.equal(stack, torch.cat([hi, lo, hi], dim=0))
    # hi + lo carries 16 significant bits of x
    assert rel_err((hi.float() + lo.float()).cpu(), x.cpu()) < 1e-5


@pytest.mark.parametrize("residual,relu", [(False, True), (True, True), (False, False)])
@pytest.mark.parametrize("C_", [64, 2048, 48])
def test_batchnorm_fp32_train(residual, relu, C_):
    from pytorchdistributed_amd.ops import fp32

    torch.manual_seed(0)
    M = 3000 if C_ < 1024 else 196
    x = torch.randn(M, C_) * 2.0 + 0.5
    r = torch.randn(M, C_) if residual else None
    gamma, beta = torch.rand(C_) + 0.5, torch.randn(C_)
    rm, rv = torch.zeros(C_), torch.ones(C_)
    rm_g, rv_g = rm.to(DEV), rv.to(DEV)
    nbt = torch.zeros((), dtype=torch.long, device=DEV)
    xg = x.to(DEV).requires_grad_()
    gg, bg = gamma.to(DEV).requires_grad_(), beta.to(DEV).requires_grad_()
    rg = r.to(DEV).requires_grad_() if residual else None
    y = fp32.batch_norm(xg, gg, bg, rm_g, rv_g, True, 0.1, 1e-5, rg, relu, nbt)
    xr = x.double().requires_grad_()
    gr, br = gamma.double().requires_grad_(), beta.double().requires_grad_()
    rr = r.double().requires_grad_() if residual else None
    rmr, rvr = rm.double(), rv.double()
    yr = F.batch_norm(xr, rmr, rvr, gr, br, True, 0.1, 1e-5)
    if residual:
        yr = yr + rr
    if relu:
        yr = torch.relu(yr)
    assert rel_err(y.cpu(), yr) < 1e-5
    assert rel_err(rm_g.cpu(), rmr) < 1e-5 and rel_err(rv_g.cpu(), rvr) < 1e-5
    assert int(nbt.item()) == 1
    dy = torch.randn(M, C_)
    y.backward(dy.to(DEV))
    yr.backward(dy.double())
    assert rel_err(xg.grad.cpu(), xr.grad) < 1e-4
    assert rel_err(gg.grad.cpu(), gr.grad) < 1e-4 and rel_err(bg.grad.cpu(), br.grad) < 1e-4
    if residual:
        assert rel_err(rg.grad.cpu(), rr.grad) < 1e-6


def test_pools_fp32():
    from pytorchdistributed_amd import ops

    torch.manual_seed(0)
    x = torch.randn(3, 17, 16, 64)
    xg = x.to(DEV).requires_grad_()
    y = ops.max_pool2d(xg, 3, 2, 1)
    xr = x.clone().requires_grad_()
    yr = F.max_pool2d(xr.permute(0, 3, 1, 2), 3, 2, 1).permute(0, 2, 3, 1)
    assert torch.equal(y.cpu(), yr.detach())
    dy = torch.randn(yr.shape)
    y.backward(dy.to(DEV))
    yr.backward(dy)
    assert rel_err(xg.grad.cpu(), xr.grad) < 1e-6
    xg2 = x.to(DEV).requires_grad_()
    p = ops.global_avg_pool2d(xg2)
    assert p.dtype == torch.float32
    pr = x.double().mean(dim=(1, 2))
    assert rel_err(p.cpu(), pr) < 1e-6
    p.sum().backward()
    assert torch.allclose(xg2.grad.cpu(), torch.full_like(x, 1.0 / (17 * 16)))


def test_resnet50_fp32_matches_cpu_fp32():
    """The fp32 ResNet-50 on the native path vs the same model on the CPU (torch fp32 ops): eval-mode
    forward end to end, and a train-mode forward + backward of a downsampling bottleneck."""
    from pytorchdistributed_amd.models.resnet import resnet50

    torch.manual_seed(0)
    cpu = resnet50()
    gpu = copy.deepcopy(cpu).to(DEV)
    cpu.eval()
    gpu.eval()
    x = torch.randn(2, 64, 64, 3)
    with torch.no_grad():
        assert rel_err(gpu(x.to(DEV)).cpu(), cpu(x)) < 5e-4  # 50 layers of ~1e-5 each
    for blk_ref in (cpu.layer2[0], cpu.layer4[0]):
        blk_ref = blk_ref.train()
        blk_gpu = copy.deepcopy(blk_ref).to(DEV)
        cin = blk_ref.conv1.in_channels
        hw = 8 if cin > 512 else 16
        xin = torch.randn(4, hw, hw, cin).requires_grad_()
        out_r = blk_ref(xin)
        dy = torch.randn_like(out_r)
        out_r.backward(dy)
        xg = xin.detach().to(DEV).requires_grad_()
        out_g = blk_gpu(xg)
        out_g.backward(dy.to(DEV))
        assert rel_err(out_g.cpu(), out_r.detach()) < 1e-4
        assert rel_err(xg.grad.cpu(), xin.grad) < 1e-3
        for (n, pr), (_, pg) in zip(blk_ref.named_parameters(), blk_gpu.named_parameters()):
            assert rel_err(pg.grad.cpu(), pr.grad) < 1e-3, n


def _round_tf32(t):
    """fp32 -> TF32 (10-bit mantissa, round to nearest) as cuDNN feeds A100 tensor cores; the rounding
    is applied to the values only (straight-through for autograd, whose conv backward sees the rounded
    operands as well)."""
    d = t.detach().contiguous()
    r = ((d.view(torch.int32) + 0x1000) & ~0x1FFF).view(torch.float32)
    return t + (r - d)


def test_resnet50_fp32_whole_model_gradients(monkeypatch):
    """Whole-model train-mode gradients of the fp32 ResNet-50 against an fp64 CPU oracle, compared with
    what the reference's own precision gets: its A100 ran the convs in TF32 (emulated here on the CPU by
    rounding every conv operand to TF32).  A random-init ResNet-50 is ill-conditioned (batch-statistics
    BN backward), so errors are judged against that yardstick, not absolute: the 3-product split must be
    at least 2x closer to fp64 than TF32, whole-vector and per parameter (measured: 8e-2 / 1.0e-1 vs
    6.4e-1 / 8.7e-1; CPU fp32 1.4e-2 / 1.7e-2 on this ill-conditioned net)."""
    from pytorchdistributed_amd.data.datasets import random_image_batch
    from pytorchdistributed_amd.models.resnet import resnet50
    from pytorchdistributed_amd.ops import conv as conv_mod
    from pytorchdistributed_amd.ops import cross_entropy, fp32

    torch.manual_seed(0)
    cpu = resnet50()
    x, y = random_image_batch(6, (96, 96), 1000)

    def grads(m, dev, dt):
        m.zero_grad()
        loss = cross_entropy(m(x.to(dev, dt).permute(0, 2, 3, 1)), y.to(dev, dt))
        loss.backward()
        return loss.item(), {n: p.grad.detach().cpu().double() for n, p in m.named_parameters()}

    l64, g64 = grads(copy.deepcopy(cpu).double(), "cpu", torch.float64)
    l32, g32 = grads(copy.deepcopy(cpu), "cpu", torch.float32)
    ref_conv = conv_mod._ref_conv
    with monkeypatch.context() as mp:
        mp.setattr(conv_mod, "_ref_conv", lambda x_, w_, *a, **k: ref_conv(_round_tf32(x_), _round_tf32(w_), *a, **k))
        ltf, gtf = grads(copy.deepcopy(cpu), "cpu", torch.float32)
    res = {}
    for nseg in (3, 4):
        fp32.set_split(nseg)
        try:
            res[nseg] = grads(copy.deepcopy(cpu).to(DEV), DEV, torch.float32)
        finally:
            fp32.set_split(3)

    def worst(g):
        return max(rel_err(g[n], g64[n]) for n in g64)

    def whole(g):
        return rel_err(torch.cat([g[n].flatten() for n in g64]), torch.cat([g64[n].flatten() for n in g64]))

    print(f"cpu fp32: whole {whole(g32):.2e} worst {worst(g32):.2e}; tf32 convs: whole {whole(gtf):.2e} "
          f"worst {worst(gtf):.2e}")
    for nseg, (loss, g) in res.items():
        print(f"split {nseg}: loss {abs(loss - l64) / abs(l64):.2e} whole {whole(g):.2e} worst {worst(g):.2e}")
    for nseg, (loss, g) in res.items():
        assert abs(loss - l64) < 1e-4 * abs(l64), (nseg, loss, l64)
    _, g3 = res[3]
    _, g4 = res[4]
    # both splits carry x as hi + lo (16 significant bits, ~2^-17 relative): a ~1e-5 floor that the
    # 4th product (lo.lo) does not remove; TF32 keeps 11 bits (~2^-12)
    assert whole(g3) < 0.5 * whole(gtf) and worst(g3) < 0.5 * worst(gtf), (whole(g3), whole(gtf), worst(g3),
                                                                         worst(gtf))
    assert whole(g4) < 1.2 * whole(g3) and worst(g4) < 1.2 * worst(g3), (whole(g4), whole(g3))


def test_resnet50_fp32_adam_step():
    """Two fp32 NB03-style steps (soft one-hot targets, fused Adam on fp32 params) run natively: the
    first loss matches the CPU fp32 model, and the fused Adam step trains the model."""
    from pytorchdistributed_amd.data.datasets import random_image_batch
    from pytorchdistributed_amd.models.resnet import resnet50
    from pytorchdistributed_amd.ops import cross_entropy
    from pytorchdistributed_amd.optim import Adam

    torch.manual_seed(0)
    cpu = resnet50()
    gpu = copy.deepcopy(cpu).to(DEV)
    x, y = random_image_batch(4, (64, 64), 1000)
    with torch.no_grad():
        c0 = cross_entropy(cpu(x.permute(0, 2, 3, 1)), y).item()
    opt = Adam(gpu.parameters(), lr=1e-3)
    run = []
    for _ in range(2):
        opt.zero_grad()
        loss = cross_entropy(gpu(x.to(DEV).permute(0, 2, 3, 1)), y.to(DEV))
        loss.backward()
        opt.step()
        run.append(loss.item())
    g0, g1 = run
    assert abs(c0 - g0) < 1e-4 * abs(c0), (c0, run)
    assert g1 == g1 and g1 < 0.8 * g0, run
