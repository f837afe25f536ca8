"""Model-level GPU checks: the native ResNet-50 path against the PyTorch reference path on the same
weights, the DDP+fused-optimizer step, and the driver smoke()."""
import copy

import pytest
import torch

pytestmark = pytest.mark.gpu


def rel_err(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


def test_resnet50_native_matches_reference():
    """Stage by stage (each stage fed the reference activation) the native path must track the fp32
    PyTorch reference to bf16 accuracy; end to end both run with bf16 activations.  (A random-init net
    with BN over tiny spatial maps amplifies rounding differences, so the end-to-end check compares
    against a reference that rounds at the same points.)"""
    from pytorchdistributed_amd.models.resnet import resnet50
    from pytorchdistributed_amd.ops import cross_entropy

    torch.manual_seed(0)
    cpu = resnet50(dtype=torch.bfloat16).float()
    gpu = copy.deepcopy(cpu).to("cuda", torch.bfloat16)
    x = torch.randn(4, 64, 64, 3).to(torch.bfloat16).float()
    a = x
    for sc, sg in zip([cpu.stem, cpu.layer1, cpu.layer2, cpu.layer3, cpu.layer4],
                      [gpu.stem, gpu.layer1, gpu.layer2, gpu.layer3, gpu.layer4]):
        with torch.no_grad():
            oc = sc(a)
            og = sg(a.to("cuda", torch.bfloat16))
        assert rel_err(og.cpu(), oc) < 3e-2
        a = oc.to(torch.bfloat16).float()
    # end to end: eval mode (no batch-statistics amplification), then a train-mode step at 128 px
    torch.manual_seed(0)
    ref = resnet50(dtype=torch.bfloat16)
    gpu = copy.deepcopy(ref).to("cuda")
    ref.eval()
    gpu.eval()
    with torch.no_grad():
        assert rel_err(gpu(x.to("cuda", torch.bfloat16)).cpu(), ref(x.to(torch.bfloat16))) < 5e-2
    # backward, block by block (a composed check without the chaotic amplification of 50 random layers):
    # a downsampling bottleneck and a strided one.  Oracle: fp32 reference; the bound is set by the same
    # block run in bf16 on the CPU reference ops (batch-statistics BN backward over tiny maps loses ~6 %
    # to bf16 rounding alone), so the native path must be no worse than 1.5x plain bf16 rounding.
    for bi, blk_ref in [(0, ref.layer1[0]), (1, ref.layer2[0]), (2, ref.layer4[0])]:
        blk_ref = blk_ref.float().train()
        blk_gpu = copy.deepcopy(blk_ref).to("cuda", torch.bfloat16)
        blk_b16 = copy.deepcopy(blk_ref).to(torch.bfloat16)
        cin = blk_ref.conv1.in_channels
        hw = {0: 16, 1: 16, 2: 8}[bi]
        xin = torch.randn(4, hw, hw, cin).to(torch.bfloat16).float().requires_grad_()
        out_r = blk_ref(xin)
        dy = torch.randn_like(out_r).to(torch.bfloat16).float()
        out_r.backward(dy)
        xb = xin.detach().to(torch.bfloat16).requires_grad_()
        blk_b16(xb).backward(dy.to(torch.bfloat16))
        xg = xin.detach().to("cuda", torch.bfloat16).requires_grad_()
        out_g = blk_gpu(xg)
        out_g.backward(dy.to("cuda", torch.bfloat16))
        assert rel_err(out_g.cpu(), out_r.detach()) < 3e-2
        assert rel_err(xg.grad.cpu(), xin.grad) < max(2e-2, 1.5 * rel_err(xb.grad, xin.grad)), bi
        for (n, pr), (_, pg), (_, pb) in zip(blk_ref.named_parameters(), blk_gpu.named_parameters(),
                                             blk_b16.named_parameters()):
            assert rel_err(pg.grad.cpu(), pr.grad) < max(2e-2, 1.5 * rel_err(pb.grad, pr.grad)), (bi, n)


def test_ddp_fused_sgd_step_single_rank():
    from pytorchdistributed_amd.models.resnet import resnet50
    from pytorchdistributed_amd.ops import cross_entropy
    from pytorchdistributed_amd.optim import SGD
    from pytorchdistributed_amd.parallel.ddp import DistributedDataParallel

    torch.manual_seed(0)
    base = resnet50(device="cuda", dtype=torch.bfloat16)
    ref = copy.deepcopy(base)
    model = DistributedDataParallel(base, device_ids=[0])
    opt = SGD(model.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4)
    ropt = SGD(ref.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4)  # per-tensor path
    x = torch.randn(4, 32, 32, 8, device="cuda", dtype=torch.bfloat16)
    y = torch.randint(0, 1000, (4,), device="cuda")
    for _ in range(2):
        for m, o in [(model, opt), (ref, ropt)]:
            o.zero_grad()
            cross_entropy(m(x), y).backward()
            o.step()
    assert len(opt._flat) == 1  # one fused launch for the whole model
    for (n, p), (_, q) in zip(base.named_parameters(), ref.named_parameters()):
        assert rel_err(p.detach().cpu(), q.detach().cpu()) < 2e-2, n


def test_graft_smoke():
    import __graft_entry__ as g

    g.smoke()


@pytest.mark.parametrize("hw", [32, 33])
def test_stem_space_to_depth_matches_direct_conv(hw):
    """The 4x4/1 space-to-depth stem equals the 7x7/2/pad-3 conv, forward and weight gradient."""
    import torch.nn.functional as F

    from pytorchdistributed_amd import ops
    from pytorchdistributed_amd.models.resnet import space_to_depth_stem

    torch.manual_seed(3)
    x = torch.randn(2, hw, hw, 3).to(torch.bfloat16).float()
    w = (torch.randn(64, 7, 7, 3) * 0.1).to(torch.bfloat16).float().requires_grad_()
    y = F.conv2d(x.permute(0, 3, 1, 2), w.permute(0, 3, 1, 2), None, 2, 3).permute(0, 2, 3, 1)
    dy = torch.randn_like(y).to(torch.bfloat16).float()
    y.backward(dy)
    wg = w.detach().to("cuda", torch.bfloat16).requires_grad_()
    x2, w2 = space_to_depth_stem(x.to("cuda", torch.bfloat16), wg)
    yg = ops.conv2d(x2, w2, None, 1, 0)
    assert yg.shape == y.shape
    assert rel_err(yg.cpu(), y.detach()) < 1e-2
    yg.backward(dy.to("cuda", torch.bfloat16))
    assert rel_err(wg.grad.cpu(), w.grad) < 1e-2


@pytest.mark.parametrize("hw,cx", [(32, 3), (33, 8)])
def test_stem_s2d_kernel_matches_torch_layout(hw, cx):
    from pytorchdistributed_amd._native import C
    from pytorchdistributed_amd.models.resnet import space_to_depth_stem

    x = torch.randn(2, hw, hw, cx, device="cuda").to(torch.bfloat16)
    w = torch.randn(64, 7, 7, 3, device="cuda", dtype=torch.bfloat16)
    ref, _ = space_to_depth_stem(x[..., :3], w)
    got = C().stem_s2d(x, 3, 3)
    assert got.shape == ref.shape
    assert torch.equal(got, ref)


def test_ddp_resnet50_two_ranks_share_gpu(tmp_path):
    """The multi-rank DDP path (hooks, native bucket reducer, bucket all-reduce, flat grads written by
    the wgrad kernels, fused SGD) at world 2 on the one GPU of the test box, over gloo."""
    import _workers
    from pytorchdistributed_amd.launch import spawn

    spawn(_workers.ddp_resnet_gpu_worker, args=(2, str(tmp_path)), nprocs=2, timeout=300)
    for r in range(2):
        assert (tmp_path / f"ok{r}").read_text().startswith("ok")


@pytest.mark.parametrize("mode", ["native", "c10d", "native_fp32"])
def test_ddp_rccl_one_rank_group_matches_local(tmp_path, mode):
    """The RCCL branch of DDP (what the driver's 2/4/8-GPU runs execute) on a one-rank RCCL group:
    the native communicator (default), torch's ProcessGroupNCCL (PDA_COMM=c10d), and fp32 reduction of
    the bf16 buckets (PDA_GRAD_REDUCE_DTYPE=fp32), each matching a plain replica's gradients."""
    import _workers
    from pytorchdistributed_amd.launch import spawn

    spawn(_workers.ddp_rccl_world1_worker, args=(1, str(tmp_path), mode), nprocs=1, timeout=300)
    assert (tmp_path / "ok0").read_text().startswith("ok")


def test_ddp_rccl_one_rank_group_lr005_stem_gemm(tmp_path):
    """The original lr-0.05 replica check: with the stem on the implicit GEMM (its BN sums in a
    fixed order, PDA_CONV_STEM_FWD=0) the DDP replica and a local one stay equal over three steps."""
    import _workers
    from pytorchdistributed_amd.launch import spawn

    spawn(_workers.ddp_rccl_world1_worker, args=(1, str(tmp_path), "native", 0.05), nprocs=1, timeout=300)
    assert (tmp_path / "ok0").read_text().startswith("ok")


def test_parameter_server_rccl_one_rank_group(tmp_path):
    """parallel/param_server.py over a one-rank RCCL group: gradients reduced to the server and
    parameters broadcast back through RCCL on device tensors; three steps equal a local replica's."""
    import _workers
    from pytorchdistributed_amd.launch import spawn

    spawn(_workers.ps_rccl_world1_worker, args=(1, str(tmp_path)), nprocs=1, timeout=300)
    assert (tmp_path / "ok0").read_text().startswith("ok")


def test_native_rccl_communicator_one_rank(tmp_path):
    """csrc/comm/communicator.cpp through comm.py: all-reduce (sum / avg, fp32 / bf16), all-gather,
    reduce-scatter, broadcast, fused send/recv, work handles, stream ordering."""
    import _workers
    from pytorchdistributed_amd.launch import spawn

    spawn(_workers.rccl_comm_world1_worker, args=(1, str(tmp_path)), nprocs=1, timeout=200)
    assert (tmp_path / "ok0").read_text().startswith("ok")


def test_fsdp_forced_comm_one_rank_rccl(tmp_path):
    """FSDP at world 1 over a one-rank RCCL group with PDA_FSDP_FORCE_COMM=1: the unit all-gathers and
    gradient reduce-scatters run as real ncclAllGather / ncclReduceScatter on the native communicator
    (no shard aliasing), the result matches an unsharded replica, and comm_stats reports exposed time."""
    import _workers
    from pytorchdistributed_amd.launch import spawn

    spawn(_workers.fsdp_llama_gpu_worker, args=(1, str(tmp_path), "rccl", True), nprocs=1, timeout=300)
    assert (tmp_path / "ok0").read_text().startswith("ok")


@pytest.mark.parametrize("schedule", ["1f1b", "interleaved"])
def test_pipeline_ddp_tickets_retire_one_rank_rccl(tmp_path, schedule):
    """Pipeline(S=1) + DDP stage over a one-rank RCCL group, run past a 5 s collective timeout in report
    mode: no expired ticket, bounded ticket list, nothing armed after an idle period;
    interleaved: chunk hand-offs through RCCL send/recv to self."""
    import _workers
    from pytorchdistributed_amd.launch import spawn

    spawn(_workers.pipeline_ddp_watchdog_worker, args=(1, str(tmp_path), schedule), nprocs=1, timeout=240)
    assert (tmp_path / "ok0").read_text().startswith("ok")


@pytest.mark.parametrize("world", [1, 2])
def test_fsdp_llama_tiny_matches_unsharded(tmp_path, world):
    """FSDP on the native transformer path: world 1 (the shard aliases the gathered buffer) and world 2
    (two ranks sharing the GPU over gloo: all-gather / reduce-scatter of bf16 shards)."""
    import _workers
    from pytorchdistributed_amd.launch import spawn

    spawn(_workers.fsdp_llama_gpu_worker, args=(world, str(tmp_path)), nprocs=world, timeout=300)
    for r in range(world):
        assert (tmp_path / f"ok{r}").read_text().startswith("ok")


def test_side_stream_wgrad_matches_single_stream():
    """Weight gradients on the side stream (ops/streams.py) must match the single-stream path: two
    DDP(world 1) + fused-SGD steps of ResNet-50 from the same init, grads written straight into the
    flat bucket buffer by wgrad kernels running concurrently with the BN backward; every parameter's
    step-2 gradient is compared (a missed dependency shows as an O(1) error on some layer; BN batch
    statistics are summed with float atomics, so the two runs agree to rounding, not bitwise).  The
    learning rate keeps step 2 well conditioned: at lr 0.05 the random-init net diverges in step 1
    (loss ~14) and a last-bit difference of one atomic sum moved step-2 BN gradients by O(1) even
    between two runs of one configuration (tools/debug_dualbwd.py)."""
    from pytorchdistributed_amd.data.device import DeviceSyntheticImages
    from pytorchdistributed_amd.models.resnet import resnet50
    from pytorchdistributed_amd.ops import cross_entropy, streams
    from pytorchdistributed_amd.optim import SGD
    from pytorchdistributed_amd.parallel.ddp import DistributedDataParallel

    def run(side):
        streams.set_enabled(side)
        try:
            torch.manual_seed(0)
            model = DistributedDataParallel(resnet50(device="cuda", dtype=torch.bfloat16), device_ids=[0])
            opt = SGD(model.parameters(), lr=1e-3, momentum=0.9, weight_decay=5e-5)
            data = DeviceSyntheticImages(16, 96, 1000, device=torch.device("cuda", 0), dtype=torch.bfloat16, seed=3)
            for _ in range(2):
                x, y = data.next()
                opt.zero_grad(set_to_none=True)
                loss = cross_entropy(model(x), y)
                loss.backward()
                grads = {n: p.grad.detach().float().clone() for n, p in model.module.named_parameters()}
                opt.step()
            torch.cuda.synchronize()
            return loss.item(), grads
        finally:
            streams.set_enabled(None)

    l0, g0 = run(False)
    l1, g1 = run(True)
    assert abs(l0 - l1) <= 1e-2 * abs(l0), (l0, l1)
    worst = max((rel_err(g1[n], g0[n]), n) for n in g0)
    assert worst[0] < 3e-2, worst


def test_tied_embedding_side_stream_matches_single_stream():
    """A small-vocab GPT-2 (tied wte under 256^3 elements, so the head's weight gradient is eligible
    for the side stream) under DDP: the tied parameter's gradient — the LM head's dW plus the
    embedding's scatter-add, summed by autograd — must match the single-stream run (the
    second use used to be summed on the compute stream while the first was still being written on
    the side stream)."""
    from pytorchdistributed_amd.models.gpt2 import GPT2, GPT2Config
    from pytorchdistributed_amd.ops import streams
    from pytorchdistributed_amd.parallel.ddp import DistributedDataParallel

    cfg = GPT2Config(vocab_size=512, n_positions=64, n_embd=128, n_layer=2, n_head=4)

    def run(side):
        streams.set_enabled(side)
        try:
            torch.manual_seed(0)
            model = DistributedDataParallel(GPT2(cfg, device="cuda", dtype=torch.bfloat16), device_ids=[0])
            g = torch.Generator(device="cuda").manual_seed(5)
            idx = torch.randint(0, cfg.vocab_size, (4, 64), device="cuda", generator=g)
            out = []
            for _ in range(2):
                for p in model.parameters():
                    p.grad = None
                loss = model(idx, targets=idx)
                loss.backward()
                out.append(model.module.wte.grad.detach().float().clone())
            torch.cuda.synchronize()
            return out
        finally:
            streams.set_enabled(None)

    ref = run(False)
    got = run(True)
    for a, b in zip(got, ref):
        assert rel_err(a, b) < 1e-2, rel_err(a, b)



@pytest.mark.parametrize("case", [
    # N, H, W, Cin(dx channels), Cout(dy channels), R, stride, pad, mask source, addend
    (4, 14, 14, 64, 256, 1, 1, 0, "ss", False),      # 1x1 dgrad, MN-major weight read in place (128 tile)
    (32, 28, 28, 256, 256, 1, 1, 0, "ss", False),    # 1x1 dgrad on a transposed weight (256 x 256 tile)
    (8, 28, 28, 128, 128, 3, 1, 1, "ss", False),     # 3x3 stride-1 dgrad (halo kernel)
    (32, 28, 28, 64, 64, 3, 1, 1, "ss", False),      # 3x3 stride-1, 64 channels (persistent res64 kernel)
    (48, 28, 28, 64, 64, 3, 1, 1, "ss", False),      # ... with 2 tiles per workgroup (next band in flight)
    (8, 28, 28, 128, 128, 3, 2, 1, "ss", False),     # 3x3 stride-2: phase launches + fill phases
    (32, 14, 14, 256, 1024, 1, 1, 0, "bits", True),  # next block's conv1: addend (shortcut) + bit mask
    (4, 14, 14, 64, 256, 1, 1, 0, "bits", True),
    (32, 14, 14, 256, 1024, 1, 1, 0, "dual", True),  # after a downsample block: two BNs, one masked dy
    (4, 14, 14, 64, 256, 1, 1, 0, "dual", True),
    # short K (64 / 128): the streaming kernel (dgrad_stream.hip), with M not a multiple of its 16-row tile
    (8, 28, 28, 256, 64, 1, 1, 0, "ss", False),
    (6, 15, 15, 256, 64, 1, 1, 0, "bits", True),
    (8, 28, 28, 256, 64, 1, 1, 0, "dual", True),
    (4, 14, 14, 512, 128, 1, 1, 0, "bits", True),
    (5, 13, 13, 512, 128, 1, 1, 0, "dual", True),
    (4, 14, 14, 256, 128, 1, 1, 0, "ss", False),
    (4, 14, 14, 128, 64, 1, 1, 0, "bits", False),   # N = 128: two waves per workgroup
])
def test_conv_dgrad_bn_bwd_stats(case):
    """The dgrad epilogue's BN-backward sums (gemm_epi.h bst_*) equal fp32 sums over the dx the same
    launch stored: sum(g) and sum(g (z - mean)), g = dx * relu_mask; dx itself is unchanged."""
    from pytorchdistributed_amd._native import C

    N, H, W, Cin, Cout, R, st, pad, src, with_add = case
    P, Q = (H + 2 * pad - R) // st + 1, (W + 2 * pad - R) // st + 1
    torch.manual_seed(0)
    dev = "cuda"
    dy = torch.randn(N, P, Q, Cout).to(dev, torch.bfloat16)
    w = (torch.randn(Cout, R, R, Cin) * 0.05).to(dev, torch.bfloat16)
    z = torch.randn(N, H, W, Cin).to(dev, torch.bfloat16)
    mean = (torch.randn(Cin) * 0.1).to(dev)
    addend = torch.randn(N, H, W, Cin).to(dev, torch.bfloat16) if with_add else None
    table = torch.zeros(64, 2, Cin, device=dev)
    kw = dict(bst_z=z, bst_mean=mean, bst_table=table)
    if src == "ss":
        scale, shift = torch.rand(Cin) + 0.5, torch.randn(Cin) * 0.2
        kw["bst_ss"] = torch.cat([scale, shift]).to(dev)
        keep = (z.float() * scale.to(dev) + shift.to(dev)) > 0
    else:
        if src == "dual":
            z2 = torch.randn(N, H, W, Cin).to(dev, torch.bfloat16)
            mean2 = (torch.randn(Cin) * 0.1).to(dev)
            table2 = torch.zeros(64, 2, Cin, device=dev)
            kw.update(bst_z2=z2, bst_mean2=mean2, bst_table2=table2)
        bits = torch.randint(0, 256, (N * H * W * Cin // 8,), dtype=torch.uint8, device=dev)
        kw["bst_bits"] = bits
        shifts = torch.arange(8, device=dev, dtype=torch.uint8)
        keep = ((bits.reshape(-1, 1) >> shifts) & 1).bool().reshape(z.shape)
    dx_ref = C().conv_dgrad(dy, w, H, W, st, pad, 1, addend, None)

    def run(mode):
        t1 = torch.zeros_like(table)
        k = dict(kw, bst_table=t1)
        t2 = None
        if src == "dual":
            t2 = torch.zeros_like(table2)
            k["bst_table2"] = t2
        C().set_dgrad_stream(mode)
        try:
            return C().conv_dgrad(dy, w, H, W, st, pad, 1, addend, None, **k), t1, t2
        finally:
            C().set_dgrad_stream(-1)

    # default routing; and for short K (64 / 128) the streaming kernel on every launch vs the 256 x 256 tile
    modes = [-1] + ([3, 0] if R == 1 and Cout in (64, 128) else [])
    for mode in modes:
        dx, tab1, tab2 = run(mode)
        assert torch.equal(dx, dx_ref), mode
        g = torch.where(keep, dx.float(), torch.zeros((), device=dev)).reshape(-1, Cin)
        s1 = g.sum(0)
        s2 = (g * (z.float().reshape(-1, Cin) - mean)).sum(0)
        tab = tab1.sum(0)
        scale1 = g.abs().sum(0) + 1e-3
        scale2 = (g * (z.float().reshape(-1, Cin) - mean)).abs().sum(0) + 1e-3
        assert ((tab[0] - s1).abs() / scale1).max().item() < 1e-4, mode
        assert ((tab[1] - s2).abs() / scale2).max().item() < 1e-4, mode
        if src == "dual":
            t2 = tab2.sum(0)
            s3 = (g * (z2.float().reshape(-1, Cin) - mean2)).sum(0)
            scale3 = (g * (z2.float().reshape(-1, Cin) - mean2)).abs().sum(0) + 1e-3
            assert ((t2[0] - s1).abs() / scale1).max().item() < 1e-4, mode
            assert ((t2[1] - s3).abs() / scale3).max().item() < 1e-4, mode
    if R == 1 and Cout in (64, 128):  # plain short-K dgrads on the streaming kernel (mode 2), with / without addend
        C().set_dgrad_stream(2)
        try:
            dx_plain = C().conv_dgrad(dy, w, H, W, st, pad, 1, addend, None)
            dx_noadd = C().conv_dgrad(dy, w, H, W, st, pad, 1, None, None)
        finally:
            C().set_dgrad_stream(-1)
        assert torch.equal(dx_plain, dx_ref)
        assert torch.equal(dx_noadd, C().conv_dgrad(dy, w, H, W, st, pad, 1, None, None))


def test_bottleneck_bwd_stats_from_dgrad_epilogue(monkeypatch):
    """layer1 (a downsample bottleneck + two identity ones): bn1 / bn2 of every block, the identity block's
    output BN and the downsample block's dual output BN pair (both through the next block's conv1 gradient
    join) take their backward sums from the dgrad epilogues — every BN backward but the last block's bn3
    (whose output has no conv consumer) finalizes from a table.  The gradients match the reduce-pass
    path and the fp32 CPU reference (to 1.5x plain bf16 rounding)."""
    from pytorchdistributed_amd._native import C as _C
    from pytorchdistributed_amd.models.resnet import resnet50
    from pytorchdistributed_amd.ops import norm as _norm

    torch.manual_seed(0)
    ref = resnet50(dtype=torch.bfloat16)
    pair_ref = torch.nn.Sequential(ref.layer1[0], ref.layer1[1], ref.layer1[2]).float().train()
    xin = torch.randn(8, 16, 16, 64).to(torch.bfloat16).float().requires_grad_()
    out_r = pair_ref(xin)
    dy = torch.randn_like(out_r).to(torch.bfloat16).float()
    out_r.backward(dy)
    pair_b16 = copy.deepcopy(pair_ref).to(torch.bfloat16)
    xb = xin.detach().to(torch.bfloat16).requires_grad_()
    pair_b16(xb).backward(dy.to(torch.bfloat16))

    calls = {"table": 0, "reduce": 0, "dual_table": 0, "dual": 0}
    mod = _C()
    real_t, real_r, real_d = mod.bn_bwd_table, mod.bn_bwd, mod.bn_bwd_dual

    def t_(*a, **k):
        calls["table"] += 1
        return real_t(*a, **k)

    def r_(*a, **k):
        calls["reduce"] += 1
        return real_r(*a, **k)

    def d_(*a, **k):
        calls["dual_table" if len(a) == 16 else "dual"] += 1
        return real_d(*a, **k)

    monkeypatch.setattr(mod, "bn_bwd_table", t_)
    monkeypatch.setattr(mod, "bn_bwd", r_)
    monkeypatch.setattr(mod, "bn_bwd_dual", d_)
    grads = {}
    for fused in (True, False):
        monkeypatch.setattr(_norm, "_BWD_EPILOGUE", fused)
        calls.update(table=0, reduce=0, dual_table=0, dual=0)
        pair_g = copy.deepcopy(pair_ref).to("cuda", torch.bfloat16)
        xg = xin.detach().to("cuda", torch.bfloat16).requires_grad_()
        pair_g(xg).backward(dy.to("cuda", torch.bfloat16))
        torch.cuda.synchronize()
        if fused:
            assert calls == {"table": 7, "reduce": 1, "dual_table": 1, "dual": 0}, calls
        else:
            assert calls == {"table": 0, "reduce": 8, "dual_table": 0, "dual": 1}, calls
        grads[fused] = [xg.grad.cpu()] + [p.grad.cpu() for p in pair_g.parameters()]
    bound_x = max(2e-2, 1.5 * rel_err(xb.grad, xin.grad))
    assert rel_err(grads[True][0], xin.grad) < bound_x
    for (n, pr), pb, gf, gu in zip(pair_ref.named_parameters(), pair_b16.parameters(), grads[True][1:], grads[False][1:]):
        assert rel_err(gf, pr.grad) < max(2e-2, 1.5 * rel_err(pb.grad, pr.grad)), n
        assert rel_err(gf, gu) < 1e-2, n


@pytest.mark.parametrize("tap", [0, 1])
def test_bn_bwd_table_skipped_for_extra_consumer(monkeypatch, tap):
    """a block output that also feeds a second loss term (an auxiliary head) gets its gradient
    summed by autograd, so the next block's conv1 dgrad epilogue saw only part of it.  The BN backward must
    notice (dy is not the dgrad's dx) and fall back to the reduce pass: the gradients equal the path with
    the epilogue sums off, for the dual output BN (tap 0, downsample block) and an identity bn3 (tap 1)."""
    from pytorchdistributed_amd.models.resnet import resnet50
    from pytorchdistributed_amd.ops import norm as _norm

    torch.manual_seed(0)
    ref = resnet50(dtype=torch.bfloat16)
    blocks = [ref.layer1[0], ref.layer1[1], ref.layer1[2]]
    xin = torch.randn(8, 16, 16, 64).to(torch.bfloat16)
    dy = torch.randn(8, 16, 16, 256).to(torch.bfloat16)
    grads = {}
    for fused in (True, False):
        monkeypatch.setattr(_norm, "_BWD_EPILOGUE", fused)
        bs = [copy.deepcopy(b).to("cuda") for b in blocks]
        xg = xin.to("cuda").requires_grad_()
        h = xg
        aux = None
        for i, b in enumerate(bs):
            h = b(h)
            if i == tap:
                aux = h
        loss = (h.float() * dy.to("cuda").float()).sum() + 0.5 * (aux.float() ** 2).sum()
        loss.backward()
        torch.cuda.synchronize()
        grads[fused] = [xg.grad.cpu()] + [p.grad.cpu() for b in bs for p in b.parameters()]
        # every table handed out was consumed or re-zeroed: nothing stays filled for the next step
        for b in bs:
            for m in b.modules():
                tok = getattr(m, "_bwd_token", None)
                if tok is not None:
                    assert not tok[0]
                    assert m._bwd_table.abs().sum().item() == 0
    for gf, gu in zip(grads[True], grads[False]):
        assert rel_err(gf, gu) < 1e-2


def test_deterministic_mode_bit_identical(monkeypatch):
    """PDA_DETERMINISTIC=1: two runs of the same ResNet-50 steps (DDP flat buffers,
    fused SGD, BN sums from the conv / dgrad epilogues, side-stream split-K weight gradients) end with
    bit-identical parameters and losses — every BN sums table gets one row per output tile, so no two
    atomic adds meet in one element."""
    from pytorchdistributed_amd.models.resnet import resnet50
    from pytorchdistributed_amd.ops import cross_entropy
    from pytorchdistributed_amd.optim import SGD
    from pytorchdistributed_amd.parallel.ddp import DistributedDataParallel

    monkeypatch.setenv("PDA_DETERMINISTIC", "1")

    def run():
        torch.manual_seed(0)
        base = resnet50(device="cuda", dtype=torch.bfloat16)
        model = DistributedDataParallel(base, device_ids=[0])
        opt = SGD(model.parameters(), lr=0.05, momentum=0.9, weight_decay=5e-5)
        g = torch.Generator(device="cuda").manual_seed(1)
        x = torch.randn(24, 112, 112, 3, device="cuda", generator=g).to(torch.bfloat16)
        y = torch.randint(0, 1000, (24,), device="cuda", generator=g)
        losses = []
        for _ in range(3):
            opt.zero_grad()
            loss = cross_entropy(model(x), y)
            loss.backward()
            opt.step()
            losses.append(loss.detach().float().clone())
        torch.cuda.synchronize()
        return [p.detach().clone() for p in base.parameters()], torch.stack(losses), \
            [b.detach().clone() for b in base.buffers()]

    p1, l1, b1 = run()
    p2, l2, b2 = run()
    assert torch.equal(l1, l2), (l1, l2)
    assert all(torch.equal(a, b) for a, b in zip(p1, p2))
    assert all(torch.equal(a, b) for a, b in zip(b1, b2))
