"""Step-1 / step-2 gradient agreement of ResNet-50 under DDP(world 1) across execution variants.

    python tools/debug_dualbwd.py            # lr 0.05 (the old side-stream test's setting)
    LR=0.001 python tools/debug_dualbwd.py

Compares single- vs side-stream weight gradients and the one-pass dual BN backward vs two BN backwards
(ops/norm.py:_DUAL_BWD).  Used to show that at lr 0.05 step 2 is chaotic — a last-bit difference of
one float-atomic BN sum moves step-2 BN gradients by O(1) even between two runs of one configuration —
while step-1 gradients agree to 1e-4 and at lr 1e-3 every variant agrees bitwise.
"""
import os, sys, torch
sys.path.insert(0, os.getcwd())
from pytorchdistributed_amd.data.device import DeviceSyntheticImages
from pytorchdistributed_amd.models.resnet import resnet50
from pytorchdistributed_amd.ops import cross_entropy, streams
from pytorchdistributed_amd.ops import norm as Nm
from pytorchdistributed_amd.optim import SGD
from pytorchdistributed_amd.parallel.ddp import DistributedDataParallel


def rel(a, b):
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


LR = float(os.environ.get('LR', '0.05'))


def run(side, dual_bwd, ddp=True):
    Nm._DUAL_BWD = dual_bwd
    streams.set_enabled(side)
    torch.manual_seed(0)
    m = resnet50(device="cuda", dtype=torch.bfloat16)
    model = DistributedDataParallel(m, device_ids=[0]) if ddp else m
    opt = SGD(model.parameters(), lr=LR, momentum=0.9, weight_decay=5e-5)
    data = DeviceSyntheticImages(16, 96, 1000, device=torch.device("cuda", 0), dtype=torch.bfloat16, seed=3)
    first = None
    for _ in range(2):
        x, y = data.next()
        opt.zero_grad(set_to_none=True)
        loss = cross_entropy(model(x), y)
        loss.backward()
        mm = model.module if ddp else model
        grads = {n: p.grad.detach().float().clone() for n, p in mm.named_parameters()}
        if first is None:
            first = grads
        opt.step()
    torch.cuda.synchronize()
    streams.set_enabled(None)
    return loss.item(), grads, first


def cmp(tag, a, b):
    errs = sorted(((rel(a[1][n], b[1][n]), n) for n in a[1]), reverse=True)
    e1 = sorted(((rel(a[2][n], b[2][n]), n) for n in a[2]), reverse=True)
    print(tag, "loss", a[0], b[0], "step2 worst", [(round(e, 4), n) for e, n in errs[:3]],
          "step1 worst", [(round(e, 4), n) for e, n in e1[:3]], flush=True)


base = run(False, True)
cmp("single dual vs single dual (determinism)", run(False, True), base)
cmp("side dual vs single dual", run(True, True), base)
cmp("single sep vs single dual", run(False, False), base)
cmp("side sep vs single sep", run(True, False), run(False, False))
cmp("nodpp single dual vs nodpp single sep", run(False, True, False), run(False, False, False))
