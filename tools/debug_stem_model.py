"""Run-to-run reproducibility of the ResNet-50 DDP step with the current conv paths (env selects them):
three runs of two SGD steps from one init (single-stream twice, side-stream once); prints the logits
and step-2 gradient differences between runs.  Usage: PDA_CONV_STEM_FWD=1 python tools/debug_stem_model.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorchdistributed_amd.data.device import DeviceSyntheticImages  # noqa: E402
from pytorchdistributed_amd.models.resnet import resnet50  # noqa: E402
from pytorchdistributed_amd.ops import cross_entropy, streams  # noqa: E402
from pytorchdistributed_amd.optim import SGD  # noqa: E402
from pytorchdistributed_amd.parallel.ddp import DistributedDataParallel  # noqa: E402


def rel(a, b):
    return ((a - b).norm() / b.norm().clamp_min(1e-12)).item()


def run(side):
    streams.set_enabled(side)
    try:
        torch.manual_seed(0)
        model = DistributedDataParallel(resnet50(device="cuda", dtype=torch.bfloat16), device_ids=[0])
        opt = SGD(model.parameters(), lr=1e-3, momentum=0.9, weight_decay=5e-5)
        data = DeviceSyntheticImages(16, 96, 1000, device=torch.device("cuda", 0), dtype=torch.bfloat16, seed=3)
        logits = []
        for _ in range(2):
            x, y = data.next()
            opt.zero_grad(set_to_none=True)
            out = model(x)
            logits.append(out.detach().float().clone())
            loss = cross_entropy(out, y)
            loss.backward()
            grads = {n: p.grad.detach().float().clone() for n, p in model.module.named_parameters()}
            opt.step()
        torch.cuda.synchronize()
        return loss.item(), logits, grads
    finally:
        streams.set_enabled(None)


runs = {"a_single": run(False), "b_single": run(False), "c_side": run(True)}
ref = runs["a_single"]
for k, (loss, logits, grads) in runs.items():
    worst = sorted(((rel(grads[n], ref[2][n]), n) for n in grads), reverse=True)[:3]
    print(k, f"loss={loss:.5f}", "logits1", f"{rel(logits[0], ref[1][0]):.2e}", "logits2", f"{rel(logits[1], ref[1][1]):.2e}",
          "worst grads", [(f"{e:.2e}", n) for e, n in worst], flush=True)
