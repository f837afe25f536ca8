"""Probe: ResNet-50 bs256 bench step eager vs one HIP graph (N=1)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorchdistributed_amd.bench.resnet_ddp import build  # noqa: E402
from pytorchdistributed_amd.ops import cross_entropy  # noqa: E402
from pytorchdistributed_amd.utils.graphs import GraphedStep  # noqa: E402


def bench(fn, steps=20, warm=5):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(steps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / steps


dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
model, opt, step = build(256, 224, dev, 0)
ms_eager = bench(step)
data_x = None
from pytorchdistributed_amd.data.device import DeviceSyntheticImages  # noqa: E402
data = DeviceSyntheticImages(256, 224, 1000, device=dev, seed=1234)
x0, y0 = data.next()


def inner(x, y):
    opt.zero_grad(set_to_none=True)
    loss = cross_entropy(model(x), y)
    loss.backward()
    opt.step()
    return loss


g = GraphedStep(inner, (x0, y0), optimizer=opt)
xs, ys = g.static_inputs


def gstep():
    data._x, data._y = xs, ys  # generate straight into the graph's static inputs
    data.next()
    return g(xs, ys)


ms_graph = bench(gstep)
print(json.dumps({"eager_ms": round(ms_eager, 3), "graph_ms": round(ms_graph, 3),
                  "eager_img_s": round(256e3 / ms_eager, 1), "graph_img_s": round(256e3 / ms_graph, 1)}))
