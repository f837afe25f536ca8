"""Host (CPU) launch time vs device time of the ResNet-50 bench step: if the Python/autograd launch
path of one step takes about as long as its kernels, the GPU waits on the CPU (kernel gaps).

    python tools/host_overhead.py [--steps 30]
Prints host ms/step (no synchronisation inside the loop: the time to ENQUEUE a step) and device
ms/step (synchronised wall time), plus a cProfile top list of the host side.
"""
import argparse
import cProfile
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pytorchdistributed_amd  # noqa: E402,F401  (raises GPU_MAX_HW_QUEUES before HIP init)
import torch  # noqa: E402

from pytorchdistributed_amd.bench.resnet_ddp import build  # noqa: E402


_parts = None


def _data_of(step):
    """The DeviceSyntheticImages object captured by bench.resnet_ddp.build's step closure."""
    from pytorchdistributed_amd.data.device import DeviceSyntheticImages

    for cell in step.__closure__:
        if isinstance(cell.cell_contents, DeviceSyntheticImages):
            return cell.cell_contents
    raise RuntimeError("no data object in the step closure")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--batch", type=int, default=256)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    global _parts
    model, opt, step = build(a.batch, 224, dev, 0)
    _parts = (model, opt, step.__closure__ and _data_of(step))
    for _ in range(5):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"host enqueue {1e3 * (t1 - t0) / a.steps:.2f} ms/step, device wall {1e3 * (t2 - t0) / a.steps:.2f} ms/step")
    # per-phase host time of the step (no synchronisation): a phase far slower than its Python work
    # hides a blocking call (device sync) that lets the GPU drain
    from pytorchdistributed_amd.bench import resnet_ddp
    ph = {"data": 0.0, "zero": 0.0, "fwd": 0.0, "loss": 0.0, "bwd": 0.0, "opt": 0.0}
    m, o, data = _parts
    from pytorchdistributed_amd.ops import cross_entropy
    torch.cuda.synchronize()
    for _ in range(a.steps):
        t = time.perf_counter()
        x, y = data.next()
        t1 = time.perf_counter(); ph["data"] += t1 - t
        o.zero_grad(set_to_none=True)
        t2 = time.perf_counter(); ph["zero"] += t2 - t1
        out = m(x)
        t3 = time.perf_counter(); ph["fwd"] += t3 - t2
        loss = cross_entropy(out, y)
        t4 = time.perf_counter(); ph["loss"] += t4 - t3
        loss.backward()
        t5 = time.perf_counter(); ph["bwd"] += t5 - t4
        o.step()
        t6 = time.perf_counter(); ph["opt"] += t6 - t5
    torch.cuda.synchronize()
    print("host ms/step by phase:", {k: round(1e3 * v / a.steps, 2) for k, v in ph.items()})
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(5):
        step()
    pr.disable()
    torch.cuda.synchronize()
    pstats.Stats(pr).sort_stats("tottime").print_stats(25)


if __name__ == "__main__":
    main()
