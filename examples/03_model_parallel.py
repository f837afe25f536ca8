"""Chapter 03 — model parallel and micro-batch pipelining of ResNet-50 (reference
`03 模型并行/03_model_parallel.ipynb`): param count / layer table (torchsummary), single device vs the
two-device layer split vs the split_size=20 pipeline, the split-size sweep, and ``auto_place`` (the
``device_map="auto"`` analogue).  Numbers are written as JSON (and a PNG when matplotlib exists).

    python examples/03_model_parallel.py [--devices 0,1] [--sweep] [--out results.json]

With one GPU the two "devices" are the same GPU (the pipeline still overlaps on two HIP streams).
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorchdistributed_amd.bench import nb03  # noqa: E402
from pytorchdistributed_amd.models import resnet50  # noqa: E402
from pytorchdistributed_amd.parallel.model_parallel import auto_place  # noqa: E402
from pytorchdistributed_amd.utils.summary import summary  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--devices", default=None)
    ap.add_argument("--sweep", action="store_true")
    ap.add_argument("--mode", default="parity", choices=["parity", "clean"])
    ap.add_argument("--out", default="model_parallel_results.json")
    a = ap.parse_args()
    print(summary(resnet50(), (3, 128, 128)))
    placed = auto_place(resnet50(), devices=(["cpu"] if not torch.cuda.is_available() else None))
    print("device_map:", placed.device_map)
    if not torch.cuda.is_available():
        print("no GPU: skipping the timing part")
        return
    argv = ["--mode", a.mode] + (["--devices", a.devices] if a.devices else []) + (["--sweep"] if a.sweep else [])
    import contextlib
    import io

    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        nb03.main(argv)
    res = json.loads(buf.getvalue().strip().splitlines()[-1])
    print(json.dumps(res, indent=1))
    with open(a.out, "w") as fh:
        json.dump(res, fh, indent=1)
    try:
        import matplotlib

        matplotlib.use("Agg")
        import matplotlib.pyplot as plt

        if "sweep" in res["results"]:
            sw = res["results"]["sweep"]
            xs = sorted(int(k) for k in sw)
            plt.errorbar(xs, [sw[str(x)]["mean_s"] for x in xs], yerr=[sw[str(x)]["std_s"] for x in xs])
            plt.xlabel("Pipeline Split Size")
            plt.ylabel("ResNet50 Execution Time (Second)")
            plt.savefig("split_size_tradeoff.png")
    except ImportError:
        pass


if __name__ == "__main__":
    main()
