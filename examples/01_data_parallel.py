"""Chapter 01 — single-process DataParallel (reference `01 数据并行/01_multi_gpus_data_parallelism.ipynb`,
raw lines 33-145): SimpleDataset (randn(1000, 10), all-zero labels), the 4-layer MLP (1,165 params),
``DataParallel`` over every visible device, and the reference's two printouts.

    python examples/01_data_parallel.py              # GPUs if present, else CPU

On MI355X each replica runs on its own device and HIP stream; replicate / scatter / gather are peer
copies.  Unlike the reference this also runs a backward + SGD step so the
gradient reduce-to-device-0 path is exercised.
"""
import os
import sys

import torch
from torch.utils.data import DataLoader

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorchdistributed_amd.data import SimpleDataset  # noqa: E402
from pytorchdistributed_amd.models import TutorialMLP  # noqa: E402
from pytorchdistributed_amd.parallel.dp import DataParallel  # noqa: E402

input_size, hidden_size, output_size, batch_size, data_size = 10, 20, 5, 32, 1000


def main():
    loader = DataLoader(SimpleDataset(data_size), batch_size=batch_size, shuffle=True)
    x, y = next(iter(loader))
    print(f"Data shape: {list(x.shape)}, Labels shape: {list(y.shape)}")
    model = TutorialMLP()
    dev = torch.device("cuda", 0) if torch.cuda.is_available() else torch.device("cpu")
    model = model.to(dev)
    if torch.cuda.device_count() > 1:
        model = DataParallel(model)  # device_ids=None -> all GPUs, output on cuda:0 (NB01:119-120)
    opt = torch.optim.SGD(model.parameters(), lr=0.01)
    for i, (data, labels) in enumerate(loader):
        out = model(data.to(dev))
        print(f"Outside: input size {list(data.shape)} output_size {list(out.shape)}")
        loss = torch.nn.functional.mse_loss(out, labels.to(dev).float())
        opt.zero_grad()
        loss.backward()
        opt.step()
        if i == 2:
            break


if __name__ == "__main__":
    main()
