"""Parameter-server training (the PS-worker concept of `02 DDP基本概念/02_ddp.ipynb:28-31`, which the
reference only describes): every rank trains on its shard, gradients are reduced to rank 0, rank 0 alone
holds the optimizer and steps it, and the parameters are broadcast back.  The data / model are chapter 02's
(`MyTrainDataset`, the 20 -> 1 linear layer), so the printed loss is 0 as in the reference demo (C = 1
soft-target cross-entropy).

    python -m pytorchdistributed_amd.run --nproc-per-node=2 --master-addr 127.0.0.1 \
        examples/04_parameter_server.py --epochs 2 --batch_size 32
"""
import argparse
import os
import sys

import torch
import torch.nn.functional as F
from torch.utils.data import DataLoader

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pytorchdistributed_amd as pda  # noqa: E402
from pytorchdistributed_amd.data import DistributedSampler, MyTrainDataset  # noqa: E402
from pytorchdistributed_amd.models.mlp import linear_20_1  # noqa: E402
from pytorchdistributed_amd.parallel import ParameterServer  # noqa: E402


def main(epochs, batch_size):
    local = int(os.environ.get("LOCAL_RANK", "0"))
    use_gpu = torch.cuda.is_available()
    if use_gpu:
        torch.cuda.set_device(local)
    pda.init_process_group("nccl" if use_gpu else "gloo")
    device = torch.device("cuda", local) if use_gpu else torch.device("cpu")
    dataset = MyTrainDataset(2048)
    sampler = DistributedSampler(dataset, shuffle=True)
    loader = DataLoader(dataset, batch_size=batch_size, sampler=sampler)
    ps = ParameterServer(linear_20_1().to(device), lambda params: torch.optim.SGD(params, lr=1e-3))
    for epoch in range(epochs):
        sampler.set_epoch(epoch)
        for x, y in loader:
            ps.zero_grad()
            loss = F.cross_entropy(ps(x.to(device)), y.to(device))
            loss.backward()
            ps.step()
        role = "server" if ps.is_server else "worker"
        print(f"[rank {ps.rank} {role}] epoch {epoch} | steps {ps.steps} | loss {loss.item():.4f} | "
              f"comm {ps.comm_bytes / 2**20:.2f} MiB")
    pda.destroy_process_group()


if __name__ == "__main__":
    ap = argparse.ArgumentParser(description="parameter-server training job")
    ap.add_argument("--epochs", default=2, type=int)
    ap.add_argument("--batch_size", default=32, type=int)
    a = ap.parse_args()
    main(a.epochs, a.batch_size)
