"""Chapter 02 (spawn flavour) — the reference's `02 DDP基本概念/ddp_gpus.py`: one process per GPU via
``spawn``, ``ddp_setup`` on 127.0.0.1:12355, ``MyTrainDataset(2048)``, ``Linear(20, 1)``, SGD(lr=1e-3),
``DistributedSampler``, and the ``Trainer`` that prints ``[GPU: i] Epoch: e | Batchsize: 32 | Steps: 32``.

    python examples/02_ddp_gpus.py --max_epochs 5 --batch_size 32 [--nprocs 2]

Backend: RCCL ("nccl") on MI355X, gloo on CPU-only hosts (so the chapter runs anywhere).
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
from pytorchdistributed_amd.train import Trainer  # noqa: E402


def ddp_setup(rank, world_size):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ.setdefault("MASTER_PORT", "12355")
    backend = "nccl" if torch.cuda.is_available() else "gloo"
    if torch.cuda.is_available():
        torch.cuda.set_device(rank)
    pda.init_process_group(backend, rank=rank, world_size=world_size)


def main(rank, world_size, total_epochs, batch_size):
    ddp_setup(rank, world_size)
    dataset = MyTrainDataset(2048)
    loader = DataLoader(dataset, batch_size=batch_size, pin_memory=torch.cuda.is_available(), shuffle=False,
                        sampler=DistributedSampler(dataset))
    model = linear_20_1()
    optimizer = torch.optim.SGD(model.parameters(), lr=1e-3)
    Trainer(model, loader, optimizer, gpu_id=rank, loss_fn=F.cross_entropy).train(total_epochs)
    pda.destroy_process_group()


if __name__ == "__main__":
    ap = argparse.ArgumentParser(description="simple distributed training job")
    ap.add_argument("--max_epochs", type=int, required=True, help="Total epochs to train the model")
    ap.add_argument("--batch_size", default=32, type=int, help="Input batch size on each device (default: 32)")
    ap.add_argument("--nprocs", type=int, default=None, help="default: GPU count, or 2 on CPU")
    a = ap.parse_args()
    world = a.nprocs or (torch.cuda.device_count() or 2)
    pda.spawn(main, args=(world, a.max_epochs, a.batch_size), nprocs=world)
