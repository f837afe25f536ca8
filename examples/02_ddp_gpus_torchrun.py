"""Chapter 02 (launcher flavour) — the reference's `02 DDP基本概念/ddp_gpus_torchrun.py`, run by the
torchrun-compatible launcher (or torchrun itself):

    python -m pytorchdistributed_amd.run --nproc-per-node=2 --master-port=12355 \
        examples/02_ddp_gpus_torchrun.py --max_epochs 5 --batch_size 32

Rendezvous from the env contract (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_*), dataset built inside
every rank, ``DistributedSampler(shuffle=True)``; add ``--save_every 1 --snapshot_path snap.pt`` and
``--max-restarts 1`` on the launcher to see snapshot/resume after an injected failure
(``PDA_FAULT=1:40:crash``).
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


def ddp_setup():
    local = int(os.environ["LOCAL_RANK"])
    if torch.cuda.is_available():
        torch.cuda.set_device(local)
    pda.init_process_group("nccl" if torch.cuda.is_available() else "gloo")


def main(total_epochs, batch_size, save_every, snapshot_path):
    ddp_setup()
    dataset = MyTrainDataset(2048)
    loader = DataLoader(dataset, batch_size=batch_size, pin_memory=torch.cuda.is_available(), shuffle=False,
                        sampler=DistributedSampler(dataset, shuffle=True))
    model = linear_20_1()
    optimizer = torch.optim.SGD(model.parameters(), lr=1e-3)
    Trainer(model, loader, optimizer, save_every=save_every, snapshot_path=snapshot_path,
            loss_fn=F.cross_entropy).train(total_epochs)
    pda.destroy_process_group()


if __name__ == "__main__":
    ap = argparse.ArgumentParser(description="simple distributed training job")
    ap.add_argument("--max_epochs", default=10, type=int, help="Total epochs to train the model")
    ap.add_argument("--batch_size", default=32, type=int, help="Input batch size on each device (default: 32)")
    ap.add_argument("--save_every", default=0, type=int)
    ap.add_argument("--snapshot_path", default=None)
    a = ap.parse_args()
    print(f"local_rank: {os.environ.get('LOCAL_RANK')}, world_size: {os.environ.get('WORLD_SIZE')}")
    main(a.max_epochs, a.batch_size, a.save_every, a.snapshot_path)
