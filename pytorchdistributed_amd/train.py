"""Trainer with the reference's API (`02 DDP基本概念/ddp_gpus.py:25-55`,
`ddp_gpus_torchrun.py:21-54`) plus snapshot/resume and fault injection.

    trainer = Trainer(model, train_data, optimizer, gpu_id)     # gpu_id=None -> LOCAL_RANK
    trainer.train(max_epochs)

``_run_batch``: zero_grad -> forward -> loss -> backward -> step (`ddp_gpus.py:37-42`);
``_run_epoch`` prints ``[GPU: {id}] Epoch: {e} | Batchsize: {b} | Steps: {n}`` (`ddp_gpus.py:46`) and
calls ``sampler.set_epoch`` (`ddp_gpus.py:47`).  Unlike the reference it does not fetch a throw-away
batch to learn the batch size.
"""
from __future__ import annotations

import os
from typing import Callable, Optional

import torch
import torch.distributed as dist

from . import distributed as pdist
from .ops import cross_entropy
from .parallel.ddp import DistributedDataParallel
from .utils import checkpoint as ckpt
from .utils.fault import maybe_inject
from .utils.log import epoch_line, log


class Trainer:
    def __init__(self, model: torch.nn.Module, train_data, optimizer: torch.optim.Optimizer,
                 gpu_id: Optional[int] = None, save_every: int = 0, snapshot_path: Optional[str] = None,
                 loss_fn: Optional[Callable] = None, wrap_ddp: Optional[bool] = None, ddp_kwargs: Optional[dict] = None):
        if gpu_id is None:
            gpu_id = int(os.environ.get("LOCAL_RANK", "0"))
        self.gpu_id = gpu_id
        self.device = torch.device("cuda", gpu_id) if torch.cuda.is_available() else torch.device("cpu")
        self.model = model.to(self.device)
        self.train_data = train_data
        self.optimizer = optimizer
        self.loss_fn = loss_fn or cross_entropy
        self.save_every = save_every
        self.snapshot_path = snapshot_path
        self.epochs_run = 0
        self.global_step = 0
        self.last_loss = None
        if wrap_ddp is None:
            wrap_ddp = dist.is_initialized()
        if snapshot_path and os.path.exists(snapshot_path):
            self.epochs_run = ckpt.load_snapshot(snapshot_path, self.model, self.optimizer, map_location=self.device)
            log(f"[GPU: {self.gpu_id}] Resuming training from snapshot at Epoch {self.epochs_run}")
        if wrap_ddp:
            self.model = DistributedDataParallel(self.model, device_ids=[gpu_id] if self.device.type == "cuda"
                                                 else None, **(ddp_kwargs or {}))

    def _run_batch(self, source, targets):
        self.optimizer.zero_grad()
        output = self.model(source)
        loss = self.loss_fn(output, targets)
        loss.backward()
        self.optimizer.step()
        self.last_loss = loss.detach()

    def _batch_size(self):
        bs = getattr(self.train_data, "batch_size", None)
        if bs is None:
            src, _ = next(iter(self.train_data))
            bs = len(src)
        return bs

    def _run_epoch(self, epoch):
        b_sz = self._batch_size()
        log(epoch_line(self.gpu_id, epoch, b_sz, len(self.train_data)))
        sampler = getattr(self.train_data, "sampler", None)
        if hasattr(sampler, "set_epoch"):
            sampler.set_epoch(epoch)
        for source, targets in self.train_data:
            maybe_inject(pdist.get_rank(), self.global_step)
            source = source.to(self.device, non_blocking=True)
            targets = targets.to(self.device, non_blocking=True)
            self._run_batch(source, targets)
            self.global_step += 1

    def _save_snapshot(self, epoch):
        if pdist.get_rank() == 0:
            ckpt.save_snapshot(self.snapshot_path, self.model, self.optimizer, epoch + 1)
            log(f"Epoch {epoch} | Training snapshot saved at {self.snapshot_path}")

    def train(self, max_epochs: int):
        for epoch in range(self.epochs_run, max_epochs):
            self._run_epoch(epoch)
            if self.snapshot_path and self.save_every and (epoch + 1) % self.save_every == 0:
                self._save_snapshot(epoch)
