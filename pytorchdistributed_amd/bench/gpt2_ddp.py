"""BASELINE config 3: GPT-2-medium DDP bf16, tokens/sec (whole job).

One process per GPU (torchrun / pda-run env contract); synthetic token batches generated on device;
bf16 parameters + fp32 masters, fused AdamW, bucketed DDP all-reduce over RCCL overlapped with backward.
    python -m torch.distributed.run --nproc-per-node 8 -m pytorchdistributed_amd.bench.gpt2_ddp --gpus 8
"""
from __future__ import annotations

import argparse

import torch

from ..data.device import DeviceSyntheticTokens
from ..models.gpt2 import GPT2, config
from ..optim import AdamW
from ..parallel.ddp import DistributedDataParallel
from .common import comm_record, emit, group_info, mem_record, setup, teardown, timed


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--model", default="gpt2-medium")
    # 32 x 1024 tokens per GPU (288 GB HBM): 293k -> 308k tok/s over 16 on one MI355X
    # (profiles/r2_transformer_batch_sweep.jsonl)
    ap.add_argument("--batch", type=int, default=32, help="per-GPU sequences")
    ap.add_argument("--seq", type=int, default=1024)
    ap.add_argument("--layers", type=int, default=None, help="override depth (smoke runs only)")
    a = ap.parse_args(argv)
    # N = 1 runs the DDP path over a one-rank RCCL group (bucket all-reduces timed, as at N > 1; the
    # ResNet headline does the same): PDA_DDP_FORCE_COMM=0 skips it
    rank, world, local, device = setup(a.gpus, one_rank_group=True)
    over = {} if a.layers is None else {"n_layer": a.layers}
    torch.manual_seed(0)
    model = GPT2(config(a.model, n_positions=max(1024, a.seq), **over), device=device, dtype=torch.bfloat16)
    ddp = DistributedDataParallel(model, device_ids=[local] if device.type == "cuda" else None)
    opt = AdamW(ddp.parameters(), lr=3e-4, weight_decay=0.1)
    data = DeviceSyntheticTokens(a.batch, a.seq, model.cfg.vocab_size, device=device, rank=rank)

    def step():
        x, y = data.next()
        opt.zero_grad(set_to_none=True)
        loss = ddp(x, y)
        loss.backward()
        opt.step()

    secs = timed(step, a.steps, a.warmup, on_start=lambda: ddp.comm_stats(reset=True))
    comm = comm_record(ddp, a.steps)
    toks = a.batch * a.seq * world * a.steps / secs
    emit({"metric": "tokens/sec (whole job) GPT-2 DDP", "value": round(toks, 1), "unit": "tokens/sec",
          "n_gpus": world, "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(secs / a.steps * 1e3, 3),
          "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "bf16",
          "data": "synthetic tokens (on-device), random-init weights", "comm": comm,
          **group_info(device), "mem": mem_record(device),
          "config": {"model": a.model + ("" if a.layers is None else f"-{a.layers}L"),
                     "global_batch": a.batch * world, "seq_len": a.seq, "parallelism": f"dp{world}",
                     "params": model.num_params()}}, rank)
    teardown()


if __name__ == "__main__":
    main()
