"""BASELINE config 4: Llama-3 8B FSDP full-shard, tokens/sec (whole job).

    python -m torch.distributed.run --nproc-per-node 8 -m pytorchdistributed_amd.bench.llama_fsdp --gpus 8
Units = transformer blocks (436 MB bf16 all-gather per block in forward and again in backward, one
reduce-scatter per block), prefetch of the next block's all-gather, fused AdamW on the fp32 shards.
"""
from __future__ import annotations

import argparse

import torch

from ..data.device import DeviceSyntheticTokens
from ..models.llama import Llama, LlamaBlock, config
from ..optim import AdamW
from ..parallel.fsdp import FullyShardedDataParallel
from .common import comm_record, emit, mem_record, setup, teardown, timed


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--model", default="llama3-8b")
    # 4 x 4096 tokens per GPU: 15.7k -> 18.6k tok/s over 1 on one MI355X (at world 1 the AdamW pass
    # over all 8.03 B parameters is amortised over more tokens; profiles/r2_transformer_batch_sweep.jsonl)
    ap.add_argument("--batch", type=int, default=4, help="per-GPU sequences")
    ap.add_argument("--seq", type=int, default=4096)
    ap.add_argument("--layers", type=int, default=None, help="override depth (smoke runs only)")
    a = ap.parse_args(argv)
    rank, world, local, device = setup(a.gpus)
    over = {} if a.layers is None else {"n_layers": a.layers}
    torch.manual_seed(0)
    # built on the meta device: FSDP materialises one block at a time and keeps this rank's shard (deferred
    # initialisation: a rank never holds the full 8 B-parameter model, only 1/world of it plus one unit)
    model = Llama(config(a.model, **over), device="meta", dtype=torch.bfloat16)
    n_params = sum(p.numel() for p in model.parameters())
    fsdp = FullyShardedDataParallel(model, unit_types=(LlamaBlock,), device=device)
    opt = AdamW(fsdp.parameters(), lr=3e-4, weight_decay=0.1)
    data = DeviceSyntheticTokens(a.batch, a.seq, model.cfg.vocab_size, device=device, rank=rank)

    def step():
        x, y = data.next()
        opt.zero_grad(set_to_none=True)
        loss = fsdp(x, y)
        loss.backward()
        opt.step()

    secs = timed(step, a.steps, a.warmup, on_start=lambda: fsdp.comm_stats(reset=True))
    comm = comm_record(fsdp, a.steps)
    toks = a.batch * a.seq * world * a.steps / secs
    emit({"metric": "tokens/sec (whole job) Llama-3 FSDP full-shard", "value": round(toks, 1),
          "unit": "tokens/sec", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
          "ms_per_step": round(secs / a.steps * 1e3, 3), "higher_is_better": True, "scaling": "weak",
          "vs_baseline": None, "dtype": "bf16", "data": "synthetic tokens (on-device), random-init weights", "comm": comm,
          "mem": dict(mem_record(device), init_peak_gib=round(fsdp.init_peak_bytes / 2 ** 30, 2)),
          "config": {"model": a.model + ("" if a.layers is None else f"-{a.layers}L"),
                     "global_batch": a.batch * world, "seq_len": a.seq, "parallelism": f"fsdp{world}",
                     "params": n_params}}, rank)
    teardown()


if __name__ == "__main__":
    main()
