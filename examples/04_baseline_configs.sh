#!/bin/bash
# BASELINE.json configs on one node (N GPUs).  Each prints one JSON line.
#   1  MNIST-MLP DDP on CPU (gloo, 2 ranks)       2  ResNet-50 DDP (headline, bench.py)
#   3  GPT-2-medium DDP                            4  Llama-3-8B FSDP full-shard
#   5  GPT-2-XL pipeline (4 stages) x DDP 2
set -e
N=${N:-8}
RUN="python -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 --master-port 29511"
python -m pytorchdistributed_amd.run --standalone --nproc-per-node 2 -m pytorchdistributed_amd.bench.mnist_ddp
$RUN bench.py --gpus $N
$RUN -m pytorchdistributed_amd.bench.gpt2_ddp --gpus $N
$RUN -m pytorchdistributed_amd.bench.llama_fsdp --gpus $N
$RUN -m pytorchdistributed_amd.bench.gpt2xl_pp --gpus $N
