#!/bin/bash
# rehearse the N-GPU path at the new default batch: one-rank RCCL group under torch.distributed.run
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
PDA_DDP_FORCE_COMM=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/rehearsal45.json 2>gpurun_out/rehearsal45.err || { tail -20 gpurun_out/rehearsal45.err; exit 1; }
cut -c1-260 gpurun_out/rehearsal45.json
timeout -k 10 400 python bench.py --steps 20 --warmup 5 | cut -c1-200
echo ok
