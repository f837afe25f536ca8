#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
export PDA_DIST_BACKEND=gloo
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 > gpurun_out/r4_rehearsal2.log 2>&1; rc=$?
echo "rc=$rc"; grep '"metric"' gpurun_out/r4_rehearsal2.log | cut -c1-300
exit $rc
