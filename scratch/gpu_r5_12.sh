#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > gpurun_out/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"; grep metric gpurun_out/$name.log | cut -c100-190
  if [ $rc -ne 0 ]; then echo "stopping after $name"; exit $rc; fi
}
export GPU_MAX_HW_QUEUES=4
PDA_DDP_FORCE_COMM=1 step tr_rccl1 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 1 --steps 30 --warmup 5
step plain 300 python bench.py --steps 30 --warmup 5
