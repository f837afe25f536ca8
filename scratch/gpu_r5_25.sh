#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > gpurun_out/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"; grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"final_loss": [0-9.-]*\|"n_gpus": [0-9]*' gpurun_out/$name.log | paste -s
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/$name.log; echo "stopping after $name"; exit $rc; fi
}
step bench512 300 python bench.py --steps 20 --warmup 5
PDA_DDP_FORCE_COMM=1 step rccl1_512 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 1 --steps 20 --warmup 5
PDA_DIST_BACKEND=gloo step gloo2_512 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2
