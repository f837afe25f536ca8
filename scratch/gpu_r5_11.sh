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
export MASTER_ADDR=127.0.0.1 MASTER_PORT=29533
PDA_DDP_FORCE_COMM=1 step q4 300 python bench.py --steps 30 --warmup 5
PDA_DDP_FORCE_COMM=1 GPU_MAX_HW_QUEUES=8 step q8 300 python bench.py --steps 30 --warmup 5
PDA_DDP_FORCE_COMM=1 GPU_MAX_HW_QUEUES=16 step q16 300 python bench.py --steps 30 --warmup 5
GPU_MAX_HW_QUEUES=8 step plain_q8 300 python bench.py --steps 30 --warmup 5
step plain_q4 300 python bench.py --steps 30 --warmup 5
