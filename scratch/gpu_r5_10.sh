#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > gpurun_out/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -1 gpurun_out/$name.log | cut -c1-250
  if [ $rc -ne 0 ]; then echo "stopping after $name"; exit $rc; fi
}
export MASTER_ADDR=127.0.0.1 MASTER_PORT=29533
PDA_DDP_FORCE_COMM=1 step bench_rccl1b 300 python bench.py --steps 30 --warmup 5
PDA_DDP_FORCE_COMM=1 PDA_WGRAD_STREAM=0 step bench_rccl1_noside 300 python bench.py --steps 30 --warmup 5
PDA_DDP_FORCE_COMM=1 PDA_COMM_PRIORITY=0 step bench_rccl1_noprio 300 python bench.py --steps 30 --warmup 5
PDA_DDP_FORCE_COMM=1 step prof_rccl1 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_rccl1 -o prof --output-format csv -- python bench.py --steps 5 --warmup 2
