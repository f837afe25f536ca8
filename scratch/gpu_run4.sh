#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > gpurun_out/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -4 gpurun_out/$name.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name"; exit $rc; fi
}
step pytest_gpu 900 python -m pytest tests -m gpu -q -x -p no:cacheprovider
step bench_conv 600 python tools/bench_conv.py
step bench 300 python bench.py --steps 20 --warmup 5
step gpt2_ddp 400 python -m pytorchdistributed_amd.bench.gpt2_ddp --steps 10 --warmup 3
