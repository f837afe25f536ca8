#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > gpurun_out/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"; grep metric gpurun_out/$name.log | cut -c100-200
  if [ $rc -ne 0 ]; then echo "stopping after $name"; exit $rc; fi
}
PDA_WGRAD_STREAM=0 step b_off 300 python bench.py --steps 30 --warmup 5
PDA_WGRAD_STREAM=1 step b_on 300 python bench.py --steps 30 --warmup 5
PDA_WGRAD_CUS=64 step b_cu64 300 python bench.py --steps 30 --warmup 5
PDA_WGRAD_CUS=128 step b_cu128 300 python bench.py --steps 30 --warmup 5
PDA_WGRAD_CUS=192 step b_cu192 300 python bench.py --steps 30 --warmup 5
PDA_WGRAD_CUS=224 step b_cu224 300 python bench.py --steps 30 --warmup 5
PDA_WGRAD_STREAM=1 step b_on2 300 python bench.py --steps 30 --warmup 5
