#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > gpurun_out/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"; grep -v amdgpu gpurun_out/$name.log | tail -4 | cut -c1-900
  if [ $rc -ne 0 ]; then echo "stopping after $name"; exit $rc; fi
}
step tests_all 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu
step bench1 200 python bench.py --steps 20 --warmup 5
step bench1_c10d 200 env PDA_COMM=c10d python bench.py --steps 20 --warmup 5
step bench1_nocomm 200 env PDA_DDP_FORCE_COMM=0 python bench.py --steps 20 --warmup 5
step bench2_gloo 300 env PDA_DIST_BACKEND=gloo python bench.py --gpus 2 --steps 5 --warmup 2 --batch 128
step gpt2 300 python -m pytorchdistributed_amd.bench.gpt2_ddp --steps 10 --warmup 3
step nb03_fp32 500 python -m pytorchdistributed_amd.bench.nb03 --mode parity --dtype fp32 --sweep
