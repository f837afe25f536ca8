#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > gpurun_out/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -2 gpurun_out/$name.log
  if [ $rc -ne 0 ]; then echo "stopping after $name"; exit $rc; fi
}
step pytest_kern 600 python -m pytest tests/test_kernels_gpu.py -q -x -p no:cacheprovider
step bench 300 python bench.py --steps 20 --warmup 5
step bench_conv 600 python tools/bench_conv.py
PDA_GEMM_BIG=1 step bench_conv_small 600 python tools/bench_conv.py
