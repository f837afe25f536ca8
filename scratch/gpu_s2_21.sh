#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/s2_21; mkdir -p $D
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > $D/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -2 $D/$name.log | cut -c1-300
  if [ $rc -ne 0 ]; then echo "stopping after $name"; exit $rc; fi
}
step pytest_conv 400 python -u -m pytest tests/test_kernels_gpu.py -k "conv" -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
step conv_new 400 python tools/bench_conv.py --batch 640 --iters 10
PDA_CONV_1X1_PLAIN=0 step conv_old 400 python tools/bench_conv.py --batch 640 --iters 10
step bench_new 300 python bench.py
PDA_CONV_1X1_PLAIN=0 step bench_old 300 python bench.py
