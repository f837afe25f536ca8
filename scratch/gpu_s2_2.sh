#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/s2_2; mkdir -p $D
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > $D/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -4 $D/$name.log | cut -c1-600
  if [ $rc -ne 0 ]; then echo "stopping after $name"; exit $rc; fi
}
step pytest_kern 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_fp32_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
step ring_ab 600 python tools/bench_ring.py
step bench_ring 300 python bench.py
PDA_WIDE_RING=0 step bench_2stage 300 python bench.py
step bench_ring_b 300 python bench.py
