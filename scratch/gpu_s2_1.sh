#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/s2_1
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > gpurun_out/s2_1/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -3 gpurun_out/s2_1/$name.log | cut -c1-600
  if [ $rc -ne 0 ]; then echo "stopping after $name"; exit $rc; fi
}
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
step bench1 300 python bench.py
step blas 300 python tools/bench_blas.py
