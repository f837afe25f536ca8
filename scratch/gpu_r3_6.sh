#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > gpurun_out/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -6 gpurun_out/$name.log | cut -c1-500
  if [ $rc -ne 0 ]; then echo "stopping after $name"; exit $rc; fi
}
step pytest_tp 300 python -u -m pytest tests/test_tensor_parallel_gpu.py -q -x -p no:cacheprovider --timeout 200 --timeout-method thread
