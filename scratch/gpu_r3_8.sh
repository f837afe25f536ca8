#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > gpurun_out/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -22 gpurun_out/$name.log | cut -c1-260
  if [ $rc -ne 0 ]; then echo "stopping after $name"; exit $rc; fi
}
step pytest_w8 300 python -u -m pytest tests/test_serving_gpu.py -q -x -p no:cacheprovider --timeout 120 --timeout-method thread -k "w8 or int8"
step bench_w8 300 python tools/bench_w8.py
step serve_int8 400 python -m pytorchdistributed_amd.bench.llama_serve --batch 32 --prompt 1024 --new 128 --graph --int8
