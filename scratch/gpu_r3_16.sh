#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > gpurun_out/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"; grep -v amdgpu gpurun_out/$name.log | tail -21 | cut -c1-230
  if [ $rc -ne 0 ]; then echo "stopping after $name"; exit $rc; fi
}
step pytest_w8 300 python -u -m pytest tests/test_serving_gpu.py -q -x -p no:cacheprovider --timeout 120 --timeout-method thread -k "w8 or int8"
step bench_w8 300 python tools/bench_w8.py
step serve_all 400 python -m pytorchdistributed_amd.bench.llama_serve --batch 32 --prompt 1024 --new 128 --graph --int8 --int8-names wqkv,wo,w13,w2 --int8-head
step serve_all_b8 400 python -m pytorchdistributed_amd.bench.llama_serve --batch 8 --prompt 1024 --new 128 --graph --int8 --int8-names wqkv,wo,w13,w2 --int8-head
