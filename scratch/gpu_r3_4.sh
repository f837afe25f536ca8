#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > gpurun_out/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -12 gpurun_out/$name.log | cut -c1-400
  if [ $rc -ne 0 ]; then echo "stopping after $name"; exit $rc; fi
}
step pytest_serving 300 python -u -m pytest tests/test_serving_gpu.py -v -x -p no:cacheprovider --timeout 120 --timeout-method thread
step bench_decode 200 python tools/bench_decode.py
step llama_serve 400 python -m pytorchdistributed_amd.bench.llama_serve --batch 32 --prompt 1024 --new 64
