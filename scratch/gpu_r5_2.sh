#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > gpurun_out/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -2 gpurun_out/$name.log | cut -c1-250
  if [ $rc -ne 0 ]; then echo "stopping after $name"; exit $rc; fi
}
PDA_WGRAD_STREAM=0 step bench_off 300 python bench.py --steps 30 --warmup 5
PDA_WGRAD_STREAM=1 step bench_on 300 python bench.py --steps 30 --warmup 5
PDA_WGRAD_STREAM=0 step bench_off2 300 python bench.py --steps 30 --warmup 5
PDA_WGRAD_STREAM=1 step bench_on2 300 python bench.py --steps 30 --warmup 5
step pytest_models 600 python -u -m pytest tests/test_models_gpu.py tests/test_graphs_gpu.py tests/test_guards_gpu.py -q -x -p no:cacheprovider --timeout 200 --timeout-method thread
