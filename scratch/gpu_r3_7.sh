#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > gpurun_out/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -4 gpurun_out/$name.log | cut -c1-500
  if [ $rc -ne 0 ]; then echo "stopping after $name"; exit $rc; fi
}
step pytest_serving 300 python -u -m pytest tests/test_serving_gpu.py tests/test_tensor_parallel_gpu.py -q -x -p no:cacheprovider --timeout 200 --timeout-method thread
step serve_graph 400 python -m pytorchdistributed_amd.bench.llama_serve --batch 32 --prompt 1024 --new 128 --graph
step prof_serve 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_serve2 -o prof --output-format csv -- python -m pytorchdistributed_amd.bench.llama_serve --batch 32 --prompt 1024 --new 64 --graph --repeat 1
