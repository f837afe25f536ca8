#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > gpurun_out/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -1 gpurun_out/$name.log | cut -c1-220
  if [ $rc -ne 0 ]; then echo "stopping after $name"; exit $rc; fi
}
step pytest_tf2 900 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py tests/test_tensor_parallel_gpu.py tests/test_serving_gpu.py tests/test_graphs_gpu.py tests/test_attention_gpu.py -q -x -p no:cacheprovider --timeout 200 --timeout-method thread
step gpt2 400 python -m pytorchdistributed_amd.bench.gpt2_ddp --steps 10 --warmup 3
step llama 500 python -m pytorchdistributed_amd.bench.llama_fsdp --steps 5 --warmup 2
step xl 500 python -m pytorchdistributed_amd.bench.gpt2xl_pp --steps 5 --warmup 2
