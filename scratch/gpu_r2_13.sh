#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > gpurun_out/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -3 gpurun_out/$name.log | cut -c1-500
  if [ $rc -ne 0 ]; then echo "stopping after $name"; exit $rc; fi
}
step pytest_fsdp 400 python -u -m pytest tests/test_models_gpu.py -k fsdp -x -v -p no:cacheprovider --timeout 240 --timeout-method thread
step llama 500 python -m pytorchdistributed_amd.bench.llama_fsdp --steps 5 --warmup 2
step prof_llama 500 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_llama_r2 -o prof --output-format csv -- python -m pytorchdistributed_amd.bench.llama_fsdp --steps 3 --warmup 1
