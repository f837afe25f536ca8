#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > gpurun_out/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -3 gpurun_out/$name.log
  if [ $rc -ne 0 ]; then echo "stopping after $name"; exit $rc; fi
}
step pytest_attn 600 python -m pytest tests/test_attention_gpu.py -q -x -p no:cacheprovider
step gpt2 300 python -m pytorchdistributed_amd.bench.gpt2_ddp --steps 10 --warmup 3
step llama 400 python -m pytorchdistributed_amd.bench.llama_fsdp --steps 4 --warmup 2
export TMPDIR=/tmp
step prof_llama 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_llama2 -o prof --output-format csv -- python -m pytorchdistributed_amd.bench.llama_fsdp --steps 2 --warmup 1
step prof_gpt2 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_gpt2b -o prof --output-format csv -- python -m pytorchdistributed_amd.bench.gpt2_ddp --steps 3 --warmup 1
