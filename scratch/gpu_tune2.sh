#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > gpurun_out/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -1 gpurun_out/$name.log | cut -c1-300
  if [ $rc -ne 0 ]; then echo "stopping after $name"; exit $rc; fi
}
export PDA_TUNABLEOP=tune PDA_TUNABLEOP_MS=8 PDA_TUNABLEOP_ITERS=4 PYTORCH_TUNABLEOP_VERBOSE=1 PYTORCH_TUNABLEOP_MAX_WARMUP_DURATION_MS=5
PDA_TUNABLEOP_OUT=gpurun_out/tunableop_llama3.csv step tune_llama 900 python -m pytorchdistributed_amd.bench.llama_fsdp --steps 1 --warmup 1
PDA_TUNABLEOP_OUT=gpurun_out/tunableop_gpt2xl.csv step tune_gpt2xl 600 python -m pytorchdistributed_amd.bench.gpt2xl_pp --steps 1 --warmup 1
