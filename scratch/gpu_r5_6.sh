#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > gpurun_out/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -1 gpurun_out/$name.log | cut -c1-260
  if [ $rc -ne 0 ]; then echo "stopping after $name"; exit $rc; fi
}



PDA_WGRAD_STREAM=0 step llama_off 500 python -m pytorchdistributed_amd.bench.llama_fsdp --steps 5 --warmup 2
PDA_WGRAD_STREAM=1 step llama_on 500 python -m pytorchdistributed_amd.bench.llama_fsdp --steps 5 --warmup 2
PDA_WGRAD_STREAM=0 step xl_off 500 python -m pytorchdistributed_amd.bench.gpt2xl_pp --steps 5 --warmup 2
PDA_WGRAD_STREAM=1 step xl_on 500 python -m pytorchdistributed_amd.bench.gpt2xl_pp --steps 5 --warmup 2
