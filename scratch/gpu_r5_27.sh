#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {
  local name=$1; shift
  timeout -k 10 400 python -m "$@" > gpurun_out/$name.log 2>&1 || { tail -3 gpurun_out/$name.log; exit 1; }
  echo "$name: $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' gpurun_out/$name.log | paste -s)"
}
run g16 pytorchdistributed_amd.bench.gpt2_ddp --steps 10 --warmup 3 --batch 16
run g32 pytorchdistributed_amd.bench.gpt2_ddp --steps 10 --warmup 3 --batch 32
run g48 pytorchdistributed_amd.bench.gpt2_ddp --steps 6 --warmup 2 --batch 48
run l1 pytorchdistributed_amd.bench.llama_fsdp --steps 4 --warmup 2 --batch 1
run l2 pytorchdistributed_amd.bench.llama_fsdp --steps 4 --warmup 2 --batch 2
run l4 pytorchdistributed_amd.bench.llama_fsdp --steps 3 --warmup 1 --batch 4
run x4 pytorchdistributed_amd.bench.gpt2xl_pp --steps 4 --warmup 2 --micro-batch 4
run x8 pytorchdistributed_amd.bench.gpt2xl_pp --steps 4 --warmup 2 --micro-batch 8
