#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > gpurun_out/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"; grep -v amdgpu gpurun_out/$name.log | tail -2 | cut -c1-400
  if [ $rc -ne 0 ]; then echo "stopping after $name"; exit $rc; fi
}
step llama 500 python -m pytorchdistributed_amd.bench.llama_fsdp --steps 5 --warmup 2
step gpt2 400 python -m pytorchdistributed_amd.bench.gpt2_ddp --steps 10 --warmup 3
step gpt2xl 500 python -m pytorchdistributed_amd.bench.gpt2xl_pp --steps 5 --warmup 2
step nb03 500 python -m pytorchdistributed_amd.bench.nb03 --mode parity
step serve_bf16 400 python -m pytorchdistributed_amd.bench.llama_serve --batch 32 --prompt 1024 --new 128 --graph
