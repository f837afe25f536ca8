#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > gpurun_out/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"; grep -v amdgpu gpurun_out/$name.log | tail -1 | grep -o '"value[^,]*\|"gemm_table[^,]*\|"decode_ms_per_step[^,]*\|"prefill_ms[^,]*'
  if [ $rc -ne 0 ]; then echo "stopping after $name"; exit $rc; fi
}
step llama_t 500 python -m pytorchdistributed_amd.bench.llama_fsdp --steps 5 --warmup 2
step llama_off 500 env PDA_TUNABLEOP=0 python -m pytorchdistributed_amd.bench.llama_fsdp --steps 5 --warmup 2
step serve_t 400 python -m pytorchdistributed_amd.bench.llama_serve --batch 32 --prompt 1024 --new 128 --graph
