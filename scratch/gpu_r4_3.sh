#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > gpurun_out/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"; grep '"metric"' gpurun_out/$name.log | cut -c1-260
  if [ $rc -ne 0 ]; then tail -3 gpurun_out/$name.log; echo "stopping after $name"; exit $rc; fi
}
step r4_gpt2 400 python -m pytorchdistributed_amd.bench.gpt2_ddp --steps 10 --warmup 3
step r4_llama 600 python -m pytorchdistributed_amd.bench.llama_fsdp --steps 5 --warmup 2
step r4_gpt2xl 600 python -m pytorchdistributed_amd.bench.gpt2xl_pp --steps 5 --warmup 2
