#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
out=gpurun_out/r2s4_transformers.jsonl
: > $out
run() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > gpurun_out/tf_$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/tf_$name.log; exit $rc; fi
  grep '^{' gpurun_out/tf_$name.log >> $out
  grep '^{' gpurun_out/tf_$name.log | cut -c1-220
}
run gpt2 200 python -m pytorchdistributed_amd.bench.gpt2_ddp
run llama 400 python -m pytorchdistributed_amd.bench.llama_fsdp
run gpt2xl 300 python -m pytorchdistributed_amd.bench.gpt2xl_pp
