#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/s2_24; mkdir -p $D
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > $D/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"; grep -h '"metric"' $D/$name.log | cut -c1-200
  if [ $rc -ne 0 ]; then tail -3 $D/$name.log; echo "stopping after $name"; exit $rc; fi
}
step gpt2 400 python -m pytorchdistributed_amd.bench.gpt2_ddp --steps 10 --warmup 3
step llama 500 python -m pytorchdistributed_amd.bench.llama_fsdp --steps 5 --warmup 2
step gpt2xl 500 python -m pytorchdistributed_amd.bench.gpt2xl_pp --steps 5 --warmup 2
