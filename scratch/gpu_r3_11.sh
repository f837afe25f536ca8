#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > gpurun_out/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"; grep -o '"weights.*' gpurun_out/$name.log | cut -c1-300
  if [ $rc -ne 0 ]; then echo "stopping after $name"; tail -5 gpurun_out/$name.log; exit $rc; fi
}
step serve_w13h 400 python -m pytorchdistributed_amd.bench.llama_serve --batch 32 --prompt 1024 --new 128 --graph --int8 --int8-names w13 --int8-head
step serve_w13h_b8 400 python -m pytorchdistributed_amd.bench.llama_serve --batch 8 --prompt 1024 --new 128 --graph --int8 --int8-names w13 --int8-head
step serve_bf16_b8 400 python -m pytorchdistributed_amd.bench.llama_serve --batch 8 --prompt 1024 --new 128 --graph
