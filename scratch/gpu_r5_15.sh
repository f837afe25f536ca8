#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
ab() {  # name dir args...
  local name=$1 dir=$2; shift 2
  (cd "$dir" && timeout -k 10 400 python -m "$@" > $R/gpurun_out/$name.log 2>&1)
  local rc=$?
  echo "== $name rc=$rc"; grep metric $R/gpurun_out/$name.log | cut -c60-160
  [ $rc -eq 0 ] || exit $rc
}
ab gpt2_base gpurun_ab/base pytorchdistributed_amd.bench.gpt2_ddp --steps 10 --warmup 3
ab gpt2_new . pytorchdistributed_amd.bench.gpt2_ddp --steps 10 --warmup 3




ab gpt2_base2 gpurun_ab/base pytorchdistributed_amd.bench.gpt2_ddp --steps 10 --warmup 3
ab gpt2_new2 . pytorchdistributed_amd.bench.gpt2_ddp --steps 10 --warmup 3
