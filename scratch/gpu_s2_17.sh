#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/s2_17; mkdir -p $D
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > $D/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -1 $D/$name.log | cut -c1-200
  if [ $rc -ne 0 ]; then echo "stopping after $name"; exit $rc; fi
}
step pytest_mlp 300 python -u -m pytest tests -m gpu -k "mlp or gelu or gpt2" -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
PDA_MLP_FUSED=1 step gpt2_fused 300 python -m pytorchdistributed_amd.bench.gpt2_ddp --steps 10 --warmup 3
PDA_MLP_FUSED=0 step gpt2_plain 300 python -m pytorchdistributed_amd.bench.gpt2_ddp --steps 10 --warmup 3
PDA_MLP_FUSED=1 step gpt2_fused2 300 python -m pytorchdistributed_amd.bench.gpt2_ddp --steps 10 --warmup 3
PDA_MLP_FUSED=0 step gpt2_plain2 300 python -m pytorchdistributed_amd.bench.gpt2_ddp --steps 10 --warmup 3
