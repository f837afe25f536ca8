#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > gpurun_out/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -2 gpurun_out/$name.log | cut -c1-300
  if [ $rc -ne 0 ]; then echo "stopping after $name"; exit $rc; fi
}
export PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_VERBOSE=0
export PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tunableop_gpt2.csv PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=20
step gpt2_tune 700 python -m pytorchdistributed_amd.bench.gpt2_ddp --steps 10 --warmup 3
export PYTORCH_TUNABLEOP_TUNING=0
step gpt2_tuned 400 python -m pytorchdistributed_amd.bench.gpt2_ddp --steps 10 --warmup 3
