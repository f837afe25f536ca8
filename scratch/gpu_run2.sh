#!/bin/bash
# GPU pass 2: tests, headline bench, other benches, kernel stats.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
step() {  # step <name> <timeout> <cmd...>; stop the script on crash/timeout, continue on plain failure
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > gpurun_out/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -4 gpurun_out/$name.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ] && [ $rc -ne 2 ]; then echo "stopping after $name"; exit $rc; fi
}
step pytest_gpu 900 python -m pytest tests -m gpu -q -p no:cacheprovider
step bench 300 python bench.py --steps 20 --warmup 5
step gpt2_ddp 400 python -m pytorchdistributed_amd.bench.gpt2_ddp --steps 10 --warmup 3
step llama_fsdp 500 python -m pytorchdistributed_amd.bench.llama_fsdp --steps 4 --warmup 2
step gpt2xl_pp 400 python -m pytorchdistributed_amd.bench.gpt2xl_pp --steps 4 --warmup 2
step nb03_parity 400 python -m pytorchdistributed_amd.bench.nb03 --mode parity --devices 0,0
step nb03_clean 500 python -m pytorchdistributed_amd.bench.nb03 --mode clean --devices 0,0 --sweep
