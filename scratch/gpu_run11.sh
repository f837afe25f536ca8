#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > gpurun_out/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -2 gpurun_out/$name.log
  if [ $rc -ne 0 ]; then echo "stopping after $name"; exit $rc; fi
}


step bench_conv 600 python tools/bench_conv.py
step pmc_fwd 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES --kernel-trace --output-format csv -d gpurun_out/pmc_fwd2 -o p -- python tools/conv_one.py fwd 14 256 256 3 1 5
step prof_resnet 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_resnet5 -o prof --output-format csv -- python bench.py --steps 5 --warmup 2
step gpt2 300 python -m pytorchdistributed_amd.bench.gpt2_ddp --steps 10 --warmup 3
