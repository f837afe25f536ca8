#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > gpurun_out/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -2 gpurun_out/$name.log | cut -c1-400
  if [ $rc -ne 0 ]; then echo "stopping after $name"; exit $rc; fi
}
step budgets 200 python -u -m pytest tests/test_kernels_gpu.py -k budgets -x -v -p no:cacheprovider --timeout 150 --timeout-method thread
PDA_WGRAD_STREAM=0 step prof_gpt2_single 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_gpt2_v27_single -o prof --output-format csv -- python -m pytorchdistributed_amd.bench.gpt2_ddp --steps 4 --warmup 2
step prof_gpt2 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_gpt2_v27 -o prof --output-format csv -- python -m pytorchdistributed_amd.bench.gpt2_ddp --steps 4 --warmup 2
