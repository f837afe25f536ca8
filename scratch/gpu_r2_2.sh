#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > gpurun_out/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -3 gpurun_out/$name.log
  if [ $rc -ne 0 ]; then echo "stopping after $name"; exit $rc; fi
}
step pytest_kern 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -q -x -p no:cacheprovider --timeout 120 --timeout-method thread
step bench 300 python bench.py --steps 20 --warmup 5
step bench_bn 200 python tools/bench_bn.py
step gpt2 300 python -m pytorchdistributed_amd.bench.gpt2_ddp --steps 10 --warmup 3
step prof_resnet 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_resnet_r2b -o prof --output-format csv -- python bench.py --steps 5 --warmup 2
step prof_gpt2 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_gpt2_r2b -o prof --output-format csv -- python -m pytorchdistributed_amd.bench.gpt2_ddp --steps 3 --warmup 1
