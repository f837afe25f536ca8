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
step kern 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
step gpt2_192 200 python -m pytorchdistributed_amd.bench.gpt2_ddp
PDA_WGRAD_CUS=256 step gpt2_256 200 python -m pytorchdistributed_amd.bench.gpt2_ddp
step gpt2_192b 200 python -m pytorchdistributed_amd.bench.gpt2_ddp
PDA_WGRAD_CUS=256 step gpt2_256b 200 python -m pytorchdistributed_amd.bench.gpt2_ddp
step prof_resnet 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_resnet_v26 -o prof --output-format csv -- python bench.py --steps 8 --warmup 3
