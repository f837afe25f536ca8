#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-v2}
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > gpurun_out/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -3 gpurun_out/$name.log | cut -c1-400
  if [ $rc -ne 0 ]; then echo "stopping after $name"; exit $rc; fi
}
#step pytest_attn 300 python -u -m pytest tests/test_attention_gpu.py -q -x -p no:cacheprovider --timeout 120 --timeout-method thread
#step attn_$tag 240 python tools/bench_attn.py --no-torch
step gpt2_$tag 400 python -m pytorchdistributed_amd.bench.gpt2_ddp --steps 10 --warmup 3
step gpt2_notable_$tag 400 env PDA_TUNABLEOP=0 python -m pytorchdistributed_amd.bench.gpt2_ddp --steps 10 --warmup 3
step prof_gpt2_$tag 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_gpt2_$tag -o prof --output-format csv -- python -m pytorchdistributed_amd.bench.gpt2_ddp --steps 4 --warmup 2
