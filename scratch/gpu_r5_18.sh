#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > gpurun_out/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -2 gpurun_out/$name.log | cut -c1-250
  if [ $rc -ne 0 ]; then echo "stopping after $name"; exit $rc; fi
}
step attn_tests 300 python -u -m pytest tests/test_attention_gpu.py -q -x -p no:cacheprovider --timeout 200 --timeout-method thread
PDA_ATTN_FWD=2 step attn_v2 120 python tools/bench_attn.py --iters 20 --no-torch
PDA_ATTN_FWD=3 step attn_v3 120 python tools/bench_attn.py --iters 20 --no-torch
PDA_ATTN_FWD=3 PDA_ATTN_FWD_QG=1 step attn_v3q1 120 python tools/bench_attn.py --iters 20 --no-torch
PDA_ATTN_FWD=3 PDA_ATTN_FWD_QG=2 step attn_v3q2 120 python tools/bench_attn.py --iters 20 --no-torch
