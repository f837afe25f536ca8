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
step pytest_attn 300 python -u -m pytest tests/test_attention_gpu.py -q -x -p no:cacheprovider --timeout 120 --timeout-method thread
step pytest_attn_qg1 300 env PDA_ATTN_FWD_QG=1 python -u -m pytest tests/test_attention_gpu.py -q -x -p no:cacheprovider --timeout 120 --timeout-method thread -k fwd_bwd
step attn_qg2 240 env PDA_ATTN_FWD_QG=2 python tools/bench_attn.py --no-torch
step attn_qg1 240 env PDA_ATTN_FWD_QG=1 python tools/bench_attn.py --no-torch
