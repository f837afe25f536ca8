#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
for d in 0 1 2 3; do
  PDA_ATTN_DBG=$d timeout -k 10 120 python tools/bench_attn.py --iters 20 --no-torch > gpurun_out/attn_dbg$d.log 2>&1 || exit 1
  echo "dbg $d: $(grep gpt2 gpurun_out/attn_dbg$d.log | grep -o '"fwd_ms": [0-9.]*')"
done
