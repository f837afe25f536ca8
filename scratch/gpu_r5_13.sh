#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
for d in 0 1 2; do
  PDA_GEMM_DEBUG_EPI=$d timeout -k 10 300 python tools/bench_conv.py --iters 30 > gpurun_out/epi_dbg$d.jsonl 2>&1 || exit 1
  echo "dbg $d done"
done
