#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python tools/bench_conv.py --batch 512 --iters 10 --compare > gpurun_out/conv512_cmp.jsonl 2>&1 || exit 1
echo ok
