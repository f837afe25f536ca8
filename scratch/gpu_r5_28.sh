#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bs512 -o prof --output-format csv -- python bench.py --steps 5 --warmup 2 > gpurun_out/prof_bs512.log 2>&1 || exit 1
PDA_WGRAD_STREAM=0 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bs512_1s -o prof --output-format csv -- python bench.py --steps 5 --warmup 2 > gpurun_out/prof_bs512_1s.log 2>&1 || exit 1
timeout -k 10 300 python tools/bench_conv.py --batch 512 --iters 10 > gpurun_out/conv_bs512.jsonl 2>&1 || exit 1
echo ok
