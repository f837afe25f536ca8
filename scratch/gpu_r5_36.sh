#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python tools/bench_conv.py --batch 512 --iters 10 --wide 0 > gpurun_out/conv512_w0.jsonl 2>&1 || exit 1
timeout -k 10 300 python tools/bench_conv.py --batch 512 --iters 10 --wide 2 > gpurun_out/conv512_w2.jsonl 2>&1 || exit 1
timeout -k 10 400 python tools/bench_conv.py --batch 512 --iters 10 --torch > gpurun_out/conv512_auto_torch.jsonl 2>&1 || exit 1
echo ok
