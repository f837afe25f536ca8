#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bs1024 -o prof --output-format csv -- python bench.py --steps 3 --warmup 2 --batch 1024 > gpurun_out/prof_bs1024.log 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bs768 -o prof --output-format csv -- python bench.py --steps 3 --warmup 2 --batch 768 > gpurun_out/prof_bs768.log 2>&1 || exit 1
echo ok
