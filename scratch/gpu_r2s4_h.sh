#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_resnet_v31 -o prof --output-format csv -- python bench.py --steps 8 --warmup 3 > gpurun_out/prof_v31.log 2>&1 || exit $?
PDA_WGRAD_STREAM=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_resnet_v31_single -o prof --output-format csv -- python bench.py --steps 8 --warmup 3 > gpurun_out/prof_v31s.log 2>&1 || exit $?
grep '^{' gpurun_out/prof_v31.log | cut -c1-300
