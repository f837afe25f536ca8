#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d gpurun_out/prof48 -o p --output-format csv -- python tools/conv_one.py wgrad 14 256 1024 1 1 10 > gpurun_out/prof48.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d gpurun_out/prof48b -o p --output-format csv -- python tools/conv_one.py wgrad 7 512 2048 1 1 10 > gpurun_out/prof48b.log 2>&1 || exit 1
echo ok
