#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_expert_parallel_gpu.py tests/test_tensor_parallel_gpu.py -q -x -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/ep.log 2>&1; rc=$?; tail -25 gpurun_out/ep.log; exit $rc
