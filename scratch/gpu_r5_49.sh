#!/bin/bash
# conflict-free epilogue staging: numerics, same-box A/B vs HEAD, conv microbench
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_models_gpu.py -k "gemm or conv or native_matches or linear" > gpurun_out/t49.log 2>&1; rc=$?; tail -3 gpurun_out/t49.log; [ $rc -eq 0 ] || exit 1
for rep in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 2>/dev/null | cut -c90-175 | sed 's/^/new  /' || exit 1
done
timeout -k 10 300 python tools/bench_conv.py --batch 512 --iters 10 > gpurun_out/conv512_v49.jsonl 2>&1 || exit 1
echo ok
