#!/bin/bash
# wave-contiguous BN apply kernels: numerics, same-box A/B vs HEAD build, single-stream profile
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_models_gpu.py -k "batchnorm or native_matches or masked_addend or side_stream" > gpurun_out/t35.log 2>&1; rc=$?; tail -3 gpurun_out/t35.log; [ $rc -eq 0 ] || exit 1
for rep in 1 2; do
  timeout -k 10 300 python ab_base/bench.py --steps 20 --warmup 5 2>/dev/null | cut -c90-175 | sed 's/^/base /' || exit 1
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 2>/dev/null | cut -c90-175 | sed 's/^/new  /' || exit 1
done
PDA_WGRAD_STREAM=0 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof35 -o prof --output-format csv -- python bench.py --steps 5 --warmup 2 > gpurun_out/prof35.log 2>&1 || exit 1
echo ok
