#!/bin/bash
# fused BN-backward sums: numerics, then A/B bench (fused vs reduction pass), then profile
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_models_gpu.py -k "bn_bwd_sums or masked_addend or epilogue_bn_sums or conv_fwd_dgrad_wgrad or wide_tile or gemm_layouts or big_tile" -s > gpurun_out/t31.log 2>&1; rc=$?; [ $rc -le 1 ] || exit 1
grep -E "worst|passed|failed|Error" gpurun_out/t31.log | tail -8
for f in 0 1 0 1; do
  PDA_BN_BWD_SUMS=$f timeout -k 10 300 python bench.py --steps 20 --warmup 5 >> gpurun_out/ab31.jsonl 2>gpurun_out/ab31.err || exit 1
  tail -1 gpurun_out/ab31.jsonl | cut -c90-200
done
for f in 0 1; do
  PDA_WGRAD_STREAM=0 PDA_BN_BWD_SUMS=$f timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof31_$f -o prof --output-format csv -- python bench.py --steps 5 --warmup 2 > gpurun_out/prof31_$f.log 2>&1 || exit 1
done
echo ok
