#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
bash scratch/gpu_r5_33.sh || exit 1
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_models_gpu.py -k "bn_bwd_sums or masked_addend or epilogue_bn_sums or conv_fwd_dgrad_wgrad or wide_tile or gemm_layouts or big_tile or native_matches" -s > gpurun_out/t34.log 2>&1; rc=$?; [ $rc -le 1 ] || exit 1
grep -E "worst|passed|failed|Error" gpurun_out/t34.log | tail -8
