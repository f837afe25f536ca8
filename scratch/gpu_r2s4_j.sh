#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -k "rownorm or add_norm" -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/rn.log 2>&1 || { tail -30 gpurun_out/rn.log; exit 1; }
tail -1 gpurun_out/rn.log
PDA_ROWNORM_FUSED_BWD=0 timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -k "rownorm or add_norm" -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/rn0.log 2>&1 || { tail -30 gpurun_out/rn0.log; exit 1; }
tail -1 gpurun_out/rn0.log
BENCH="python -m pytorchdistributed_amd.bench.gpt2_ddp --steps 10 --warmup 3" CFGS="X=1;PDA_ROWNORM_FUSED_BWD=0" bash scratch/gpu_r2s4_d.sh
