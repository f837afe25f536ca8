#!/bin/bash
# fused GELU MLP (sigmoid-form GELU) x wgrad routing: numerics + GPT-2-medium same-box A/B
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_kernels_gpu.py tests/test_models_gpu.py -k "gelu or act or gpt2 or linear" > gpurun_out/t07.log 2>&1; rc=$?; tail -3 gpurun_out/t07.log; [ $rc -eq 0 ] || exit 1
out=gpurun_out/mlp_fused_ab2.jsonl; : > $out
for rep in 1 2; do
for cfg in "0 0" "0 4194304" "1 0" "1 4194304"; do
  set -- $cfg
  r=$(PDA_MLP_FUSED=$1 PDA_WGRAD_BLAS_MIN_OUT=$2 timeout -k 10 200 python -m pytorchdistributed_amd.bench.gpt2_ddp --steps 8 --warmup 3) || exit 1
  echo "{\"mlp_fused\": $1, \"wgrad_blas_min_out\": $2, \"rep\": $rep, \"bench\": $r}" >> $out
  echo "fused=$1 minout=$2 $(echo $r | cut -c40-100)"
done
done
