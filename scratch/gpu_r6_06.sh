#!/bin/bash
# fused GELU MLP: numerics, GPT-2 model tests, GPT-2-medium bench A/B (fused vs PDA_MLP_FUSED=0)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_kernels_gpu.py tests/test_models_gpu.py -k "gelu or gemm or gpt2 or linear" > gpurun_out/t06.log 2>&1; rc=$?; tail -3 gpurun_out/t06.log; [ $rc -eq 0 ] || exit 1
out=gpurun_out/mlp_fused_ab.jsonl; : > $out
for rep in 1 2; do
for f in 0 1; do
  r=$(PDA_MLP_FUSED=$f timeout -k 10 200 python -m pytorchdistributed_amd.bench.gpt2_ddp --steps 8 --warmup 3) || exit 1
  echo "{\"mlp_fused\": $f, \"rep\": $rep, \"bench\": $r}" >> $out
  echo "fused=$f $(echo $r | cut -c40-120)"
done
done
