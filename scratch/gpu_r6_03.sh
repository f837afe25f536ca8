#!/bin/bash
# fused BN-backward finalize: numerics, model/graph tests, same-box A/B vs the separate finalize launch
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_kernels_gpu.py tests/test_graphs_gpu.py tests/test_models_gpu.py -k "batchnorm or graphed or resnet" > gpurun_out/t03.log 2>&1; rc=$?; tail -3 gpurun_out/t03.log; [ $rc -eq 0 ] || exit 1
out=gpurun_out/bnfin_ab.jsonl; : > $out
for rep in 1 2; do
for f in 0 1; do
  r=$(PDA_BN_BWD_FUSED=$f timeout -k 10 150 python bench.py --steps 20 --warmup 5) || exit 1
  echo "{\"bn_bwd_fused\": $f, \"rep\": $rep, \"bench\": $r}" >> $out
  echo "fused=$f $(echo $r | cut -c90-140)"
done
done
