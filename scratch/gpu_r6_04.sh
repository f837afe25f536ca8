#!/bin/bash
# fused BN-backward finalize by channel threshold: same-box A/B
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
out=gpurun_out/bnfin_maxc_ab.jsonl; : > $out
for rep in 1 2; do
for f in 0 64 256 2048; do
  r=$(PDA_BN_BWD_FUSED_MAXC=$f timeout -k 10 150 python bench.py --steps 20 --warmup 5) || exit 1
  echo "{\"bn_bwd_fused_maxc\": $f, \"rep\": $rep, \"bench\": $r}" >> $out
  echo "maxc=$f $(echo $r | cut -c90-140)"
done
done
