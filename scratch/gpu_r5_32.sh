#!/bin/bash
# fused BN-backward sums: numerics, then A/B bench (fused vs reduction pass), then profile
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
true
true
for f in 0 1 0 1; do
  PDA_BN_BWD_SUMS=$f timeout -k 10 300 python bench.py --steps 20 --warmup 5 >> gpurun_out/ab32.jsonl 2>gpurun_out/ab32.err || exit 1
  tail -1 gpurun_out/ab32.jsonl | cut -c90-200
done
for f in 0 1; do
  PDA_WGRAD_STREAM=0 PDA_BN_BWD_SUMS=$f timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof32_$f -o prof --output-format csv -- python bench.py --steps 5 --warmup 2 > gpurun_out/prof32_$f.log 2>&1 || exit 1
done
echo ok
