#!/bin/bash
# same-box A/B: HEAD build (scratch/base) vs working tree, fused BN-backward sums on/off
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for rep in 1 2; do
  timeout -k 10 300 python ab_base/bench.py --steps 20 --warmup 5 2>/dev/null | cut -c90-175 | sed 's/^/base    /' || exit 1
  PDA_BN_BWD_SUMS=0 timeout -k 10 300 python bench.py --steps 20 --warmup 5 2>/dev/null | cut -c90-175 | sed 's/^/unfused /' || exit 1
  PDA_BN_BWD_SUMS=1 timeout -k 10 300 python bench.py --steps 20 --warmup 5 2>/dev/null | cut -c90-175 | sed 's/^/fused   /' || exit 1
done
