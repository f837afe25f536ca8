#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
for b in 640 768 1024; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --batch $b > gpurun_out/bs$b.log 2>&1 || exit 1
  echo "bs $b: $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' gpurun_out/bs$b.log | paste -s)"
done
