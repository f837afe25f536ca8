#!/bin/bash
# per-GPU batch sweep on the current kernels
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for b in 512 576 640 704 768; do
  timeout -k 10 300 python bench.py --batch $b --steps 20 --warmup 5 2>/dev/null | python -c "import json,sys; r=json.loads(sys.stdin.read()); print(json.dumps({'per_gpu_batch': $b, 'value': r['value'], 'ms_per_step': r['ms_per_step'], 'final_loss': r.get('final_loss')}))" | tee -a gpurun_out/sweep44.jsonl || exit 1
done
echo ok
