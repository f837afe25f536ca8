#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
out=gpurun_out/r2s4_batch_sweep.jsonl
: > $out
for rep in 1 2; do
  for b in 576 640 704 768; do
    timeout -k 10 150 python bench.py --steps 20 --warmup 5 --batch $b > gpurun_out/bs_$b.log 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then echo "rc=$rc at b=$b"; tail -5 gpurun_out/bs_$b.log; exit $rc; fi
    grep '^{' gpurun_out/bs_$b.log >> $out
    python -c "import json; d=json.loads(open('$out').readlines()[-1]); print(d['config']['per_gpu_batch'], d['value'], d['ms_per_step'])"
  done
done
PDA_WGRAD_STREAM=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_resnet_v26_single -o prof --output-format csv -- python bench.py --steps 8 --warmup 3 > gpurun_out/prof_single.log 2>&1
echo "single rc=$?"
