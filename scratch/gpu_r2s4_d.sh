#!/bin/bash
# A/B: wgrad tile shape x CU budget (env sets), ResNet-50 bs 640, interleaved
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
out=gpurun_out/r2s4_ab.jsonl
: > $out
i=0
for rep in 1 2; do
  IFS=";" read -ra CL <<< "${CFGS:-X=1}"
  for cfg in "${CL[@]}"; do
    i=$((i+1))
    env $cfg timeout -k 10 150 ${BENCH:-python bench.py --steps 20 --warmup 5} > gpurun_out/ab_$i.log 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then echo "rc=$rc at $cfg"; tail -5 gpurun_out/ab_$i.log; exit $rc; fi
    echo "{\"env\": \"$cfg\", \"rep\": $rep, \"bench\": $(grep '^{' gpurun_out/ab_$i.log)}" >> $out
    python -c "import json; d=json.loads(open('$out').readlines()[-1]); print(d['env'], d['bench']['value'], d['bench']['ms_per_step'])"
  done
done
