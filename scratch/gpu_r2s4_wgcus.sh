#!/bin/bash
# A/B: side-stream wgrad grid sized for n CUs (PDA_WGRAD_CUS), ResNet-50 bs 640, interleaved
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
out=gpurun_out/r2s4_wgcus.jsonl
: > $out
for rep in 1 2; do
  for n in ${WG_LIST:-256 128 192 160 224}; do
    PDA_WGRAD_CUS=$n timeout -k 10 150 python bench.py --steps 20 --warmup 5 > gpurun_out/wg_$n.log 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then echo "rc=$rc at n=$n"; tail -5 gpurun_out/wg_$n.log; exit $rc; fi
    echo "{\"wgrad_cus\": $n, \"rep\": $rep, \"bench\": $(grep '^{' gpurun_out/wg_$n.log)}" >> $out
    python -c "import json,sys; d=json.loads(open('$out').readlines()[-1]); print(d['wgrad_cus'], d['bench']['value'], d['bench']['ms_per_step'])"
  done
done
