#!/bin/bash
# A/B: side-stream queue priority (PDA_WGRAD_PRIO) x main-stream priority (PDA_MAIN_PRIO), same box
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/prio_ab.jsonl; : > $out
for rep in 1 2; do
for cfg in "normal none" "low none" "normal high" "low high"; do
  set -- $cfg
  r=$(PDA_WGRAD_PRIO=$1 PDA_MAIN_PRIO=$2 timeout -k 10 150 python bench.py --steps 20 --warmup 5) || exit 1
  echo "{\"wgrad_prio\": \"$1\", \"main_prio\": \"$2\", \"rep\": $rep, \"bench\": $r}" | tee -a $out
done
done
