#!/bin/bash
# Interleaved A/B of two package trees (one GPU box, same command): each arm runs the module command
# from its own directory, so `python -m pytorchdistributed_amd...` imports that tree's package.
#   bash tools/ab_tree.sh OUT.jsonl ROUNDS DIR_A DIR_B [...] -- python -u -m pytorchdistributed_amd.bench.resnet_ddp --steps 20
# DIR "." is the working tree; gpurun_ab/<name> comes from tools/ab_build.sh.  A failing run stops it.
set -e
out=$1; rounds=$2; shift 2
arms=()
while [ "$1" != "--" ]; do arms+=("$1"); shift; done
shift
mkdir -p "$(dirname "$out")"
root=$(pwd)
for r in $(seq 1 "$rounds"); do
  for a in "${arms[@]}"; do
    line=$(cd "$a" && timeout -k 10 300 "$@" 2>"$root/$out.err.log" | tail -1)
    echo "{\"arm\": \"$a\", \"round\": $r, \"result\": $line}" >> "$out"
    echo "$a round $r: $line" | cut -c1-200
  done
done
