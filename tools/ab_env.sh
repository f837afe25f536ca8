#!/bin/bash
# Interleaved A/B of environment settings on one benchmark command (one GPU box, same process tree):
#   bash tools/ab_env.sh OUT.jsonl ROUNDS "ENV_A" "ENV_B" [...] -- python -u bench.py --steps 20
# Each arm's JSON line (the benchmark's last stdout line) is appended to OUT.jsonl with "arm" added.
# Every run has its own time limit; a failing run stops the whole A/B (no retries).
set -e
out=$1; rounds=$2; shift 2
arms=()
while [ "$1" != "--" ]; do arms+=("$1"); shift; done
shift
mkdir -p "$(dirname "$out")"
for r in $(seq 1 "$rounds"); do
  for a in "${arms[@]}"; do
    line=$(env $a timeout -k 10 300 "$@" 2>"$out.err.log" | tail -1)
    echo "{\"arm\": \"$a\", \"round\": $r, \"result\": $line}" >> "$out"
    echo "$a round $r: $line" | cut -c1-300
  done
done
