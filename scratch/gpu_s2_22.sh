#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/s2_22; mkdir -p $D
export TMPDIR=/tmp
for rnd in 1 2; do
  for cus in 192 160 224 256; do
    PDA_WGRAD_CUS=$cus timeout -k 10 300 python bench.py > $D/cus${cus}_r$rnd.log 2>&1; rc=$?
    echo "== cus $cus round $rnd rc=$rc $(grep -h '"metric"' $D/cus${cus}_r$rnd.log | cut -c90-125)"
    if [ $rc -ne 0 ]; then exit $rc; fi
  done
done
