#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > gpurun_out/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -1 gpurun_out/$name.log | cut -c1-200
  if [ $rc -ne 0 ]; then echo "stopping after $name"; exit $rc; fi
}
PDA_BN_STAT_ROWS=32 step bench_r32 300 python bench.py --steps 20 --warmup 5
PDA_BN_STAT_ROWS=128 step bench_r128 300 python bench.py --steps 20 --warmup 5
PDA_BN_STAT_ROWS=512 step bench_r512 300 python bench.py --steps 20 --warmup 5
PDA_BN_STAT_ROWS=128 step prof_resnet 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_resnet_r2f -o prof --output-format csv -- python bench.py --steps 5 --warmup 2
