#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > gpurun_out/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -3 gpurun_out/$name.log | cut -c1-300
  if [ $rc -ne 0 ]; then echo "stopping after $name"; exit $rc; fi
}
step pytest_gpu 600 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread
step bench 300 python bench.py --steps 20 --warmup 5
step bench_es0 300 env PDA_BN_EPILOGUE_STATS=0 python bench.py --steps 20 --warmup 5
step bench_b 300 python bench.py --steps 20 --warmup 5
step prof_resnet 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_resnet_r2k -o prof --output-format csv -- python bench.py --steps 5 --warmup 2
