#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/s2_23; mkdir -p $D
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > $D/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -2 $D/$name.log | cut -c1-250
  if [ $rc -ne 0 ]; then echo "stopping after $name"; exit $rc; fi
}
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench1 300 python bench.py
step bench2 300 python bench.py
PDA_WGRAD_STREAM=0 step prof_single 400 rocprofv3 --kernel-trace --stats -d $D/prof_single -o run -- python bench.py --steps 10 --warmup 5
step prof_two 400 rocprofv3 --kernel-trace --stats -d $D/prof_two -o run -- python bench.py --steps 10 --warmup 5
