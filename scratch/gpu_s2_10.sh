#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
D=gpurun_out/s2_10; mkdir -p $D
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > $D/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -2 $D/$name.log | cut -c1-300
  if [ $rc -ne 0 ]; then echo "stopping after $name"; exit $rc; fi
}
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread
step bench_both 300 python bench.py
PDA_CONV_STEM_FWD=0 step bench_wg 300 python bench.py
PDA_CONV_STEM_FWD=0 PDA_CONV_STEM_WG=0 step bench_none 300 python bench.py
step bench_both2 300 python bench.py
PDA_CONV_STEM_FWD=0 step bench_wg2 300 python bench.py
PDA_CONV_STEM_FWD=0 PDA_CONV_STEM_WG=0 step bench_none2 300 python bench.py
