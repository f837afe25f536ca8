#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > gpurun_out/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"; grep -o '"shape": "[a-z0-9-]*"\|"bwd_ms": [0-9.]*\|"bwd_tflops": [0-9.]*\|[0-9]* passed.*' gpurun_out/$name.log | paste -s
  if [ $rc -ne 0 ]; then echo "stopping after $name"; exit $rc; fi
}
PDA_ATTN_BWD_DB=3 step attn_tests_db 300 python -u -m pytest tests/test_attention_gpu.py tests/test_ulysses_gpu.py -q -x -p no:cacheprovider --timeout 200 --timeout-method thread
for d in 0 1 2 3 0; do PDA_ATTN_BWD_DB=$d step bwd_db$d 120 python tools/bench_attn.py --iters 20 --no-torch; done
