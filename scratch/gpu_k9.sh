#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/k9
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > gpurun_out/k9/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"; grep -v amdgpu gpurun_out/k9/$name.log | tail -30 | cut -c1-400
  if [ $rc -ne 0 ]; then echo "stopping after $name"; exit $rc; fi
}
step pp_tests 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "pingpong"
step variants 500 python tools/bench_wide_variants.py --rounds 3 --convs
step b_native 200 python bench.py --steps 20 --warmup 5
step b_c10d 200 env PDA_COMM=c10d python bench.py --steps 20 --warmup 5
step b_normprio 200 env PDA_COMM_PRIORITY=normal python bench.py --steps 20 --warmup 5
step b_q12 200 env PDA_HW_QUEUES=12 python bench.py --steps 20 --warmup 5
step b_nocomm 200 env PDA_DDP_FORCE_COMM=0 python bench.py --steps 20 --warmup 5
