#!/bin/bash
# ping-pong wide schedule: equality tests, GEMM / conv A/B vs the current schedule and hipBLASLt, bench A/B
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/k8
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > gpurun_out/k8/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"; grep -v amdgpu gpurun_out/k8/$name.log | tail -14 | cut -c1-600
  if [ $rc -ne 0 ]; then echo "stopping after $name"; exit $rc; fi
}
step pp_tests 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "pingpong or persistent or conv_fwd_dgrad_wgrad or gemm"
step variants 400 python tools/bench_wide_variants.py --rounds 3 --convs
step bench_v3 200 python bench.py --steps 20 --warmup 5
step bench_v4 200 env PDA_WIDE_VARIANT=4 python bench.py --steps 20 --warmup 5
step bench_v3b 200 python bench.py --steps 20 --warmup 5
step bench_v4b 200 env PDA_WIDE_VARIANT=4 python bench.py --steps 20 --warmup 5
step bench_c10d 200 env PDA_COMM=c10d python bench.py --steps 20 --warmup 5
