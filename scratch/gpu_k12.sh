#!/bin/bash
# conv per-shape table at batch 640 with roofline columns; counters of the wide GEMM / conv kernels
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/k12
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > gpurun_out/k12/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"; grep -v amdgpu gpurun_out/k12/$name.log | grep -v "^W2026\|^E2026" | tail -5 | cut -c1-300
  if [ $rc -ne 0 ]; then echo "stopping after $name"; exit $rc; fi
}
step conv640 500 python tools/bench_conv.py --batch 640 --iters 10 --blas
PMC="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS GRBM_GUI_ACTIVE"
step pmc4k 120 timeout -s KILL 100 rocprofv3 --pmc $PMC --kernel-trace --output-format csv -d gpurun_out/k12/pmc4k -o p -- python tools/gemm_one.py 4096 4096 4096 10
step pmc8k 120 timeout -s KILL 100 rocprofv3 --pmc $PMC --kernel-trace --output-format csv -d gpurun_out/k12/pmc8k -o p -- python tools/gemm_one.py 8192 8192 8192 5
step pmc_c1 120 timeout -s KILL 100 rocprofv3 --pmc $PMC --kernel-trace --output-format csv -d gpurun_out/k12/pmc_c1 -o p -- python tools/conv_one.py fwd 56 64 256 1 1 10
step pmc_c1f 120 timeout -s KILL 100 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/k12/pmc_c1f -o p -- python tools/conv_one.py fwd 56 64 256 1 1 10
step pmc_c1w 120 timeout -s KILL 100 rocprofv3 --pmc WRITE_SIZE GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/k12/pmc_c1w -o p -- python tools/conv_one.py fwd 56 64 256 1 1 10
