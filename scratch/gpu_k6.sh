#!/bin/bash
# GEMM diagnostics: native vs hipBLASLt TFLOP/s, then SQ counters of the native wide kernel on 4096^3 / 8192^3
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/k6
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > gpurun_out/k6/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"; grep -v amdgpu gpurun_out/k6/$name.log | tail -12 | cut -c1-300
  if [ $rc -ne 0 ]; then echo "stopping after $name"; exit $rc; fi
}
step blas 300 python tools/bench_blas.py
step conv640 400 python tools/bench_conv.py --batch 640 --iters 10
step copies 300 python tools/find_copies.py --model gpt2 --steps 2 --batch 8
step pmc4k 120 timeout -s KILL 100 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/k6/pmc4k -o p -- python tools/gemm_one.py 4096 4096 4096 10
step pmc8k 120 timeout -s KILL 100 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/k6/pmc8k -o p -- python tools/gemm_one.py 8192 8192 8192 5
step pmc_c1 120 timeout -s KILL 100 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/k6/pmc_c1 -o p -- python tools/conv_one.py fwd 56 64 256 1 1 10
step pmc_c2 120 timeout -s KILL 100 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/k6/pmc_c2 -o p -- python tools/conv_one.py fwd 14 256 256 3 1 10
step pmc_c3 120 timeout -s KILL 100 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/k6/pmc_c3 -o p -- python tools/conv_one.py fwd 56 64 256 1 1 10
