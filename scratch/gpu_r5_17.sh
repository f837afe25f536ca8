#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  timeout -s KILL "$t" "$@" > gpurun_out/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -2 gpurun_out/$name.log | cut -c1-200
  if [ $rc -ne 0 ]; then echo "stopping after $name"; exit $rc; fi
}
step attn_plain 120 python tools/bench_attn.py --iters 10 --no-torch
step pmc_a 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/pmc_attn_a -o p -- python tools/bench_attn.py --iters 3 --no-torch
step pmc_b 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_INSTS_SALU SQ_BUSY_CYCLES --kernel-trace --output-format csv -d gpurun_out/pmc_attn_b -o p -- python tools/bench_attn.py --iters 3 --no-torch
