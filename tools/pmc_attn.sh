#!/bin/bash
# PMC passes (counters only, one rocprofv3 run per group) over tools/bench_attn.py --iters 3 --no-torch:
# MFMA busy, wait / active shares, LDS traffic and bank conflicts of the flash-attention kernels.
#   bash tools/pmc_attn.sh OUTDIR
set -e
out=$1
mkdir -p "$out"
export TMPDIR=/tmp
p1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
p2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE"
i=0
for p in "$p1" "$p2"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $p --output-format csv -d "$out/p$i" -o run -- python3 tools/bench_attn.py --iters 3 --no-torch
done
