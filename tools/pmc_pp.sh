#!/bin/bash
# PMC passes (one rocprofv3 run per counter group, counters only, no tracing) over tools/pp_one.py.
#   bash tools/pmc_pp.sh OUTDIR VARIANT LAYOUT M N K
set -e
out=$1; v=$2; lay=$3; M=$4; N=$5; K=$6
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
p1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
p2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE"
i=0
for p in "$p1" "$p2"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $p --output-format csv -d "$out/p$i" -o run -- python3 tools/pp_one.py $v $lay $M $N $K 10
done
