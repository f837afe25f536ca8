#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/pmc38
export TMPDIR=/tmp
for shape in "56 64 256 1 1" "56 64 64 3 1"; do
  tag=$(echo $shape | tr ' ' '_')
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VALU --kernel-trace --output-format csv -d gpurun_out/pmc38/$tag -o p -- python tools/conv_one.py fwd $shape 5 > gpurun_out/pmc38/$tag.log 2>&1 || exit 1
done
echo ok
