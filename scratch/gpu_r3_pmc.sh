#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
export PDA_WGRAD_STREAM=0
timeout -s KILL 150 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/pmc_r3f_sq -o p -- python bench.py --steps 2 --warmup 1 > gpurun_out/pmc_sq.log 2>&1 || exit $?
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_r3f_fetch -o p -- python bench.py --steps 2 --warmup 1 > gpurun_out/pmc_fetch.log 2>&1 || exit $?
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_r3f_write -o p -- python bench.py --steps 2 --warmup 1 > gpurun_out/pmc_write.log 2>&1 || exit $?
echo pmc done
