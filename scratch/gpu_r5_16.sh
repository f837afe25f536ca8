#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
(cd gpurun_ab/base && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_gpt2_base -o prof --output-format csv -- python -m pytorchdistributed_amd.bench.gpt2_ddp --steps 4 --warmup 2 > $R/gpurun_out/pg_base.log 2>&1) || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_gpt2_new -o prof --output-format csv -- python -m pytorchdistributed_amd.bench.gpt2_ddp --steps 4 --warmup 2 > $R/gpurun_out/pg_new.log 2>&1 || exit 1
echo done
