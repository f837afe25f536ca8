#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python tools/bench_conv.py --torch > gpurun_out/bench_conv.log 2>&1
rc=$?; echo "bench_conv rc=$rc"; tail -3 gpurun_out/bench_conv.log
if [ $rc -ne 0 ]; then exit $rc; fi
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_gpt2 -o prof --output-format csv -- python -m pytorchdistributed_amd.bench.gpt2_ddp --steps 4 --warmup 2 > gpurun_out/prof_gpt2.log 2>&1
echo "prof rc=$?"
