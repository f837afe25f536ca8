#!/bin/bash
# GPT-2-medium DDP (32x1024 tokens/GPU) kernel profile + occupancy on the current tree
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
true

export PYTHONPATH="$GRAFT_REPO_ROOT"; cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof7" -o run -- python3 -m pytorchdistributed_amd.bench.gpt2_ddp --steps 4 --warmup 2 > "$GRAFT_REPO_ROOT/gpurun_out/prof7.log" 2>&1 || exit 1
cd "$GRAFT_REPO_ROOT"
kt=$(find gpurun_out/prof7 -name '*kernel_trace.csv' | head -1)
ks=$(find gpurun_out/prof7 -name '*kernel_stats.csv' | head -1)
python tools/busy_timeline.py "$kt" adam_kernel 2 gpurun_out/r7_gpt2_busy.md || exit 1
python tools/prof_summary.py "$ks" 6 45 gpurun_out/r7_gpt2_kernels.md > /dev/null || exit 1
rm -f gpurun_out/prof7/*kernel_trace.csv
echo ok
