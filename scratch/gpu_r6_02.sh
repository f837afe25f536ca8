#!/bin/bash
# kernel trace of the headline step (bs 640): per-step occupancy (union busy vs span) and stats
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof6" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 6 --warmup 2 > "$GRAFT_REPO_ROOT/gpurun_out/prof6.log" 2>&1 || exit 1
cd "$GRAFT_REPO_ROOT"
kt=$(find gpurun_out/prof6 -name '*kernel_trace.csv' | head -1)
ks=$(find gpurun_out/prof6 -name '*kernel_stats.csv' | head -1)
python tools/busy_timeline.py "$kt" sgd_kernel 3 gpurun_out/r6_busy.md || exit 1
python tools/prof_summary.py "$ks" 8 40 gpurun_out/r6_kernels.md > /dev/null || exit 1
# keep the trace small enough to merge back
gzip -c "$kt" > gpurun_out/r6_kernel_trace.csv.gz
rm -rf gpurun_out/prof6/*/*kernel_trace.csv
echo ok
