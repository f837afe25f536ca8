set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/s9; mkdir -p $out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/lm -o run -- python -u tools/lmhead_probe.py > $out/lm.log 2>&1 || exit 1
f=$(find $out/lm -name "*kernel_stats.csv" | head -1); head -8 $f | cut -c1-200
find $out/lm -name "*kernel_trace.csv" -delete
PDA_FSDP_FORCE_COMM=1 PDA_TRACK_COMM=1 timeout -k 10 400 python -u -m pytorchdistributed_amd.bench.llama_fsdp --steps 3 --warmup 2 > $out/llama_forced.log 2>&1; tail -1 $out/llama_forced.log | cut -c1-600
timeout -k 10 300 python -u -m pytorchdistributed_amd.bench.gpt2_ddp --steps 8 --warmup 3 > $out/gpt2.log 2>&1; tail -1 $out/gpt2.log | cut -c1-300
