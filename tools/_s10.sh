set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/s10; mkdir -p $out
PDA_FSDP_FORCE_COMM=1 PDA_TRACK_COMM=1 timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $out/ll -o run -- python -u -m pytorchdistributed_amd.bench.llama_fsdp --steps 2 --warmup 1 > $out/ll.log 2>&1 || exit 1
f=$(find $out/ll -name "*kernel_trace.csv" | head -1)
python tools/step_kernels.py $f --marker adam_kernel --top 40 --out $out/llama_forced_step.md --title "llama3-8b fsdp forced comm" > /dev/null
head -30 $out/llama_forced_step.md | cut -c1-220
rm -f $f
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $out/g2 -o run -- python -u -m pytorchdistributed_amd.bench.gpt2_ddp --steps 3 --warmup 2 > $out/g2.log 2>&1 || exit 1
f=$(find $out/g2 -name "*kernel_trace.csv" | head -1)
python tools/step_kernels.py $f --marker adam_kernel --top 40 --out $out/gpt2_step.md --title "gpt2-medium ddp" > /dev/null
head -30 $out/gpt2_step.md | cut -c1-220
rm -f $f
