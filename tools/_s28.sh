set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/s28; mkdir -p $out
timeout -k 10 500 rocprofv3 --kernel-trace --output-format csv -d $out/ll -o run -- python -u -m pytorchdistributed_amd.bench.llama_fsdp --steps 3 --warmup 2 > $out/llp.log 2>&1 || exit 1
f=$(find $out/ll -name "*kernel_trace.csv" | head -1)
python tools/step_kernels.py $f --marker ce_fwd_kernel --step -2 --top 40 --out $out/llama_step.md --title "llama3-8b fsdp (one rank, steady step 4 of 5)" > /dev/null
head -8 $out/llama_step.md | cut -c1-200
rm -f $f
PDA_WGRAD_STREAM=0 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $out/rn -o run -- python -u -m pytorchdistributed_amd.bench.resnet_ddp --steps 3 --warmup 3 > $out/rn.log 2>&1 || exit 1
f=$(find $out/rn -name "*kernel_trace.csv" | head -1)
python tools/step_kernels.py $f --top 70 --out $out/resnet_step.md --title "round-5 final tree, single stream" > /dev/null || exit 1
head -4 $out/resnet_step.md | cut -c1-200
rm -f $f
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $out/g2 -o run -- python -u -m pytorchdistributed_amd.bench.gpt2_ddp --steps 3 --warmup 2 > $out/g2.log 2>&1 || exit 1
f=$(find $out/g2 -name "*kernel_trace.csv" | head -1)
python tools/step_kernels.py $f --marker adam_kernel --top 40 --out $out/gpt2_step.md --title "gpt2-medium ddp, round-5 final tree" > /dev/null
head -4 $out/gpt2_step.md | cut -c1-200
rm -f $f
