set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/s13; mkdir -p $out
timeout -k 10 600 python -u tools/bench_conv.py --batch 640 --iters 10 > $out/conv_table.jsonl 2> $out/conv_table.err || { tail -5 $out/conv_table.err; exit 1; }
tail -1 $out/conv_table.jsonl
timeout -k 10 400 bash tools/pmc_attn.sh $out/pmc > $out/pmc.log 2>&1 || { tail -5 $out/pmc.log; exit 1; }
echo pmc done
for r in 1 2; do
  PDA_FSDP_FORCE_COMM=1 PDA_TRACK_COMM=1 timeout -k 10 400 python -u -m pytorchdistributed_amd.bench.llama_fsdp --steps 6 --warmup 2 > $out/ll_forced_$r.log 2>&1 || exit 1
  echo "forced $(tail -1 $out/ll_forced_$r.log | cut -c1-900)"
done
timeout -k 10 400 python -u -m pytorchdistributed_amd.bench.llama_fsdp --steps 6 --warmup 2 > $out/ll_plain.log 2>&1 || exit 1
echo "plain $(tail -1 $out/ll_plain.log | cut -c1-300)"
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $out/ll -o run -- python -u -m pytorchdistributed_amd.bench.llama_fsdp --steps 2 --warmup 1 > $out/llp.log 2>&1 || exit 1
f=$(find $out/ll -name "*kernel_trace.csv" | head -1)
python tools/step_kernels.py $f --marker ce_fwd_kernel --top 40 --out $out/llama_step.md --title "llama3-8b fsdp (one rank, no forced comm)" > /dev/null
head -26 $out/llama_step.md | cut -c1-200
rm -f $f
