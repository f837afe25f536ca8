set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/s11; mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_attention_gpu.py -x -q --timeout 120 --timeout-method thread > $out/tests.log 2>&1 || { tail -40 $out/tests.log; exit 1; }
tail -3 $out/tests.log
for m in 0 1 0 1; do
  PDA_ATTN_BWD_FUSED=$m timeout -k 10 300 python -u -m pytorchdistributed_amd.bench.gpt2_ddp --steps 10 --warmup 3 > $out/g2_$m.log 2>&1 || exit 1
  echo "fused=$m $(tail -1 $out/g2_$m.log | cut -c1-200)"
done
PDA_ATTN_BWD_FUSED=1 timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $out/g2 -o run -- python -u -m pytorchdistributed_amd.bench.gpt2_ddp --steps 3 --warmup 2 > $out/g2p.log 2>&1 || exit 1
f=$(find $out/g2 -name "*kernel_trace.csv" | head -1)
python tools/step_kernels.py $f --marker adam_kernel --top 40 --out $out/gpt2_step.md --title "gpt2-medium ddp fused attn bwd" > /dev/null
head -24 $out/gpt2_step.md | cut -c1-200
rm -f $f
for m in 0 2 0 2; do
  PDA_ATTN_BWD_FUSED=$m timeout -k 10 400 python -u -m pytorchdistributed_amd.bench.llama_fsdp --steps 6 --warmup 2 > $out/ll_$m.log 2>&1 || exit 1
  echo "fused=$m $(tail -1 $out/ll_$m.log | cut -c1-200)"
done
