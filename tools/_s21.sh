set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/s21; mkdir -p $out
timeout -k 10 300 python -u tools/bench_gpt2_gemm.py --kinds fwd,dgrad,wgrad > $out/gemm.jsonl 2> $out/gemm.err || { tail -5 $out/gemm.err; exit 1; }
cut -c1-220 $out/gemm.jsonl
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $out/g2 -o run -- python -u -m pytorchdistributed_amd.bench.gpt2_ddp --steps 3 --warmup 2 > $out/g2.log 2>&1 || exit 1
f=$(find $out/g2 -name "*kernel_trace.csv" | head -1)
python tools/concurrency.py $f "gemm_pp_kernel<true, false" "gemm_pp_kernel<true, true" "gemm_pp_kernel<false, false" "attn_bwd_dkdv2" "attn_fwd3"
python tools/busy_timeline.py $f adam_kernel 2 $out/busy.md > /dev/null && head -30 $out/busy.md
gzip -c $f > $out/gpt2_trace.csv.gz; rm -f $f
