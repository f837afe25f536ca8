set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/s22; mkdir -p $out
PDA_WGRAD_STREAM=0 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $out/p -o run -- python -u -m pytorchdistributed_amd.bench.resnet_ddp --steps 3 --warmup 3 > $out/p.log 2>&1 || exit 1
f=$(find $out/p -name "*kernel_trace.csv" | head -1)
python tools/step_kernels.py $f --top 70 --out $out/step.md --title "round-5 tree, single stream" > /dev/null || exit 1
gzip -c $f > $out/resnet_trace.csv.gz; rm -f $f
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $out/q -o run -- python -u -m pytorchdistributed_amd.bench.resnet_ddp --steps 3 --warmup 3 > $out/q.log 2>&1 || exit 1
f=$(find $out/q -name "*kernel_trace.csv" | head -1)
python tools/busy_timeline.py $f sgd_kernel 2 $out/busy.md > /dev/null && cat $out/busy.md
python tools/concurrency.py $f conv3x3_wg_kernel gemm_wide_kernel "gemm_pp_kernel<false, false" bn_bwd_apply
gzip -c $f > $out/resnet_trace_ms.csv.gz; rm -f $f
