set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/s30; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_models_gpu.py tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "resnet or bottleneck or conv or bn or determin or stats" > $out/t.log 2>&1 || { tail -30 $out/t.log; exit 1; }
tail -1 $out/t.log
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $out/rn_$r.log 2>&1 || exit 1
  echo "$(tail -1 $out/rn_$r.log | cut -c100-190)"
done
PDA_WGRAD_STREAM=0 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $out/rn -o run -- python -u -m pytorchdistributed_amd.bench.resnet_ddp --steps 3 --warmup 3 > $out/rnp.log 2>&1 || exit 1
f=$(find $out/rn -name "*kernel_trace.csv" | head -1)
python tools/step_kernels.py $f --top 70 --out $out/resnet_step.md --title "lean res64 bst" > /dev/null || exit 1
head -3 $out/resnet_step.md | cut -c1-200; grep res64 $out/resnet_step.md | cut -c1-120
rm -f $f
