set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/s3
for v in 1 0; do
  PDA_BN_BWD_EPILOGUE=$v PDA_WGRAD_STREAM=0 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/s3/p$v -o run -- python -u -m pytorchdistributed_amd.bench.resnet_ddp --steps 3 --warmup 3 > gpurun_out/s3/p$v.log 2>&1 || exit 1
  f=$(find gpurun_out/s3/p$v -name "*kernel_trace.csv" | head -1)
  python tools/step_kernels.py $f --top 60 --out gpurun_out/s3/step$v.md --title "bwd_epilogue=$v" > /dev/null || exit 1
  rm -f $f
done
