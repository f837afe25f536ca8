set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/s7; mkdir -p $out
for v in 0 1; do
  PDA_PP_SYNC_P2P=$v PDA_PP_FORCE_COMM=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $out/pp$v -o run -- python -u -m pytorchdistributed_amd.bench.gpt2xl_pp --schedule interleaved --chunks 2 --layers 8 --micro 4 --micro-batch 4 --seq 1024 --steps 3 --warmup 2 > $out/pp$v.log 2>&1 || exit 1
  f=$(find $out/pp$v -name "*kernel_trace.csv" | head -1)
  python tools/overlap_report.py $f --skip-first 16 --json > $out/overlap$v.json || exit 1
  tail -1 $out/pp$v.log | cut -c1-300
  cat $out/overlap$v.json
  rm -f $f
done
