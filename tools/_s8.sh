set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/s8; mkdir -p $out
for i in 1 2; do
  timeout -k 10 300 python -u bench.py > $out/bench_v2_$i.log 2>&1 && tail -1 $out/bench_v2_$i.log | cut -c1-160
  PDA_CONV_WG3V2=0 timeout -k 10 300 python -u bench.py > $out/bench_v1_$i.log 2>&1 && tail -1 $out/bench_v1_$i.log | cut -c1-160
done
timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --output-format csv -d $out/fills -o run -- python -u -m pytorchdistributed_amd.bench.gpt2_ddp --steps 2 --warmup 1 > $out/fills.log 2>&1 || exit 1
python tools/fill_sources.py $out/fills > $out/fill_sources.txt; cat $out/fill_sources.txt
find $out/fills -name "*.csv" -size +1M -delete
