set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/s26; mkdir -p $out
for r in 1 2; do
for b in 640 768 704 576; do
  PDA_BENCH_BATCH=$b timeout -k 10 300 python -u bench.py --steps 15 --warmup 4 > $out/rn_$b.log 2>&1 || exit 1
  echo "batch=$b $(tail -1 $out/rn_$b.log | cut -c100-190)"
done
done
