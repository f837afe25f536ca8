set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/s46; mkdir -p $out
for r in 1 2 3; do
  for m in 1 0; do
    PDA_ROWSUM_FUSED=$m timeout -k 10 300 python -u -m pytorchdistributed_amd.bench.gpt2_ddp --steps 12 --warmup 3 > $out/g2_$m.log 2>&1 || exit 1
    echo "fused=$m $(tail -1 $out/g2_$m.log | cut -c60-100)"
  done
done
