set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/s44; mkdir -p $out
i=0
for p in "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  PDA_WGRAD_STREAM=0 timeout -s KILL 240 rocprofv3 --pmc $p --kernel-trace --output-format csv -d $out/p$i -o run -- python3 -u -m pytorchdistributed_amd.bench.resnet_ddp --steps 2 --warmup 2 > $out/p$i.log 2>&1 || { tail -5 $out/p$i.log; exit 1; }
done
python3 tools/pmc_table.py $out/p1 $out/p2 $out/p3 40 $out/resnet_pmc.md > /dev/null || exit 1
head -30 $out/resnet_pmc.md | cut -c1-200
find $out -name "*.csv" -size +20M -delete
