set -o pipefail
out=gpurun_out/s5; mkdir -p $out
export TMPDIR=/tmp
p1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
p2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE"
for shape in "56 64 64 3 1" "7 512 512 3 1"; do
  tag=$(echo $shape | tr ' ' '_')
  i=0
  for p in "$p1" "$p2"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $p --output-format csv -d $out/${tag}_p$i -o run -- python3 tools/conv_one.py wgrad $shape 10 > $out/${tag}_p$i.log 2>&1 || exit 1
    f=$(find $out/${tag}_p$i -name "*counter_collection.csv" | head -1)
    python3 tools/pmc_summary.py $f conv3x3_wg > $out/${tag}_p$i.txt || exit 1
    rm -f $f
  done
done
