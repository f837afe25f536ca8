set -o pipefail
out=gpurun_out/s24; mkdir -p $out
export TMPDIR=/tmp
p1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
p2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE"
p3="TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"
i=0
for p in "$p1" "$p2" "$p3"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $p --kernel-trace --output-format csv -d $out/p$i -o run -- python3 tools/conv_one.py fwd 56 64 64 3 1 10 > $out/p$i.log 2>&1 || exit 1
  f=$(find $out/p$i -name "*counter_collection.csv" | head -1)
  python3 tools/pmc_summary.py $f res64 > $out/p$i.txt || exit 1
  cat $out/p$i.txt | head -30
  k=$(find $out/p$i -name "*kernel_trace.csv" | head -1)
  python3 - "$k" <<'PY'
import csv,sys
r=[x for x in csv.DictReader(open(sys.argv[1])) if 'res64' in x['Kernel_Name']]
d=[(int(x['End_Timestamp'])-int(x['Start_Timestamp']))/1e3 for x in r]
print('res64 kernel us', [round(v,1) for v in d][-4:])
PY
  rm -f $f $k
done
