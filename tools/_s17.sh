set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/s17; mkdir -p $out
PDA_FSDP_FORCE_COMM=1 timeout -k 10 400 python -u -m pytorchdistributed_amd.bench.llama_fsdp --steps 3 --warmup 2 > $out/ll_forced_notrack.log 2>&1 || exit 1
echo "forced no-track $(tail -1 $out/ll_forced_notrack.log | cut -c1-700)"
PDA_FSDP_FORCE_COMM=1 timeout -k 10 500 rocprofv3 --hip-trace --output-format csv -d $out/ll -o run -- python -u -m pytorchdistributed_amd.bench.llama_fsdp --steps 3 --warmup 2 > $out/llp.log 2>&1 || exit 1
f=$(find $out/ll -name "*hip_api_trace.csv" | head -1)
python - "$f" <<'PY'
import csv,sys,collections
rows=list(csv.DictReader(open(sys.argv[1])))
t0=min(int(r['Start_Timestamp']) for r in rows); t1=max(int(r['End_Timestamp']) for r in rows)
print(len(rows),"hip calls over",(t1-t0)/1e9,"s")
agg=collections.defaultdict(lambda:[0,0.0,0.0])
for r in rows:
    d=(int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e6
    a=agg[r['Function']]; a[0]+=1; a[1]+=d; a[2]=max(a[2],d)
for k,v in sorted(agg.items(), key=lambda kv:-kv[1][1])[:25]: print(f"{v[1]:10.1f} ms {v[0]:7d} calls max {v[2]:8.1f} ms  {k}")
PY
rm -f $f
