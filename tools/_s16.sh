set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/s16; mkdir -p $out
PDA_FSDP_FORCE_COMM=1 PDA_TRACK_COMM=1 timeout -k 10 500 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $out/ll -o run -- python -u -m pytorchdistributed_amd.bench.llama_fsdp --steps 3 --warmup 2 > $out/llp.log 2>&1 || exit 1
grep tokens $out/llp.log | cut -c1-400
f=$(find $out/ll -name "*kernel_trace.csv" | head -1)
python tools/step_kernels.py $f --marker ce_fwd_kernel --top 30 --out $out/llama_forced_step.md --title "llama3-8b fsdp forced comm" > /dev/null
head -36 $out/llama_forced_step.md | cut -c1-200
m=$(find $out/ll -name "*memory_copy_trace.csv" | head -1)
[ -n "$m" ] && python - "$m" <<'PY'
import csv,sys,collections
rows=list(csv.DictReader(open(sys.argv[1])))
print(len(rows),"memcopies", list(rows[0].keys())[:20] if rows else "")
agg=collections.defaultdict(lambda:[0,0.0,0])
for r in rows:
    k=r.get('Direction') or r.get('Kind') or '?'
    d=(int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e6
    agg[k][0]+=1; agg[k][1]+=d; agg[k][2]+=int(r.get('Bytes',0) or 0)
for k,v in agg.items(): print(k, v[0], f"{v[1]:.1f} ms", f"{v[2]/2**30:.1f} GiB")
PY
rm -f $f
