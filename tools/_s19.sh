set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/s19; mkdir -p $out
run() { echo "$1 $(tail -1 $out/ll.log | cut -c1-90) $(tail -1 $out/ll.log | grep -o '"comm.*"config"' | cut -c1-300)"; }
PDA_FSDP_POOL=0 PYTORCH_ALLOC_CONF=expandable_segments:True PDA_FSDP_FORCE_COMM=1 PDA_TRACK_COMM=1 timeout -k 10 400 python -u -m pytorchdistributed_amd.bench.llama_fsdp --steps 4 --warmup 2 > $out/ll.log 2>&1 || { tail -3 $out/ll.log; exit 1; }; run "nopool expandable"
PYTORCH_ALLOC_CONF=expandable_segments:True PDA_FSDP_FORCE_COMM=1 PDA_TRACK_COMM=1 timeout -k 10 400 python -u -m pytorchdistributed_amd.bench.llama_fsdp --steps 4 --warmup 2 > $out/ll.log 2>&1 || { tail -3 $out/ll.log; exit 1; }; run "pool expandable"
PYTORCH_ALLOC_CONF=expandable_segments:True timeout -k 10 400 python -u -m pytorchdistributed_amd.bench.llama_fsdp --steps 4 --warmup 2 > $out/ll.log 2>&1 || { tail -3 $out/ll.log; exit 1; }; run "plain expandable"
