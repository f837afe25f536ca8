set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/s15; mkdir -p $out
PDA_FSDP_FORCE_COMM=1 PDA_TRACK_COMM=1 timeout -k 10 400 python -u -m pytorchdistributed_amd.bench.llama_fsdp --steps 4 --warmup 2 > $out/ll_forced.log 2>&1 || exit 1
echo "forced $(tail -1 $out/ll_forced.log | cut -c1-1200)"
PYTORCH_HIP_ALLOC_CONF=expandable_segments:True PDA_FSDP_FORCE_COMM=1 PDA_TRACK_COMM=1 timeout -k 10 400 python -u -m pytorchdistributed_amd.bench.llama_fsdp --steps 4 --warmup 2 > $out/ll_forced_exp.log 2>&1 || exit 1
echo "forced+expandable $(tail -1 $out/ll_forced_exp.log | cut -c1-1200)"
timeout -k 10 400 python -u -m pytorchdistributed_amd.bench.llama_fsdp --steps 4 --warmup 2 > $out/ll_plain.log 2>&1 || exit 1
echo "plain $(tail -1 $out/ll_plain.log | cut -c1-1200)"
