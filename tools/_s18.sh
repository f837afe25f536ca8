set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/s18; mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_models_gpu.py -x -q --timeout 120 --timeout-method thread -k "fsdp" > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
run() { echo "$1 $(tail -1 $out/ll.log | cut -c1-90) $(tail -1 $out/ll.log | grep -o '"comm.*"config"' | cut -c1-300)"; }
PDA_FSDP_FORCE_COMM=1 PDA_TRACK_COMM=1 timeout -k 10 400 python -u -m pytorchdistributed_amd.bench.llama_fsdp --steps 4 --warmup 2 > $out/ll.log 2>&1 || exit 1; run pool
PDA_FSDP_POOL=0 PYTORCH_HIP_ALLOC_CONF=max_split_size_mb:512 PDA_FSDP_FORCE_COMM=1 PDA_TRACK_COMM=1 timeout -k 10 400 python -u -m pytorchdistributed_amd.bench.llama_fsdp --steps 4 --warmup 2 > $out/ll.log 2>&1 || exit 1; run "nopool max_split512"
PDA_FSDP_FORCE_COMM=1 PDA_TRACK_COMM=1 timeout -k 10 400 python -u -m pytorchdistributed_amd.bench.llama_fsdp --steps 8 --warmup 2 > $out/ll.log 2>&1 || exit 1; run "pool 8 steps"
