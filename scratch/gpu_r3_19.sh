#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
( while true; do echo "tick $(date +%s)"; sleep 30; done ) &
TICK=$!
PDA_TUNABLEOP=tune PDA_TUNABLEOP_OUT=gpurun_out/tunableop_llama3.csv timeout -k 10 700 python -m pytorchdistributed_amd.bench.llama_fsdp --steps 1 --warmup 1 > gpurun_out/tune_llama.log 2>&1
rc=$?
kill $TICK
echo "tune rc=$rc"; tail -2 gpurun_out/tune_llama.log | cut -c1-300; ls -la gpurun_out/ | grep tunable
exit $rc
