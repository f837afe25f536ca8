set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/s43; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py tests/test_attention_gpu.py -x -q --timeout 120 --timeout-method thread -k "wgrad_db or linear or gpt2 or llama or rebase" > $out/t.log 2>&1 || { tail -30 $out/t.log; exit 1; }
tail -1 $out/t.log
for r in 1 2; do
  for m in 1 0; do
    PDA_ROWSUM_FUSED=$m timeout -k 10 300 python -u -m pytorchdistributed_amd.bench.gpt2_ddp --steps 10 --warmup 3 > $out/g2_$m.log 2>&1 || exit 1
    echo "fused=$m $(tail -1 $out/g2_$m.log | cut -c1-120)"
  done
done
