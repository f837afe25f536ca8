set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/s12; mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_attention_gpu.py -x -q --timeout 120 --timeout-method thread > $out/tests.log 2>&1 || { tail -40 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for m in 0 1 17 2; do
  PDA_ATTN_BWD_FUSED=$m timeout -k 10 200 python -u tools/bench_attn.py --no-torch > $out/attn_$m.log 2>&1 || exit 1
  echo "mode=$m"; cut -c1-300 $out/attn_$m.log
done
PDA_ATTN_BWD_FUSED=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/prof -o run -- python -u tools/bench_attn.py --no-torch --iters 5 > $out/prof.log 2>&1 || exit 1
for m in 0 1 0 1; do
  PDA_ATTN_BWD_FUSED=$m timeout -k 10 300 python -u -m pytorchdistributed_amd.bench.gpt2_ddp --steps 10 --warmup 3 > $out/g2_$m.log 2>&1 || exit 1
  echo "fused=$m $(tail -1 $out/g2_$m.log | cut -c1-160)"
done
