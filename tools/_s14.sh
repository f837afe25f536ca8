set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/s14; mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -x -q --timeout 120 --timeout-method thread -k "conv or bn or bottleneck or dgrad or resnet" > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
timeout -k 10 600 python -u tools/bench_conv.py --batch 640 --iters 10 > $out/conv_table.jsonl 2> $out/conv_table.err || { tail -5 $out/conv_table.err; exit 1; }
tail -1 $out/conv_table.jsonl
for r in 1 2; do
  for m in 1 0; do
    PDA_EPI_BST_LEAN=$m timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $out/rn_$m.log 2>&1 || exit 1
    echo "lean=$m $(tail -1 $out/rn_$m.log | cut -c1-150)"
  done
done
