set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/s23; mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "conv_fwd_dgrad_wgrad" > $out/t1.log 2>&1 || { tail -30 $out/t1.log; exit 1; }
tail -1 $out/t1.log
timeout -k 10 300 python -u -m pytest tests/test_models_gpu.py -x -q --timeout 120 --timeout-method thread -k "bn_bwd_stats or bottleneck or resnet" > $out/t2.log 2>&1 || { tail -30 $out/t2.log; exit 1; }
tail -1 $out/t2.log
timeout -k 10 600 python -u tools/bench_conv.py --batch 640 --iters 10 > $out/conv_table.jsonl 2> $out/conv_table.err || { tail -5 $out/conv_table.err; exit 1; }
grep '"H": 56, "Cin": 64, "Cout": 64, "R": 3' $out/conv_table.jsonl | cut -c1-300
for r in 1 2; do
  for m in 1 0; do
    PDA_CONV_RES64=$m timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $out/rn_${m}_$r.log 2>&1 || exit 1
    echo "res64=$m $(tail -1 $out/rn_${m}_$r.log | cut -c1-150)"
  done
done
