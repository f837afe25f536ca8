set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/s27; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_models_gpu.py tests/test_graphs_gpu.py tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "resnet or graph or bottleneck or conv or bn or determin" > $out/t.log 2>&1 || { tail -30 $out/t.log; exit 1; }
tail -1 $out/t.log
for r in 1 2; do
  for m in 1 0; do
    PDA_CONV_PRE_WT=$m timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $out/rn_${m}_$r.log 2>&1 || exit 1
    echo "pre_wt=$m $(tail -1 $out/rn_${m}_$r.log | cut -c100-190)"
  done
done
