set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/s45; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_models_gpu.py -x -q --timeout 120 --timeout-method thread -k "conv or bn_bwd_stats or bottleneck or resnet" > $out/t.log 2>&1 || { tail -30 $out/t.log; exit 1; }
tail -1 $out/t.log
for shape in "640 56 128 128 3 2" "640 28 256 256 3 2" "640 14 512 512 3 2" "640 56 256 512 1 2"; do
  timeout -k 10 120 python -u tools/dgrad_bst_probe.py $shape > $out/p.log 2>&1 || { cat $out/p.log; exit 1; }
  grep -v amdgpu $out/p.log
done
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $out/rn_$r.log 2>&1 || exit 1
  echo "$(tail -1 $out/rn_$r.log | cut -c100-190)"
done
