set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/s37; mkdir -p $out
for i in 1 2 3 4 5; do
  timeout -k 10 300 python -u -m pytest tests/test_xgmi_gpu.py -q --timeout 200 --timeout-method thread -k "fsdp_over_xgmi" > $out/t$i.log 2>&1; rc=$?
  echo "run $i rc=$rc $(grep -E 'passed|failed' $out/t$i.log | tail -1) $(grep -o "AssertionError: .*" $out/t$i.log | head -1)"
done
