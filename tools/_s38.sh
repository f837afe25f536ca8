set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/s38; mkdir -p $out
for sk in 0 3 0 3; do
  PDA_TEST_SKEW_S=$sk timeout -k 10 300 python -u -m pytest tests/test_xgmi_gpu.py -q --timeout 200 --timeout-method thread -k "fsdp_over_xgmi" > $out/t.log 2>&1; rc=$?
  echo "skew=$sk rc=$rc $(grep -E 'passed|failed' $out/t.log | tail -1) $(grep -o "AssertionError: .*" $out/t.log | head -1)"
done
