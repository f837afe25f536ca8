set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/s36; mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_xgmi_gpu.py -q --timeout 200 --timeout-method thread > $out/t.log 2>&1; rc=$?
grep -E "passed|failed|AssertionError" $out/t.log | tail -5
exit $rc
