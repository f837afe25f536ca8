set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/s39; mkdir -p $out
PDA_TEST_DEBUG=1 timeout -k 10 300 python -u -m pytest tests/test_xgmi_gpu.py -q -s --timeout 200 --timeout-method thread -k "fsdp_over_xgmi" > $out/t1.log 2>&1; echo "rc=$?"
grep -E "^\[rank|^\[ref|passed|failed" $out/t1.log | cut -c1-400
PDA_TEST_DEBUG=1 timeout -k 10 300 python -u -m pytest tests/test_xgmi_gpu.py -q -s --timeout 200 --timeout-method thread -k "fsdp_over_xgmi" > $out/t2.log 2>&1; echo "rc=$?"
grep -E "^\[rank|^\[ref|passed|failed" $out/t2.log | cut -c1-400
